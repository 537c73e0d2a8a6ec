"""Time the sum16 kernel variants (sum16_kernel.hip launch_sum16_segments: 0 = line rows with default-policy
edge lines, 1 = r1c half-line rows, 2 = line rows default policy, 5 = line rows all nt) on 1 M x 1500-B
segments, round-robin medians; each variant's sums are checked against variant 1's.
usage: sum16_variants.py [REPS] [V1,V2,...]"""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import lneto_amd as L
from lneto_amd import synth
L.research_lib().lnx__sum16_variant.restype = ctypes.c_int
L.research_lib().lnx__sum16_variant.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_uint64] + [ctypes.c_void_p] * 2
dev = torch.device("cuda:0")
off = synth.workload_offsets("mtu1500")
n = len(off) - 1
d = synth.bytes_torch(int(off[-1]), dev)
o = torch.from_numpy(off[:-1].astype(np.int64)).to(dev)
ln = torch.from_numpy(np.diff(off).astype(np.int32)).to(dev)
out = torch.empty(n, dtype=torch.int16, device=dev)
s = torch.cuda.current_stream()
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 5
launch = lambda v: L.research_lib().lnx__sum16_variant(v, d.data_ptr(), o.data_ptr(), ln.data_ptr(), None, n, out.data_ptr(), s.cuda_stream)
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    launch(0)
torch.cuda.synchronize()
vs = [int(x) for x in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 3, 4, 5]
launch(1)
ref = out.clone()
ok = {}
res = {v: [] for v in vs}
for r in range(reps):
    for v in vs:
        e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        e[0].record(s)
        for _ in range(20):
            launch(v)
        e[1].record(s)
        torch.cuda.synchronize()
        res[v].append(e[0].elapsed_time(e[1]) / 20)
        ok[v] = ok.get(v, True) and torch.equal(out, ref)
for v in vs:
    ms = float(np.median(res[v]))
    tag = "sums ok" if ok[v] else "SUM MISMATCH"
    print(f"sum16 variant {v}: {ms:.4f} ms  {off[-1] / ms / 1e6:.1f} GB/s  {tag}  [{' '.join(f'{x:.4f}' for x in res[v])}]")
