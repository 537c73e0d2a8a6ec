"""Time the CRC kernel's profiling variants on one workload.
0 = product kernel, 1 = loads + bookkeeping only, 2 = lookups + bookkeeping only
(other numbers: crc32_kernel.hip launch_rows).  The GPU is warmed for ~0.5 s
first (the first few hundred microseconds of launches run at lower clocks),
then the variants are timed round-robin REPS times and the median is printed,
so box drift hits every variant alike.

usage: variants.py WORKLOAD V1,V2,... [REPS]"""
import ctypes
import sys
import os
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth

L.research_lib().lnx__crc32_variant.restype = ctypes.c_int
L.research_lib().lnx__crc32_variant.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_void_p]
wl = sys.argv[1] if len(sys.argv) > 1 else "mtu1500"
dev = torch.device("cuda:0")
off = synth.workload_offsets(wl)
n = len(off) - 1
d = synth.bytes_torch(int(off[-1]), dev)
o = torch.from_numpy(off.astype(np.int64)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
vars_ = [int(v) for v in sys.argv[2].replace("+", ",").split(",")] if len(sys.argv) > 2 else [0, 1, 2]
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 5
NOT_CRC = {1, 2, 26, 27, 32, 34, 38, 53, 54, 58, 71, 72, 91, 135, 136, 151, 152, 154, 155, 161, 162, 328, 330, 332, 334, 340, 342}  # timing-only variants (loads only / math only)
ref = torch.empty_like(out)
L.crc32_batch(d, o, out=ref)
torch.cuda.synchronize()
print(f"lib {L.LIB_PATH}")


def launch(var):
    assert L.research_lib().lnx__crc32_variant(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), s.cuda_stream) == 0


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    for _ in range(20):
        launch(0)
    torch.cuda.synchronize()
res = {v: [] for v in vars_}
ok = {}
for r in range(reps):
    for var in vars_:
        launch(var)
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(s)
        for _ in range(20):
            launch(var)
        ev[1].record(s)
        torch.cuda.synchronize()
        res[var].append(ev[0].elapsed_time(ev[1]) / 20)
        if var not in NOT_CRC:
            ok[var] = ok.get(var, True) and torch.equal(out, ref)
for var in vars_:
    ms = float(np.median(res[var]))
    tag = "" if var in NOT_CRC else ("  crc ok" if ok[var] else "  CRC MISMATCH")
    spread = " ".join(f"{x:.4f}" for x in res[var])
    print(f"{wl} variant {var}: {ms:.4f} ms  {off[-1] / ms / 1e6:.1f} GB/s{tag}   [{spread}]", flush=True)
