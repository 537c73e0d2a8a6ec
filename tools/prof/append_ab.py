"""A/B of the TX FCS append variants (lnx__fcs_append_variant: 0 / 100 = the product, one launch,
200 = two launches (CRC kernel into a compact scratch, then a scatter kernel),
results held and flushed; 4 = FCS / length / status stored as each frame
finishes; 7 = the FCS written with its whole 64-byte sector; -1 = no append: lnx_crc32_segments
over the same frames, the body's cost alone) on bench.py's fcs_append workload: 1 M frames of 1496 B in 1536-B
slots, lengths reset before every launch.  Round-robin, median of REPS.

usage: append_ab.py [VARS (e.g. 0+4)] [REPS]"""
import ctypes
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth

L.research_lib().lnx__fcs_append_variant.restype = ctypes.c_int
L.research_lib().lnx__fcs_append_variant.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_void_p]
vars_ = [int(v) for v in (sys.argv[1] if len(sys.argv) > 1 else "0+4").replace(",", "+").replace("m", "-").split("+")]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 9
dev = torch.device("cuda:0")
n, flen, cap = 1 << 20, 1496, 1536
d0 = synth.bytes_torch(n * cap, dev)
start = torch.arange(n, dtype=torch.int64, device=dev) * cap
len0 = torch.full((n,), flen, dtype=torch.int32, device=dev)
ln = len0.clone()
st = torch.empty(n, dtype=torch.uint8, device=dev)
crc = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
d = d0.clone()


def launch(var):
    ln.copy_(len0)
    if var < 0:
        assert L.lib.lnx_crc32_segments(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(start.data_ptr()),
                                        ctypes.c_void_p(ln.data_ptr()), ctypes.c_uint64(n),
                                        ctypes.c_void_p(crc.data_ptr()), ctypes.c_void_p(s.cuda_stream)) == 0
        return
    assert L.research_lib().lnx__fcs_append_variant(var, d.data_ptr(), start.data_ptr(), ln.data_ptr(), n, cap, st.data_ptr(),
                                         s.cuda_stream) == 0


outs = {}
for var in [v for v in vars_ if v >= 0]:
    d.copy_(d0)
    launch(var)
    torch.cuda.synchronize()
    outs[var] = (d.clone(), ln.clone(), st.clone())
v0 = next(iter(outs))
same = all(torch.equal(outs[v][i], outs[v0][i]) for v in outs for i in range(3))
print("variants agree:", same, "| lengths", int(outs[v0][1].min()), int(outs[v0][1].max()))
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    for _ in range(10):
        launch(0)
    torch.cuda.synchronize()
res = {v: [] for v in vars_}
for r in range(reps):
    for var in vars_:
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(s)
        for _ in range(20):
            launch(var)
        ev[1].record(s)
        torch.cuda.synchronize()
        res[var].append(ev[0].elapsed_time(ev[1]) / 20)
for var in vars_:
    ms = float(np.median(res[var]))
    print(f"fcs_append variant {var}: {ms:.4f} ms per launch (incl. 4 B/frame length reset), "
          f"{n * flen / ms / 1e6:.1f} GB/s  [{' '.join(f'{x:.4f}' for x in res[var])}]", flush=True)
