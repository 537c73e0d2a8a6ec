"""The plain entry's second launch: lnx_crc32_batch (rows
kernel, then the staged kernel, which owns no slice of a uniform batch and
exits) against the rows kernel launched alone (research hook
lnx__crc32_variant 0, policy kPolicyRows), round-robin, HIP events around 20
back-to-back launches each, median of REPS; then an empty-batch-sized launch
of the staged kernel alone for its fixed cost.

usage: second_launch.py [FRAMES] [REPS]   (1500-B frames)"""
import ctypes
import os
import statistics
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth

R = L.research_lib()
R.lnx__crc32_variant.restype = ctypes.c_int
R.lnx__crc32_variant.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                                 ctypes.c_void_p]
n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 9
dev = torch.device("cuda:0")
d = synth.bytes_torch(n * 1500, dev)
o = torch.arange(n + 1, dtype=torch.int64, device=dev) * 1500
out = torch.empty(n, dtype=torch.int32, device=dev)
ref = torch.empty_like(out)
s = torch.cuda.current_stream()


def plain():
    L.crc32_batch(d, o, out=ref, stream=s)


def rows_only():
    assert R.lnx__crc32_variant(0, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), s.cuda_stream) == 0


t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    for _ in range(10):
        plain()
    torch.cuda.synchronize()
res = {"plain": [], "rows_only": []}
for r in range(reps):
    for name, fn in (("plain", plain), ("rows_only", rows_only)) if r % 2 == 0 else (("rows_only", rows_only), ("plain", plain)):
        fn()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        ev[0].record(s)
        for _ in range(20):
            fn()
        ev[1].record(s)
        torch.cuda.synchronize()
        res[name].append(ev[0].elapsed_time(ev[1]) / 20)
assert torch.equal(out, ref)
m = {k: statistics.median(v) for k, v in res.items()}
for k, v in res.items():
    print(f"{k:10s} median {m[k]:.4f} ms  ({' '.join(f'{x:.4f}' for x in v)})")
print(f"frames {n}: second launch {1e3 * (m['plain'] - m['rows_only']):.2f} us per call "
      f"({100 * (m['plain'] / m['rows_only'] - 1):.2f} %); rows alone frac {n * 1500 / m['rows_only'] / 1e6 / 8000:.4f}")
