"""Per-wave timeline of one CRC kernel launch (entry, LDS image copied, exit;
100 MHz s_memrealtime) through the lnx__crc32_timeline profiling hook.

usage: timeline.py WORKLOAD [VARIANT ...]
Prints, per variant: dispatch skew, image-copy time, and the distribution of
wave end times (tail = how long the last waves run after most have finished),
overall and per XCD (blockIdx % 8, round-robin placement)."""
import ctypes
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

import lneto_amd as L
from lneto_amd import synth

f = L.research_lib().lnx__crc32_timeline
f.restype = ctypes.c_int64
f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
              ctypes.c_void_p]

wl = sys.argv[1] if len(sys.argv) > 1 else "mtu1500"
variants = [int(v) for v in sys.argv[2:]] or [0]
dev = torch.device("cuda:0")
off = synth.workload_offsets(wl)
n = len(off) - 1
d = synth.bytes_torch(int(off[-1]), dev)
o = torch.from_numpy(off.astype(np.int64)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
waves = int(f(0, 0, 0, n, 0, None, None))
tl = torch.zeros(3 * waves, dtype=torch.int64, device=dev)
for var in variants:
    for _ in range(3):  # warm (and keep the last launch's timeline)
        assert f(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), tl.data_ptr(), s.cuda_stream) == 0
    torch.cuda.synchronize()
    t = tl.cpu().numpy().reshape(waves, 3).astype(np.float64) * 10.0  # ns
    live = t[:, 2] > 0
    t0 = t[:, 0].min()
    start, copied, end = t[:, 0] - t0, t[:, 1] - t0, t[:, 2] - t0
    span = end[live].max()
    q = lambda a, p: float(np.percentile(a, p)) / 1e3  # noqa: E731
    print(f"{wl} variant {var}: waves {waves} span {span / 1e3:.1f} us  ({off[-1] / span:.1f} GB/s over the span)")
    print(f"  entry skew   p50 {q(start, 50):.2f}  p99 {q(start, 99):.2f}  max {start.max() / 1e3:.2f} us")
    print(f"  image copied p50 {q(copied - start, 50):.2f}  max {(copied - start).max() / 1e3:.2f} us after entry")
    e = end[live]
    print(f"  wave end     p1 {q(e, 1):.1f}  p10 {q(e, 10):.1f}  p50 {q(e, 50):.1f}  p90 {q(e, 90):.1f}  "
          f"p99 {q(e, 99):.1f}  max {e.max() / 1e3:.1f} us")
    blk = np.arange(waves) // 16
    nb = waves // 16
    bmax = np.array([end[b * 16:(b + 1) * 16].max() for b in range(nb)])
    bmin = np.array([end[b * 16:(b + 1) * 16][live[b * 16:(b + 1) * 16]].min() for b in range(nb)])
    print(f"  per CU: last wave p1 {q(bmax, 1):.1f}  p50 {q(bmax, 50):.1f}  max {bmax.max() / 1e3:.1f} us;"
          f"  first wave p50 {q(bmin, 50):.1f}; in-CU spread p50 {q(bmax - bmin, 50):.1f} us")
    for x in range(8):
        m = live & (blk % 8 == x)
        print(f"    xcd {x}: end p10 {q(end[m], 10):.1f}  p50 {q(end[m], 50):.1f}  max {end[m].max() / 1e3:.1f} us")
