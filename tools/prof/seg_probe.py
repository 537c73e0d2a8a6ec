"""Segment-mode CRC (lnx_crc32_segments) against offsets mode (lnx_crc32_batch) on
1 M frames: slot layouts (1496 or 1500 B in 1536-B slots) and packed frames,
HIP-event timed on the launch stream.  Not part of the product."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import lneto_amd as L  # noqa: E402
from lneto_amd import synth  # noqa: E402

dev = torch.device("cuda:0")
n = 1 << 20


def timeit(fn, reps=50):
    for _ in range(20):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps


for stride, flen in [(1536, 1496), (1536, 1500), (1500, 1500), (1496, 1496), (1600, 1500)]:
    d = synth.bytes_torch(n * stride + 64, dev)
    st = torch.arange(n, dtype=torch.int64, device=dev) * stride
    ln = torch.full((n,), flen, dtype=torch.int32, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    ms = timeit(lambda: L.crc32_segments(d, st, ln, out=out))
    line = f"segments stride {stride} len {flen}: {ms:.4f} ms, {n * flen / ms / 1e9:.2f} TB/s of frame bytes"
    if stride == flen:
        off = torch.arange(n + 1, dtype=torch.int64, device=dev) * stride
        ms2 = timeit(lambda: L.crc32_batch(d, off, out=out))
        line += f"; offsets mode {ms2:.4f} ms"
    print(line, flush=True)
    del d
