"""Staged lane streams (variants 300 / 302): print the wrong frames of one
Zipf batch with their block position (lane of start / end, the block's Q)
and what the kernel returned against the oracle and against a few corrupted
forms (tail piece zeroed), to classify a parity failure.
usage: stage_dbg.py [var] [n] [seed]"""
import ctypes
import os
import sys
import zlib

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch

import lneto_amd as L
from lneto_amd import synth

var = int(sys.argv[1]) if len(sys.argv) > 1 else 300
n = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 16
seed = int(sys.argv[3]) if len(sys.argv) > 3 else 11
f = L.research_lib().lnx__crc32_variant
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
off = synth.offsets_from_lengths(synth.zipf_lengths(n, seed=seed)).astype(np.int64)
data = synth.bytes_np(int(off[-1]) + 8, seed=seed)
dev = torch.device("cuda:0")
d = torch.from_numpy(data).to(dev)
o = torch.from_numpy(off).to(dev)
out = torch.full((n,), -1, dtype=torch.int32, device=dev)
assert f(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
torch.cuda.synchronize()
got = out.cpu().numpy().view(np.uint32)
print("base ptr mod 128:", d.data_ptr() % 128)
bad = 0
BF = 382
per = -(-n // min(256, -(-n // BF)))
for i in range(n):
    s, e = int(off[i]), int(off[i + 1])
    want = zlib.crc32(data[s:e].tobytes())
    if got[i] == want:
        continue
    bad += 1
    if bad > 40:
        continue
    fb0 = (i // per) * per
    f0 = fb0 + ((i - fb0) // BF) * BF
    A, E = int(off[f0]), int(off[min(f0 + BF, n, fb0 + per)])
    adj = (d.data_ptr() + A) & 127
    sp = E - A + adj
    Q = max(128, ((sp + 63) // 64 + 127) & ~127)
    rs, re = s - A + adj, e - A + adj
    forms = {}
    for z in (1, 2, 3, 4, 8, 16):
        buf = bytearray(data[s:e].tobytes())
        for k in range(max(0, len(buf) - z), len(buf)):
            buf[k] = 0
        forms[f"tail{z}=0"] = zlib.crc32(bytes(buf))
    hit = [k for k, v in forms.items() if v == got[i]]
    other = np.nonzero(got == got[i])[0]
    print(f"frame {i} (block {f0}, +{i - f0}) len {e - s} rel [{rs},{re}) Q {Q} sp {sp} lanes {rs // Q}->{re // Q} "
          f"(+{rs % Q},+{re % Q}) got {got[i]:08x} want {want:08x} matches {hit} same-value frames {other[:4]}")
print("bad", bad, "of", n)
