"""Debug: does a flipped byte change the giant-frame CRC?  (test_gpu_giant_frame)"""
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth
from oracle import oracle as O

cuda = torch.device("cuda:0")
giant = 2_200_000_000
d = synth.bytes_torch(giant + 64, cuda, seed=92)
o = torch.tensor([8, 8 + giant], dtype=torch.int64, device=cuda)


def crc():
    return int(L.crc32_batch(d, o).cpu().numpy().view(np.uint32)[0])


def small(i):
    so = torch.tensor([i - 40, i + 24], dtype=torch.int64, device=cuda)
    return int(L.crc32_batch(d, so).cpu().numpy().view(np.uint32)[0])


base = crc()
print("base", hex(base), flush=True)
for pos in (8 + 47, 8 + 16384 * 3 + 100, 8 + 16384 * 5000 + 8191, 8 + giant // 2 + 7, 8 + giant - 100):
    s0 = small(pos)
    d[pos] ^= 1
    torch.cuda.synchronize()
    s1 = small(pos)
    c1 = crc()
    d2 = d.clone()
    c2 = int(L.crc32_batch(d2, o).cpu().numpy().view(np.uint32)[0])
    del d2
    d[pos] ^= 1
    torch.cuda.synchronize()
    c3 = crc()
    print(f"pos {pos}: small {s0:#x}->{s1:#x}  giant {base:#x}->{c1:#x} clone {c2:#x} restored {c3:#x}", flush=True)
