import sys, struct
sys.path.insert(0, '.')
import numpy as np, torch
import lneto_amd as L
from oracle import oracle as O
sys.path.insert(0, 'tests')
from test_gpu_parity import _pack, _dev
cuda = torch.device('cuda:0')
rng = np.random.default_rng(11)
frames, want = [], []
for i in range(600):
    n = int(rng.integers(0, 1600))
    payload = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
    f = payload + struct.pack("<I", O.crc32(payload))
    kind = i % 4
    if kind == 1 and n > 0:
        b = bytearray(f); b[int(rng.integers(0, n))] ^= 0x01; f = bytes(b)
    elif kind == 2:
        b = bytearray(f); b[-1] ^= 0x80; f = bytes(b)
    elif kind == 3:
        f = f[: int(rng.integers(0, 4))]
    frames.append(f)
    ok = len(f) >= 4 and O.crc32(f[:-4]) == struct.unpack("<I", f[-4:])[0]
    want.append(1 if ok else 0)
data, off = _pack(frames, gaps=rng.integers(0, 4, size=len(frames)))
d, o = _dev(cuda, data, off)
got = L.fcs_verify_batch(d, o).cpu().numpy()
crc = L.crc32_batch(d, o).cpu().numpy().view(np.uint32)
ref = O.crc32_frames(data, off)
print("crc mismatches", np.nonzero(crc != ref)[0][:20])
bad = np.nonzero(got != np.array(want))[0]
print("verify mismatches", len(bad), bad[:40])
for i in bad[:10]:
    print(i, len(frames[i]), int(off[i]), int(off[i+1]), hex(int(crc[i])), hex(int(ref[i])), got[i], want[i])
