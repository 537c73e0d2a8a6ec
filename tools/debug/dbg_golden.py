import sys, json
sys.path.insert(0, '.'); sys.path.insert(0, 'tests')
import numpy as np, torch
import lneto_amd as L
from oracle import oracle as O
from test_gpu_parity import _pack, _crc_gpu
cuda = torch.device('cuda:0')
g = json.load(open('tests/golden/vectors.json'))
frames = [bytes.fromhex(v["data"]) for v in g["crc32_vectors"]]
data, off = _pack(frames)
got = _crc_gpu(cuda, data, off)
want = O.crc32_frames(data, off)
n = len(frames)
bad = np.nonzero(got != want)[0]
print("n", n, "bad", bad.tolist())
waves = ((n + 63)//64) * 16
fpw = (n + waves - 1)//waves
print("fpw", fpw)
for i in bad[:20]:
    w = i // fpw; fw0 = w*fpw
    print(i, "len", len(frames[i]), "off", int(off[i]), int(off[i+1]), "e%4", int(off[i+1]) % 4, "wave", w, "row", i - fw0, "o0", int(off[fw0]))
# same frames, one per batch
for i in bad[:6]:
    d2, o2 = _pack([frames[i]], base_pad=int(off[i]) % 4)
    print("alone", i, int(_crc_gpu(cuda, d2, o2)[0]) == O.crc32(frames[i]))
