"""First-touch check of the sum16 kernel variants on freshly copied data (GPU
debug aid): each trial copies the blob into a new device tensor and runs one
variant on it once.  usage: dbg_sum16.py"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import lneto_amd as L
from lneto_amd import synth
from oracle import oracle as O
L.research_lib().lnx__sum16_variant.restype = ctypes.c_int
L.research_lib().lnx__sum16_variant.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_uint64] + [ctypes.c_void_p] * 2
cuda = torch.device("cuda:0")
rng = np.random.default_rng(21)
n = 5000
blob = synth.bytes_np(1 << 22, seed=77)
lens = rng.integers(0, 1600, size=n).astype(np.uint32)
starts = rng.integers(0, len(blob) - 10000, size=n).astype(np.uint64)
seeds = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
want = O.sum16_segments(blob, starts, lens, seeds)
o = torch.from_numpy(starts.astype(np.int64)).to(cuda)
ln = torch.from_numpy(lens.view(np.int32)).to(cuda)
sd = torch.from_numpy(seeds.view(np.int32)).to(cuda)
junk = []
modes = ["plain", "sync", "touch", "plain"]
for trial in range(16):
    var = (0, 2, 1, 0)[trial % 4]
    mode = modes[(trial // 4) % 4]
    junk.append(torch.randint(0, 255, (1 << 22,), dtype=torch.uint8, device=cuda))
    if len(junk) > 2:
        junk.pop(0)
    d = torch.from_numpy(blob).to(cuda)
    if mode == "sync":
        torch.cuda.synchronize()
    if mode == "touch":
        _ = int(d.sum())
    out = torch.full((n,), 0x5A5A, dtype=torch.int16, device=cuda)
    rc = L.research_lib().lnx__sum16_variant(var, d.data_ptr(), o.data_ptr(), ln.data_ptr(), sd.data_ptr(), n, out.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint16)
    bad = np.nonzero(got != want)[0]
    sentinel = int((got[bad] == 0x5A5A).sum())
    again = np.zeros(0)
    if bad.size:
        rc = L.research_lib().lnx__sum16_variant(var, d.data_ptr(), o.data_ptr(), ln.data_ptr(), sd.data_ptr(), n,
                                      out.data_ptr(), torch.cuda.current_stream().cuda_stream)
        torch.cuda.synchronize()
        again = np.nonzero(out.cpu().numpy().view(np.uint16) != want)[0]
    print(f"trial {trial} var {var} {mode}: bad {bad.size} (unwritten {sentinel}) {bad[:6]} relaunch bad {again.size}",
          flush=True)
    del d
