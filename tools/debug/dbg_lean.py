"""Which frames does a forced CRC variant get wrong on a workload? (GPU debug aid)
usage: dbg_lean.py WORKLOAD VAR"""
import ctypes, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np, torch
import lneto_amd as L
from lneto_amd import synth
from oracle import oracle as O
L.research_lib().lnx__crc32_variant.restype = ctypes.c_int
L.research_lib().lnx__crc32_variant.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_void_p]
wl, var = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda:0")
off = synth.workload_offsets(wl)
n = len(off) - 1
d = synth.bytes_torch(int(off[-1]), dev)
o = torch.from_numpy(off.astype(np.int64)).to(dev)
ref = L.crc32_batch(d, o).cpu().numpy().view(np.uint32)
for rep in range(3):
    out = torch.zeros(n, dtype=torch.int32, device=dev)
    assert L.research_lib().lnx__crc32_variant(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(),
                                    torch.cuda.current_stream().cuda_stream) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    bad = np.nonzero(got != ref)[0]
    print(f"rep {rep}: {bad.size} wrong of {n}; first {bad[:12]}")
    if bad.size:
        print("  row (f%4):", np.bincount(bad % 4, minlength=4), " got==0:", int((got[bad] == 0).sum()))
        s = off[bad]
        print("  start%128 of first:", (s[:12] % 128).tolist(), " len:", np.diff(off)[bad[:12]].tolist())
# the frame's own data, checked on the CPU for the first few
data = d[: int(off[min(n, 64)])].cpu().numpy()
print("oracle agrees with product on first 64:", np.array_equal(O.crc32_frames(data, off[:65]), ref[:64]))
