"""Time the CRC kernel's profiling variants on the 1M x 1500 B batch.
0 = product kernel, 1 = loads + bookkeeping only, 2 = lookups + bookkeeping only."""
import ctypes
import sys
import os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth

L.lib.lnx__crc32_variant.restype = ctypes.c_int
L.lib.lnx__crc32_variant.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_void_p]
wl = sys.argv[1] if len(sys.argv) > 1 else "mtu1500"
dev = torch.device("cuda:0")
off = synth.workload_offsets(wl)
n = len(off) - 1
d = synth.bytes_torch(int(off[-1]), dev)
o = torch.from_numpy(off.astype(np.int64)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
vars_ = [int(v) for v in sys.argv[2].split(",")] if len(sys.argv) > 2 else [0, 1, 2, 0]
NOT_CRC = {1, 2, 26, 27}  # timing-only variants (loads only / math only)
ref = torch.empty_like(out)
L.crc32_batch(d, o, out=ref)
torch.cuda.synchronize()
print(f"lib {L.LIB_PATH}")
for var in vars_:
    for _ in range(3):
        L.lib.lnx__crc32_variant(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), s.cuda_stream)
    torch.cuda.synchronize()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record(s)
    for _ in range(20):
        L.lib.lnx__crc32_variant(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), s.cuda_stream)
    ev[1].record(s)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / 20
    ok = "" if var in NOT_CRC else ("  crc ok" if torch.equal(out, ref) else "  CRC MISMATCH")
    print(f"{wl} variant {var}: {ms:.4f} ms  {off[-1] / ms / 1e6:.1f} GB/s{ok}")
