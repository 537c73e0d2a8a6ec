"""launch one staged-kernel research form
on the 16 M-frame Zipf batch (configs[3]) 20 times after a warm-up, for a
rocprofv3 pass that reads GRBM_GUI_ACTIVE (the GPU clock's cycles) beside the
kernel trace.  314 = the product form, 340 = its loads alone, 342 = loads +
the LDS transpose (timing-only forms).

usage: zipf_diag.py VARIANT"""
import ctypes
import os
import sys
import time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth

var = int(sys.argv[1])
f = L.research_lib().lnx__crc32_variant
f.restype = ctypes.c_int
f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
dev = torch.device("cuda:0")
off = synth.workload_offsets("zipf64_1500")
n = len(off) - 1
d = synth.bytes_torch(int(off[-1]), dev)
o = torch.from_numpy(off.astype(np.int64)).to(dev)
out = torch.empty(n, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream()
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.5:
    assert f(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), s.cuda_stream) == 0
    torch.cuda.synchronize()
for _ in range(20):
    assert f(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), s.cuda_stream) == 0
torch.cuda.synchronize()
print(f"variant {var} done", flush=True)
