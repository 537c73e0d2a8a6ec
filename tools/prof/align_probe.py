"""Probe: does the absolute alignment of each row's 64-byte load step matter?
Times lnx_crc32_batch on ~1.5 GB batches of fixed-length frames whose lengths
put the window ends at different alignments (1536 B: every step 64-B aligned)."""
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth

dev = torch.device("cuda:0")
total = 1536 << 20
lens = [int(a) for a in sys.argv[1].split(",")] if len(sys.argv) > 1 else [1500, 1536, 1472, 1504, 1528, 1024, 2048]
d = synth.bytes_torch(total + 4096, dev)
s = torch.cuda.current_stream()
for fl in lens:
    n = total // fl
    off = synth.fixed_offsets(n, fl)
    o = torch.from_numpy(off.astype(np.int64)).to(dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    for _ in range(3):
        L.crc32_batch(d, o, out=out, stream=s)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    torch.cuda.synchronize()
    ev[0].record(s)
    for _ in range(20):
        L.crc32_batch(d, o, out=out, stream=s)
    ev[1].record(s)
    torch.cuda.synchronize()
    ms = ev[0].elapsed_time(ev[1]) / 20
    print(f"frame {fl:5d} B x {n}: {ms:.4f} ms  {n * fl / ms / 1e6:.1f} GB/s", flush=True)
