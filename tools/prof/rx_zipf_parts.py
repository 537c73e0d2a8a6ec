"""Where lnx_rx_verify_batch spends its time on the Zipf mix (configs[3]'s
16 M frames, valid UDP/IPv4 with their FCS, bench.py's _udp4_device): the
receive check with and without the CRC (LNX_RX_NO_FCS: sums and verdicts
only), the FCS verify alone (rows / staged kernels), the verdicts alone
(ingress kernel on the frames without FCS), by HIP events (median of 10)."""
import json
import os
import sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth
from bench import _udp4_device

dev = torch.device("cuda:0")
n = 1 << 24
off = synth.offsets_from_lengths(synth.zipf_lengths(n)).astype(np.int64)
d = synth.bytes_torch(int(off[-1]), dev)
o = torch.from_numpy(off).to(dev)
_udp4_device(L, torch, d, o[:-1].contiguous(), o[1:] - o[:-1], fcs=True)
o2 = torch.stack([o[:-1], o[1:] - 4], 1).reshape(-1).contiguous()  # frames without FCS, FCS as frames between


def t(fn, reps=10):
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    return round(float(np.median(ts)), 4)


ok, v = L.rx_verify_batch(d, o)
assert int(ok.sum()) == n and int(v.sum()) == 0
out = {
    "rx_verify_ms": t(lambda: L.rx_verify_batch(d, o)),
    "rx_verify_no_fcs_ms": t(lambda: L.rx_verify_batch(d, o, flags=L.RX_NO_FCS)),
    "fcs_verify_plain_ms": t(lambda: L.fcs_verify_batch(d, o)),
    "fcs_verify_short_ms": t(lambda: L.fcs_verify_batch(d, o, short_frames=True)),
    "ingress_2n_ms": t(lambda: L.ingress_verify_batch(d, o2)),
}
print(json.dumps(out))
