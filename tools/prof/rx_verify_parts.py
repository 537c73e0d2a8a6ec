"""Time rx_verify_batch on 1 M x 1500-B frames with and without the CRC
(LNX_RX_NO_FCS: sums and verdicts only), and the FCS-verify and ingress
kernels alone, by HIP events (median of 20)."""
import json
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth

dev = torch.device("cuda:0")
n, flen = 1 << 20, 1500
d = synth.bytes_torch(n * flen, dev)
o = torch.arange(n + 1, dtype=torch.int64, device=dev) * flen
o2 = torch.stack([o[:-1], o[1:] - 4], 1).reshape(-1).contiguous()


def t(fn, reps=20):
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
    return float(np.median(ts))


out = {
    "rx_verify_ms": t(lambda: L.rx_verify_batch(d, o)),
    "rx_verify_no_fcs_ms": t(lambda: L.rx_verify_batch(d, o, flags=L.RX_NO_FCS)),
    "fcs_verify_ms": t(lambda: L.fcs_verify_batch(d, o)),
    "ingress_ms": t(lambda: L.ingress_verify_batch(d, o2)),
}
print(json.dumps(out))
