"""Time lnx_tx_finish_batch on 1 M x 1496-B UDP/IPv4 frames in 1536-B slots
(bench.py --op tx_finish) by flags (3: checksum + FCS, 2: FCS only, 1:
checksum only), the two-call sequence, and rx_verify_batch on random bytes
packed and on bench.py --op rx_verify's frames, by HIP events (median of 20; the length restore timed alone too)."""
import json
import numpy as np
import torch
import lneto_amd as L
from lneto_amd import synth

dev = torch.device("cuda:0")
n, flen, cap = 1 << 20, 1500, 1536
d = synth.bytes_torch(n * cap, dev)
fr = d.view(n, cap)
hdr = bytes.fromhex("c0ffee00dead4e8b3af9fb6b0800") + bytes([0x45, 0]) + (flen - 18).to_bytes(2, "big") \
    + bytes.fromhex("1234400040110000c0a80a01c0a80a02") + bytes.fromhex("14e90035") + (flen - 38).to_bytes(2, "big")
fr[:, : len(hdr)] = torch.tensor(list(hdr), dtype=torch.uint8, device=dev)
ds = torch.arange(n, dtype=torch.int64, device=dev) * cap
l0 = torch.full((n,), flen - 4, dtype=torch.int32, device=dev)
dl = l0.clone()
st = torch.empty(n, dtype=torch.uint8, device=dev)
p = synth.bytes_torch(n * flen, dev)
o = torch.arange(n + 1, dtype=torch.int64, device=dev) * flen
ph = synth.bytes_torch(n * flen, dev)  # the same with bench.py --op rx_verify's UDP/IPv4 headers
hdr2 = bytes.fromhex("c0ffee00dead4e8b3af9fb6b0800") + bytes([0x45, 0]) + (flen - 14).to_bytes(2, "big") \
    + bytes.fromhex("1234400040110000c0a80a01c0a80a02") + bytes.fromhex("14e90035") + (flen - 34).to_bytes(2, "big")
ph.view(n, flen)[:, : len(hdr2)] = torch.tensor(list(hdr2), dtype=torch.uint8, device=dev)


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


def fin(flags):
    def f():
        dl.copy_(l0)
        L.tx_finish_batch(d, ds, dl, cap, flags=flags, status=st)
    return f


def two():
    dl.copy_(l0)
    L.tx_checksum_batch(d, ds, dl, status=st)
    L.fcs_append_batch(d, ds, dl, cap, status=st)


out = {
    "restore_ms": t(lambda: dl.copy_(l0)),
    "tx_finish_3_ms": t(fin(3)),
    "tx_finish_2_ms": t(fin(2)),
    "tx_finish_1_ms": t(fin(1)),
    "two_calls_ms": t(two),
    "rx_verify_packed_ms": t(lambda: L.rx_verify_batch(p, o)),
    "rx_verify_headers_ms": t(lambda: L.rx_verify_batch(ph, o)),
    "rx_verify_packed_no_fcs_ms": t(lambda: L.rx_verify_batch(p, o, flags=L.RX_NO_FCS)),
}
print(json.dumps(out))
