"""The receive verdicts and the transmit checksums two ways on the same frames
(no FCS), by HIP events (median of 10):
  receive: the ingress kernel (lnx_ingress_verify_batch: 16-lane rows, the
  headers parsed in the row) against the receive check without its CRC
  (lnx_rx_verify_batch with LNX_RX_NO_FCS: rows for the sums, one lane per
  frame for the headers), frames packed back to back;
  transmit: lnx_tx_checksum_batch (the ingress rows, GEN) against
  lnx_tx_finish_batch with LNX_TX_CHECKSUM only, frames in 1536-byte slots;
over uniform lengths 128 .. 1500 and configs[3]'s Zipf mix (valid UDP/IPv4,
bench.py's _udp4_device); verdicts and frames compared."""
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


N = 1 << 22
sets = [(f"u{m}", np.full(N, m, np.int64)) for m in (128, 256, 384, 512, 768, 1024, 1500)]
sets.append(("zipf", synth.zipf_lengths(1 << 24)))
out = {}
for name, lens in sets:
    n = len(lens)
    off = synth.offsets_from_lengths(lens).astype(np.int64)
    d = synth.bytes_torch(int(off[-1]), dev)
    o = torch.from_numpy(off).to(dev)
    _udp4_device(L, torch, d, o[:-1].contiguous(), o[1:] - o[:-1], fcs=False)
    v1 = L.ingress_verify_batch(d, o)
    ok, v2 = L.rx_verify_batch(d, o, flags=L.RX_NO_FCS)
    assert torch.equal(v1.cpu(), v2.cpu()) and int((v1 == 0).sum()) == n, name
    r = {"mean": float(lens.mean()), "ingress_ms": t(lambda: L.ingress_verify_batch(d, o)),
         "rx_verify_no_fcs_ms": t(lambda: L.rx_verify_batch(d, o, flags=L.RX_NO_FCS))}
    del d, o
    ds = synth.bytes_torch(n * 1536, dev)
    st = torch.arange(n, dtype=torch.int64, device=dev) * 1536
    ln = torch.from_numpy(lens).to(dev)
    _udp4_device(L, torch, ds, st, ln, fcs=False)
    l32 = ln.to(torch.int32)
    s1 = L.tx_checksum_batch(ds, st, l32)
    ref = ds.clone()
    s2 = L.tx_finish_batch(ds, st, l32, 1536, flags=L.TX_CHECKSUM)
    s2 = s2[0] if isinstance(s2, tuple) else s2
    assert torch.equal(ref, ds) and int((s1 == 0).sum()) == n, name
    r["tx_checksum_ms"] = t(lambda: L.tx_checksum_batch(ds, st, l32))
    r["tx_finish_ck_ms"] = t(lambda: L.tx_finish_batch(ds, st, l32, 1536, flags=L.TX_CHECKSUM))
    del ds, st, ln, l32, ref
    out[name] = r
    print(name, json.dumps(r), flush=True)
print(json.dumps(out))
