"""Batched transmit checksum generate.

CPU: the oracle restatement of encapsulate4 / encapsulate6 / the ICMP clients'
checksum step (oracle.tx_checksum) pinned on the reference's own frames
(lneto_test.go:119-160: regenerating them from zeroed fields gives back
0xa3aa / 0xaa6a and 0x62bc / 0xde02), and generated frames pass the receive
path's verdict (oracle.ingress_verdict).  GPU: lnx_tx_checksum_batch against
the oracle byte for byte, including UDP sums that fold to 0 (NeverZeroSum)."""
import json
import os
import struct

import numpy as np
import pytest

from oracle import oracle as O
from tests import framegen as G

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _kat_frames():
    g = json.load(open(os.path.join(ROOT, "tests", "golden", "vectors.json")))
    return [(bytes.fromhex(f["frame"]), f) for f in g["lneto_tcp_frames"]]


def test_reference_frames_regenerated_from_zeroed_fields():
    for frame, kat in _kat_frames():
        b = bytearray(frame)
        b[24:26] = b"\0\0"          # IPv4 header CRC
        b[50:52] = b"\0\0"          # TCP CRC (14 + 20 + 16)
        b[16:18] = b"\0\0"          # total length: set from the frame (SetTotalLength(n + hl))
        got, st = O.tx_checksum(bytes(b))
        assert st == 0
        assert got == frame
        assert struct.unpack(">H", got[24:26])[0] == kat["ipv4_sum_want"]
        assert struct.unpack(">H", got[50:52])[0] == kat["tcp_sum_want"]


def _udp_zero_sum_frame(ipv6: bool) -> bytes:
    """A UDP datagram whose checksum computes to 0, so NeverZeroSum stores
    0xFFFF (crc.go:65-71): the last payload word is set to the checksum the
    datagram has with that word zero."""
    pay = bytearray(b"zero-sum payload" + bytes(2))
    f = G.ether(0x86DD, G.ipv6(17, G.udp(bytes(pay)), fix_l4=False)) if ipv6 else \
        G.ether(0x0800, G.ipv4(17, G.udp(bytes(pay)), fix_l4=False))
    g, _ = O.tx_checksum(f)
    at = 54 + 6 if ipv6 else 34 + 6
    c = struct.unpack(">H", g[at:at + 2])[0]
    b = bytearray(f)
    b[-2:] = struct.pack(">H", c)
    return bytes(b)


def tx_frames(seed: int = 5, count: int = 1200) -> list[bytes]:
    """Frames as the stack hands them to the checksum step: headers written,
    checksum and length fields holding stale values (random), every protocol
    the step knows plus ones it leaves alone and frames too short for it."""
    rng = np.random.default_rng(seed)

    def pay(lo=0, hi=1400):
        return rng.integers(0, 256, size=int(rng.integers(lo, hi)), dtype=np.uint8).tobytes()

    out = []
    for i in range(count):
        kind = i % 14
        if kind == 0:
            f = G.ether(0x0800, G.ipv4(6, G.tcp(pay()), fix_l4=False))
        elif kind == 1:
            f = G.ether(0x0800, G.ipv4(17, G.udp(pay()), fix_l4=False))
        elif kind == 2:  # options: the header CRC still covers 20 bytes (ipv4/frame.go:144-146)
            f = G.ether(0x0800, G.ipv4(6, G.tcp(pay()), opts=bytes(4 * int(rng.integers(1, 11))), fix_l4=False))
        elif kind == 3:
            f = G.ether(0x86DD, G.ipv6(6, G.tcp(pay()), fix_l4=False))
        elif kind == 4:
            f = G.ether(0x86DD, G.ipv6(17, G.udp(pay()), fix_l4=False))
        elif kind == 5:  # ICMPv4 echo (ipv4/icmpv4/client.go:210-214)
            f = G.ether(0x0800, G.ipv4(1, bytes([8, 0, 0, 0]) + pay(4, 600)))
        elif kind == 6:  # ICMPv6 (ipv6/icmpv6/client.go:135-148)
            f = G.ether(0x86DD, G.ipv6(58, bytes([128, 0, 0, 0]) + pay(4, 600)))
        elif kind == 7:
            f = _udp_zero_sum_frame(bool(i % 2))
        elif kind == 8:  # other protocols: header CRC (IPv4) / payload length only
            f = G.ether(int(rng.choice([0x0800, 0x86DD])), pay(40, 200))
            b = bytearray(f)
            if b[12:14] == b"\x08\x00":
                b[14] = 0x45
                b[23] = 0x2F
            else:
                b[20] = 0x2C
            f = bytes(b)
        elif kind == 9:  # transport too short for its header: untouched, ErrTruncatedFrame
            proto = int(rng.choice([6, 17, 1]))
            f = G.ether(0x0800, G.ipv4(proto, pay(0, 8 if proto != 6 else 20), fix_l4=False))
        elif kind == 10:  # too short for the IP header / bad IHL
            f = G.ether(int(rng.choice([0x0800, 0x86DD])), pay(0, 40))
            if rng.integers(0, 2) and len(f) >= 34:
                b = bytearray(f)
                b[12:14] = b"\x08\x00"
                b[14] = 0x40 | int(rng.integers(0, 5))
                f = bytes(b)
        elif kind == 11:  # other EtherTypes (ARP, VLAN): untouched
            f = G.ether(int(rng.choice([0x0806, 0x8100, 0x88CC])), pay(0, 100))
        elif kind == 12:  # odd-length transport (trailing byte weighted << 8)
            f = G.ether(0x0800, G.ipv4(int(rng.choice([6, 17])), G.tcp(pay(1, 60) + b"\x7f"), fix_l4=False))
        else:  # jumbo
            f = G.ether(0x0800, G.ipv4(6, G.tcp(pay(3000, 8900)), fix_l4=False))
        b = bytearray(f)
        # stale checksum and length fields: the step must not depend on them
        def stale(at):
            if len(b) >= at + 2:
                b[at:at + 2] = rng.integers(0, 256, 2, dtype=np.uint8).tobytes()
        if kind != 7 and len(b) >= 34 and b[12:14] == b"\x08\x00":
            la = 14 + 4 * (b[14] & 15)
            stale(16), stale(24)
            if b[23] == 6:
                stale(la + 16)
            elif b[23] == 17:
                stale(la + 4), stale(la + 6)
            elif b[23] == 1:
                stale(la + 2)
        if kind != 7 and len(b) >= 54 and b[12:14] == b"\x86\xdd":
            stale(18)
            stale({6: 70, 17: 60, 58: 56}.get(b[20], 0)) if b[20] in (6, 17, 58) else None
            if b[20] == 17:
                stale(58)
        out.append(bytes(b))
    return out


def test_generated_frames_pass_the_receive_path():
    st = {}
    for f in tx_frames(count=700):
        g, s = O.tx_checksum(f)
        st[s] = st.get(s, 0) + 1
        # (the step writes lengths and sums only; encapsulate4 itself writes
        # version 4, so frames with another version nibble are skipped)
        ip_ok = len(g) >= 15 and (g[12:14] == b"\x86\xdd" or (g[12:14] == b"\x08\x00" and g[14] >> 4 == 4))
        if s == 0 and ip_ok:
            assert O.ingress_verdict(g) == 0, g[:60].hex()
        if s != 0:
            assert g == f
    assert st.get(0, 0) > 400 and st.get(O.ERR_TRUNCATED_FRAME, 0) > 20 and st.get(O.ERR_INVALID_LENGTH_FIELD, 0) > 0


def test_never_zero_sum_applied():
    for v6 in (False, True):
        f = _udp_zero_sum_frame(v6)
        g, st = O.tx_checksum(f)
        at = 54 + 6 if v6 else 34 + 6
        assert st == 0 and g[at:at + 2] == b"\xff\xff"
        assert O.ingress_verdict(g) == 0


def _pack_slots(frames, cap, base_pad):
    n = len(frames)
    buf = np.full(base_pad + n * cap + 8, 0xA5, dtype=np.uint8)
    starts = base_pad + np.arange(n, dtype=np.int64) * cap
    for i, f in enumerate(frames):
        buf[starts[i]:starts[i] + len(f)] = np.frombuffer(f, dtype=np.uint8)
    return buf, starts, np.array([len(f) for f in frames], dtype=np.int32)


@pytest.mark.gpu
@pytest.mark.parametrize("base_pad", [0, 1, 2, 5])
def test_gpu_tx_checksum_matches_oracle(cuda, base_pad):
    import torch
    import lneto_amd as L
    frames = tx_frames(seed=50 + base_pad, count=2800)
    cap = 9100
    buf, starts, lens = _pack_slots(frames, cap, base_pad)
    d = torch.from_numpy(buf).to(cuda)
    st = L.tx_checksum_batch(d, torch.from_numpy(starts).to(cuda), torch.from_numpy(lens).to(cuda))
    got_st = st.cpu().numpy()
    host = d.cpu().numpy()
    bad = []
    for i, f in enumerate(frames):
        want, ws = O.tx_checksum(f)
        s = int(starts[i])
        g = host[s:s + len(f)].tobytes()
        if g != want or int(got_st[i]) != ws:
            bad.append((i, len(f), int(got_st[i]), ws))
    assert not bad, bad[:10]
    # the bytes between frames are untouched
    mask = np.ones(len(buf), dtype=bool)
    for i, f in enumerate(frames):
        mask[starts[i]:starts[i] + len(f)] = False
    assert np.array_equal(host[mask], buf[mask])


@pytest.mark.gpu
def test_gpu_tx_checksum_then_ingress_verify(cuda):
    """Frames generated on the device pass lnx_ingress_verify_batch with verdict 0."""
    import torch
    import lneto_amd as L
    frames = [f for f in tx_frames(seed=77, count=1400) if O.tx_checksum(f)[1] == 0
              and (f[12:14] == b"\x86\xdd" or (f[12:14] == b"\x08\x00" and f[14] >> 4 == 4))]
    buf, starts, lens = _pack_slots(frames, 9100, 3)
    d = torch.from_numpy(buf).to(cuda)
    st = L.tx_checksum_batch(d, torch.from_numpy(starts).to(cuda), torch.from_numpy(lens).to(cuda))
    assert int(st.sum()) == 0
    ends = starts + lens
    # ingress verdicts over the same slots (segment form: offsets of each frame's start and end)
    offs = np.empty(2 * len(frames), dtype=np.int64)
    offs[0::2], offs[1::2] = starts, ends
    v = L.ingress_verify_batch(d, torch.from_numpy(offs).to(cuda)).cpu().numpy()[0::2]
    assert int(v.max()) == 0, np.nonzero(v)[0][:10]
    # with the ICMP clients attached: no generated ICMP message fails its sum
    # (other ICMPv4 types than echo are dropped before the sum, as the client does)
    vi = L.ingress_verify_batch(d, torch.from_numpy(offs).to(cuda), flags=L.VERIFY_ICMP).cpu().numpy()[0::2]
    img = d.cpu().numpy()
    want = [O.ingress_verdict(img[s:e].tobytes(), O.VERIFY_ICMP) for s, e in zip(starts, ends)]
    assert vi.tolist() == want
    assert O.ERR_BAD_CRC not in want


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["tx_finish", "generate_rows"])
@pytest.mark.parametrize("base_pad", [0, 3])
def test_gpu_tx_checksum_both_routes(cuda, route, base_pad):
    """lnx_tx_checksum_batch launches the generate rows and tx_finish's checksum
    step, and the one the batch's sampled mean length picks works (api.cpp
    kTxChecksumShortMean, 896 B over 64 lengths spread across the batch): the
    generator's frames under 600 B alone (tx_finish), and after as many jumbo
    frames (the generate rows); bytes and status against the oracle, the bytes
    between the frames and the length array untouched either way."""
    import torch
    import lneto_amd as L
    rng = np.random.default_rng(70 + base_pad)
    short = [f for f in tx_frames(seed=60 + base_pad, count=3000) if len(f) < 600]
    frames = list(short)
    if route == "generate_rows":
        jumbo = []
        for _ in range(len(short)):
            b = bytearray(G.ether(0x0800, G.ipv4(int(rng.choice([6, 17])), G.tcp(
                rng.integers(0, 256, int(rng.integers(3000, 8900)), dtype=np.uint8).tobytes()), fix_l4=False)))
            b[24:26] = rng.integers(0, 256, 2, dtype=np.uint8).tobytes()  # stale header CRC
            jumbo.append(bytes(b))
        frames = jumbo + short
    n = len(frames)
    idx = [(i * n) >> 6 for i in range(64)]
    assert (sum(len(frames[i]) for i in idx) < 64 * 896) == (route == "tx_finish")
    buf, starts, lens = _pack_slots(frames, 9100, base_pad)
    d = torch.from_numpy(buf).to(cuda)
    d_len = torch.from_numpy(lens).to(cuda)
    st = L.tx_checksum_batch(d, torch.from_numpy(starts).to(cuda), d_len).cpu().numpy()
    host = d.cpu().numpy()
    assert np.array_equal(d_len.cpu().numpy(), lens)
    bad = []
    codes = set()
    for i, f in enumerate(frames):
        want, ws = O.tx_checksum(f)
        codes.add(ws)
        s = int(starts[i])
        if host[s:s + len(f)].tobytes() != want or int(st[i]) != ws:
            bad.append((i, len(f), int(st[i]), ws))
    assert not bad, bad[:10]
    assert len(codes) >= 3
    mask = np.ones(len(buf), dtype=bool)
    for i, f in enumerate(frames):
        mask[starts[i]:starts[i] + len(f)] = False
    assert np.array_equal(host[mask], buf[mask])
