"""Receive-path checksum verdicts: the oracle restatement
of StackEthernet.Demux -> demux4 / demux6 pinned on the reference's own frames
and its documented quirks (CPU), and the fused HIP kernel
lnx_ingress_verify_batch against it (GPU)."""
import collections
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
    return [bytes.fromhex(f["frame"]) for f in g["lneto_tcp_frames"]]


def test_reference_tcp_frames_pass():
    """lneto_test.go:119-160 frames carry valid IPv4 and TCP checksums."""
    for f in _kat_frames():
        assert O.ingress_verdict(f) == 0


def test_reference_tcp_frames_corrupted():
    for f in _kat_frames():
        for i in (15, 24, 26, 40, 50, 73):  # ToS, header CRC, src addr, TCP seq, TCP CRC, options
            b = bytearray(f)
            b[i] ^= 0x01
            assert O.ingress_verdict(bytes(b)) == O.ERR_BAD_CRC, i


def test_validation_order_and_codes():
    ok4 = G.ether(0x0800, G.ipv4(6, G.tcp(b"hello")))
    assert O.ingress_verdict(ok4) == 0
    assert O.ingress_verdict(ok4[:13]) == O.ERR_TRUNCATED_FRAME            # ethernet.NewFrame
    assert O.ingress_verdict(G.ether(1000, b"x" * 10)) == O.ERR_INVALID_LENGTH_FIELD  # size field > frame
    assert O.ingress_verdict(G.ether(46, b"x" * 60)) == 0                  # size-type frame: no IP
    assert O.ingress_verdict(G.ether(0x8100, b"ab")) == O.ERR_TRUNCATED_FRAME
    assert O.ingress_verdict(ok4[:14 + 19]) == O.ERR_TRUNCATED_FRAME       # ipv4.NewFrame
    b = bytearray(ok4); b[16:18] = struct.pack(">H", 19)
    assert O.ingress_verdict(bytes(b)) == O.ERR_INVALID_LENGTH_FIELD       # tl < 20 (first error)
    assert O.ingress_verdict(ok4[:-1]) == O.ERR_TRUNCATED_FRAME            # tl > len
    b = bytearray(ok4); b[14] = 0x44
    assert O.ingress_verdict(bytes(b)) == O.ERR_INVALID_LENGTH_FIELD       # ihl < 5
    b = bytearray(ok4); b[14] = 0x65
    assert O.ingress_verdict(bytes(b)) == O.ERR_INVALID_FIELD              # version != 4
    evil = G.ether(0x0800, G.ipv4(6, G.tcp(b""), flags=0x2000))
    assert O.ingress_verdict(evil) == 0
    assert O.ingress_verdict(evil, O.VERIFY_EVIL_BIT) == O.ERR_PACKET_DROP
    assert O.ingress_verdict(G.ether(0x0800, G.ipv4(17, b"1234567", fix_l4=False))) == O.ERR_TRUNCATED_FRAME
    assert O.ingress_verdict(G.ether(0x0800, G.ipv4(17, G.udp(b"", length=7)))) == O.ERR_INVALID_LENGTH_FIELD
    assert O.ingress_verdict(G.ether(0x0800, G.ipv4(17, G.udp(b"ab", length=11)))) == O.ERR_TRUNCATED_FRAME
    ok6 = G.ether(0x86DD, G.ipv6(17, G.udp(b"payload")))
    assert O.ingress_verdict(ok6) == 0
    assert O.ingress_verdict(ok6[:14 + 39]) == O.ERR_TRUNCATED_FRAME
    assert O.ingress_verdict(ok6[:-1]) == O.ERR_INVALID_LENGTH_FIELD       # pl + 40 > len


def test_quirks_kept():
    # UDP checksum 0 is not special-cased on receive (internet/stack-ip4.go:152-167)
    b = bytearray(G.ether(0x0800, G.ipv4(17, G.udp(b"data"))))
    b[40:42] = b"\0\0"
    assert O.ingress_verdict(bytes(b)) == O.ERR_BAD_CRC
    # IPv4 options are outside the header sum (ipv4/frame.go:144-146): flipping
    # an option byte breaks nothing the receive path checks
    b = bytearray(G.ether(0x0800, G.ipv4(6, G.tcp(b"x"), opts=b"\x01\x01\x01\x00")))
    b[34] ^= 0x40
    assert O.ingress_verdict(bytes(b)) == 0
    # IPv6 UDP sums the whole IPv6 payload, not the UDP length (stack-ip6.go:133-134):
    # bytes after the UDP length still count
    b = bytearray(G.ether(0x86DD, G.ipv6(17, G.udp(b"abcdef", length=10))))
    b[-1] ^= 0x01
    assert O.ingress_verdict(bytes(b)) == O.ERR_BAD_CRC


def test_generator_covers_every_verdict():
    hist = collections.Counter(O.ingress_verdict(f, O.VERIFY_EVIL_BIT) for f in G.frames(count=2400))
    for code in (0, O.ERR_PACKET_DROP, O.ERR_BAD_CRC, O.ERR_INVALID_FIELD, O.ERR_INVALID_LENGTH_FIELD,
                 O.ERR_TRUNCATED_FRAME):
        assert hist[code] > 0, (code, hist)


def _pack(frames, base_pad):
    parts, offs, pos = [b"\xAA" * base_pad], [base_pad], base_pad
    for f in frames:
        parts.append(f)
        pos += len(f)
        offs.append(pos)
    return np.frombuffer(b"".join(parts) + b"\0" * 8, dtype=np.uint8).copy(), np.array(offs, dtype=np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("base_pad", [0, 1, 2, 3])
@pytest.mark.parametrize("flags", [0, 1])
def test_gpu_ingress_verdicts_match_oracle(cuda, base_pad, flags):
    import torch
    import lneto_amd as L
    frames = G.frames(seed=10 + base_pad, count=4800)
    data, off = _pack(frames, base_pad)
    d = torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    got = L.ingress_verify_batch(d, o, flags=flags).cpu().numpy()
    want = np.array([O.ingress_verdict(f, flags) for f in frames], dtype=np.uint8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i]), len(frames[i])) for i in bad[:10]]


@pytest.mark.gpu
def test_gpu_ingress_reference_frames(cuda):
    import torch
    import lneto_amd as L
    frames = _kat_frames()
    frames += [bytes(b) for b in (bytearray(frames[0]),)]
    bad = bytearray(frames[1]); bad[60] ^= 0x20
    frames.append(bytes(bad))
    data, off = _pack(frames, 0)
    got = L.ingress_verify_batch(torch.from_numpy(data).to(cuda),
                                 torch.from_numpy(off.astype(np.int64)).to(cuda)).cpu().numpy()
    assert got.tolist() == [0, 0, 0, O.ERR_BAD_CRC]


def test_trailing_bytes_are_ignored():
    """Bytes past the transport end never reach a sum (the reference slices the
    frame to tl / the UDP length / pl + 40 before summing): valid frames pass
    whatever follows them, and a flip inside the covered range is ErrBadCRC."""
    frames = G.trailing_frames(count=300)
    for i, f in enumerate(frames):
        want = O.ERR_BAD_CRC if i % 3 == 0 else 0
        assert O.ingress_verdict(f) == want, i


@pytest.mark.gpu
@pytest.mark.parametrize("base_pad", [0, 1, 6])
def test_gpu_ingress_trailing_bytes(cuda, base_pad):
    """the first batch of qwords is loaded to the frame end;
    the ones past the transport end must not be summed."""
    import torch
    import lneto_amd as L
    frames = G.trailing_frames(seed=40 + base_pad, count=1200)
    data, off = _pack(frames, base_pad)
    got = L.ingress_verify_batch(torch.from_numpy(data).to(cuda),
                                 torch.from_numpy(off.astype(np.int64)).to(cuda)).cpu().numpy()
    want = np.array([O.ingress_verdict(f) for f in frames], dtype=np.uint8)
    assert (want == 0).sum() > 600
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i]), len(frames[i])) for i in bad[:10]]


def _header_then_udp_frames():
    """Corrupted IPv4 header AND a broken UDP size: demux4 checks the header sum
    (internet/stack-ip4.go:128-131) before udp.NewFrame / ValidateSize (:150-158),
    so the verdict is ErrBadCRC, not the UDP size error."""
    out = []
    for pay, ulen in [(b"", 7), (b"ab", 11), (b"abcdef", 40), (b"", None)]:
        for cut in (0, 4):
            good = G.ether(0x0800, G.ipv4(17, G.udp(pay, length=ulen)))
            if cut:  # transport shorter than a UDP header: tl shrunk with the frame
                b = bytearray(good[:14 + 20 + 4])
                b[16:18] = (24).to_bytes(2, "big")
                b[24:26] = b"\0\0"
                b[24:26] = O.ipv4_header_sum16(bytes(b[14:34])).to_bytes(2, "big")
                good = bytes(b)
            out.append(good)
            bad = bytearray(good)
            bad[22] ^= 0x01  # TTL: header sum breaks, lengths stay
            out.append(bytes(bad))
    return out


def test_header_sum_precedes_udp_size_checks():
    codes = [O.ingress_verdict(f) for f in _header_then_udp_frames()]
    assert codes[1::2] == [O.ERR_BAD_CRC] * (len(codes) // 2)
    assert set(codes[0::2]) >= {O.ERR_INVALID_LENGTH_FIELD, O.ERR_TRUNCATED_FRAME}


@pytest.mark.gpu
@pytest.mark.parametrize("base_pad", [0, 3])
def test_gpu_header_sum_precedes_udp_size_checks(cuda, base_pad):
    import torch
    import lneto_amd as L
    frames = _header_then_udp_frames()
    data, off = _pack(frames, base_pad)
    got = L.ingress_verify_batch(torch.from_numpy(data).to(cuda),
                                 torch.from_numpy(off.astype(np.int64)).to(cuda)).cpu().numpy()
    want = [O.ingress_verdict(f) for f in frames]
    assert got.tolist() == want


@pytest.mark.gpu
@pytest.mark.parametrize("base_pad", [0, 5])
def test_gpu_ingress_jumbo_frames(cuda, base_pad):
    """Jumbo IPv4/IPv6 TCP and UDP frames (up to 9000 B: several batches of
    lines per row), valid and with one corrupted payload byte each."""
    import torch
    import lneto_amd as L
    rng = np.random.default_rng(31 + base_pad)
    frames = []
    for i in range(400):
        n = int(rng.integers(1400, 8900))
        pay = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        kind = i % 4
        f = G.ether(0x0800, G.ipv4(6, G.tcp(pay))) if kind == 0 else \
            G.ether(0x0800, G.ipv4(17, G.udp(pay))) if kind == 1 else \
            G.ether(0x86DD, G.ipv6(6, G.tcp(pay))) if kind == 2 else G.ether(0x86DD, G.ipv6(17, G.udp(pay)))
        if i % 3 == 0:
            b = bytearray(f)
            b[int(rng.integers(60, len(b)))] ^= 0x10
            f = bytes(b)
        frames.append(f)
    data, off = _pack(frames, base_pad)
    d = torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    got = L.ingress_verify_batch(d, o).cpu().numpy()
    want = np.array([O.ingress_verdict(f, 0) for f in frames], dtype=np.uint8)
    assert (want == 3).sum() > 50 and (want == 0).sum() > 100
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i]), len(frames[i])) for i in bad[:10]]


# ---------------------------------------------------------------- ICMP verdicts
def _icmp_echo_cases():
    """TestStackAsync_ICMPEchoChecksum (x/xnet/xnet_test.go:1015-1110): a valid
    echo request, the same with 4 trailing FCS-like bytes (accepted: the client
    sums Payload(), sliced to tl), and both with the last payload byte flipped
    (rejected)."""
    pay = b"abcdefghijklmnopqrstuvwxyz012345"
    good = G.ltesto_icmp_echo(pay, 0x1234, 1)
    trailing = G.ltesto_icmp_echo(pay, 0x1234, 2) + bytes.fromhex("deadbeef")
    bad = bytearray(G.ltesto_icmp_echo(pay, 0x1234, 3)); bad[-1] ^= 0xFF
    bad_trailing = bytearray(G.ltesto_icmp_echo(pay, 0x1234, 4)); bad_trailing[-1] ^= 0xFF
    return [good, trailing, bytes(bad), bytes(bad_trailing) + bytes.fromhex("deadbeef")]


def test_reference_icmp_echo_checksum_cases():
    frames = _icmp_echo_cases()
    assert [O.ingress_verdict(f, O.VERIFY_ICMP) for f in frames] == [0, 0, O.ERR_BAD_CRC, O.ERR_BAD_CRC]
    # without the ICMP clients the checksum stage has nothing to say about ICMP
    assert [O.ingress_verdict(f) for f in frames] == [0, 0, 0, 0]


def test_icmp_order_and_codes():
    v4 = G.ether(0x0800, G.ipv4(1, G.icmp(8, b"ping")))
    assert O.ingress_verdict(v4, O.VERIFY_ICMP) == 0
    # a non-echo ICMPv4 type is dropped before its sum (ipv4/icmpv4/client.go:95-98)
    b = bytearray(G.ether(0x0800, G.ipv4(1, G.icmp(11, b"ttl exceeded")))); b[-1] ^= 1
    assert O.ingress_verdict(bytes(b), O.VERIFY_ICMP) == O.ERR_PACKET_DROP
    assert O.ingress_verdict(G.ether(0x0800, G.ipv4(1, b"1234567")), O.VERIFY_ICMP) == O.ERR_TRUNCATED_FRAME
    # the IPv4 header sum comes first
    b = bytearray(G.ether(0x0800, G.ipv4(1, b"1234567"))); b[22] ^= 1
    assert O.ingress_verdict(bytes(b), O.VERIFY_ICMP) == O.ERR_BAD_CRC
    # ICMPv6: size, then the pseudo-header sum; every type passes this stage
    for t in (1, 128, 129, 135, 136, 200):
        assert O.ingress_verdict(G.ether(0x86DD, G.ipv6(58, G.icmp(t, b"x" * t))), O.VERIFY_ICMP) == 0
    assert O.ingress_verdict(G.ether(0x86DD, G.ipv6(58, b"1234567")), O.VERIFY_ICMP) == O.ERR_TRUNCATED_FRAME
    b = bytearray(G.ether(0x86DD, G.ipv6(58, G.icmp(128, b"abc")))); b[30] ^= 4  # source address
    assert O.ingress_verdict(bytes(b), O.VERIFY_ICMP) == O.ERR_BAD_CRC
    assert O.ingress_verdict(bytes(b)) == 0


def test_icmp_generator_covers_every_verdict():
    hist = collections.Counter(O.ingress_verdict(f, O.VERIFY_ICMP) for f in G.icmp_frames(count=1200))
    for code in (0, O.ERR_PACKET_DROP, O.ERR_BAD_CRC, O.ERR_TRUNCATED_FRAME):
        assert hist[code] > 50, (code, hist)


def test_icmp_generate_then_verify():
    """The TX generate step (oracle.tx_checksum, the ICMP clients' SetCRC) and
    the ICMP verdicts agree: a generated echo passes."""
    for f in G.icmp_frames(seed=5, count=240)[::12]:
        regen, st = O.tx_checksum(f)
        if st == 0:
            assert O.ingress_verdict(regen, O.VERIFY_ICMP) == 0


@pytest.mark.gpu
@pytest.mark.parametrize("base_pad", [0, 1, 6])
@pytest.mark.parametrize("flags", [2, 3])
def test_gpu_icmp_verdicts_match_oracle(cuda, base_pad, flags):
    import torch
    import lneto_amd as L
    frames = G.icmp_frames(seed=50 + base_pad, count=2400) + _icmp_echo_cases() \
        + G.frames(seed=60 + base_pad, count=2400)
    data, off = _pack(frames, base_pad)
    got = L.ingress_verify_batch(torch.from_numpy(data).to(cuda), torch.from_numpy(off.astype(np.int64)).to(cuda),
                                 flags=flags).cpu().numpy()
    want = np.array([O.ingress_verdict(f, flags) for f in frames], dtype=np.uint8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i]), len(frames[i])) for i in bad[:10]]


@pytest.mark.gpu
@pytest.mark.parametrize("route", ["rx_verify", "ingress_rows"])
@pytest.mark.parametrize("filt", [None, "plain", "few_handlers"])
@pytest.mark.parametrize("flags", [0, 3])
def test_gpu_ingress_both_routes(cuda, route, filt, flags):
    """lnx_ingress_verify_batch launches the ingress rows and the receive check
    without its CRC (rx_verify_kernel), and the one the batch's mean frame
    length picks works (api.cpp kIngressShortMean, 1280 B): the generator's,
    the ICMP and the filter frames alone (mean ~100 B: the receive check) and
    with long valid frames after them so that the mean passes 1280 B (the
    ingress rows), both against the oracle, with and without a stack filter."""
    import torch
    import lneto_amd as L
    from tests.test_rx_filter import _pair
    frames = G.frames(seed=91, count=1500) + G.icmp_frames(seed=92, count=400) + G.filter_frames(seed=93, count=600)
    if route == "ingress_rows":
        rng = np.random.default_rng(94)
        need = 1280 * len(frames) - sum(len(f) for f in frames)
        while need > -1280 * (len(frames) + 1):  # (the mean past the threshold with margin)
            pay = rng.integers(0, 256, size=int(rng.integers(7000, 8900)), dtype=np.uint8).tobytes()
            f = G.ether(0x0800, G.ipv4(17, G.udp(pay))) if len(frames) % 2 else G.ether(0x86DD, G.ipv6(6, G.tcp(pay)))
            frames.append(f)
            need += 1280 - len(f)
    mean = sum(len(f) for f in frames) / len(frames)
    assert (mean >= 1280) == (route == "ingress_rows")
    of, lf = _pair(filt) if filt else (None, None)
    data, off = _pack(frames, 3)
    got = L.ingress_verify_batch(torch.from_numpy(data).to(cuda), torch.from_numpy(off.astype(np.int64)).to(cuda),
                                 flags=flags, filter=lf).cpu().numpy()
    want = np.array([O.ingress_verdict(f, flags, of) for f in frames], dtype=np.uint8)
    assert len(set(want.tolist())) >= 4
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, [(int(i), int(got[i]), int(want[i]), len(frames[i])) for i in bad[:10]]
