"""The fused receive check (lnx_rx_verify_batch, lneto_amd/csrc/rx_verify_kernel.hip,
DESIGN.md §3.12) on the GPU against the oracle: for every frame carrying its LE
FCS (internet/stack-ethernet.go:211-214), fcs_ok = CRC32(frame) == residue
(len >= 4) and verdict = oracle.ingress_verdict(frame without its FCS)
(StackEthernet.Demux + demux4 / demux6, internet/stack-ethernet.go:139-168,
internet/stack-ip4.go:100-167, internet/stack-ip6.go:86-138), with and without
the stack filter, the ICMP and evil-bit flags, FCS-less devices
(LNX_RX_NO_FCS), every base alignment, Zipf and jumbo frames.  The CRC algebra
is pinned on the host in tests/test_rx_verify_algebra.py."""
import struct

import numpy as np
import pytest

from oracle import oracle as O
from tests import framegen as G
from tests.test_rx_filter import FILTERS, _pair

pytestmark = pytest.mark.gpu


def _with_fcs(f: bytes) -> bytes:
    return f + struct.pack("<I", O.crc32(f))


def _case_frames(frames, seed):
    """Frames with FCS: a flipped byte (FCS fails) in some, a few shorter than 4 bytes."""
    rng = np.random.default_rng(seed)
    out = []
    for f in frames:
        b = bytearray(_with_fcs(f))
        r = rng.random()
        if r < 0.15 and len(b) > 4:
            b[rng.integers(0, len(b))] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.17:
            b = b[: int(rng.integers(0, 4))]
        out.append(bytes(b))
    return out


def _pack(frames, base_pad):
    parts, offs, pos = [b"\xAA" * base_pad], [base_pad], base_pad
    for f in frames:
        parts.append(f)
        pos += len(f)
        offs.append(pos)
    return np.frombuffer(b"".join(parts) + b"\xBB" * 24, dtype=np.uint8).copy(), np.array(offs, dtype=np.int64)


def _run(cuda, frames, base_pad, flags=0, cfilt=None):
    import torch
    import lneto_amd as L
    data, off = _pack(frames, base_pad)
    d, o = torch.from_numpy(data).to(cuda), torch.from_numpy(off).to(cuda)
    ok, verdict = L.rx_verify_batch(d, o, flags=flags, filter=cfilt)
    return ok.cpu().numpy(), verdict.cpu().numpy()


def _want(frames, flags=0, ofilt=None, fcs=True):
    if not fcs:
        return np.ones(len(frames), np.uint8), np.array([O.ingress_verdict(f, flags & 3, ofilt) for f in frames], np.uint8)
    ok = np.array([int(len(f) >= 4 and O.crc32(f) == O.CRC32_RESIDUE) for f in frames], np.uint8)
    v = np.array([O.ingress_verdict(f[:-4] if len(f) >= 4 else b"", flags & 3, ofilt) for f in frames], np.uint8)
    return ok, v


def _cmp(got, want, frames):
    for name, g, w in zip(("fcs_ok", "verdict"), got, want):
        bad = np.nonzero(g != w)[0]
        assert bad.size == 0, (name, [(int(i), int(g[i]), int(w[i]), len(frames[i])) for i in bad[:8]])


@pytest.mark.parametrize("base_pad", range(8))
@pytest.mark.parametrize("flags", [0, 1, 2, 3])
def test_rx_verify_matches_oracle(cuda, base_pad, flags):
    frames = _case_frames(G.frames(seed=40 + base_pad, count=2000) + G.icmp_frames(seed=50 + base_pad, count=400)
                          + G.trailing_frames(seed=60 + base_pad, count=200), seed=base_pad)
    _cmp(_run(cuda, frames, base_pad, flags), _want(frames, flags), frames)


@pytest.mark.parametrize("name", sorted(FILTERS))
@pytest.mark.parametrize("base_pad", [0, 3, 5])
def test_rx_verify_filtered(cuda, name, base_pad):
    import lneto_amd as L
    ofilt, cfilt = _pair(name)
    frames = _case_frames(G.filter_frames(seed=70 + base_pad, count=2400), seed=80 + base_pad)
    for flags in (0, L.VERIFY_ICMP):
        _cmp(_run(cuda, frames, base_pad, flags, cfilt), _want(frames, flags, ofilt), frames)


@pytest.mark.parametrize("base_pad", [0, 1, 6])
def test_rx_verify_no_fcs(cuda, base_pad):
    """LNX_RX_NO_FCS: no CRC, fcs_ok = 1, the verdict on the whole frame."""
    import lneto_amd as L
    frames = G.frames(seed=90 + base_pad, count=1500)
    _cmp(_run(cuda, frames, base_pad, L.RX_NO_FCS), _want(frames, 0, None, fcs=False), frames)


def test_rx_verify_lengths_zipf_jumbo(cuda):
    """Every length 0..2000 (raw bytes: the FCS test alone decides), the Zipf mix,
    9000-B and 20 000-B frames (several batches of 1536 bytes per row)."""
    import torch
    import lneto_amd as L
    from lneto_amd import synth
    rng = np.random.default_rng(99)
    for lens, pad in ((rng.permutation(np.arange(0, 2001)), 3), (synth.zipf_lengths(200_000, seed=98), 0),
                      (np.array([9000, 20000, 64, 9018, 1518] * 200), 7)):
        lens = np.asarray(lens, np.int64)
        off = synth.offsets_from_lengths(lens).astype(np.int64) + pad
        data = synth.bytes_np(int(off[-1]) + 16, seed=int(lens.size))
        # two thirds of the frames get a valid FCS
        for i in range(0, len(lens), 3):
            for j in (i, i + 1):
                if j < len(lens) and lens[j] >= 4:
                    s, e = int(off[j]), int(off[j + 1])
                    data[e - 4:e] = np.frombuffer(int(O.c_crc32(data[s:e - 4].tobytes())).to_bytes(4, "little"), np.uint8)
        d, o = torch.from_numpy(data).to(cuda), torch.from_numpy(off).to(cuda)
        ok, verdict = L.rx_verify_batch(d, o)
        ok, verdict = ok.cpu().numpy(), verdict.cpu().numpy()
        want = O.crc32_frames(data, off.astype(np.uint64), threads=8)
        want_ok = ((want == O.CRC32_RESIDUE) & (lens >= 4)).astype(np.uint8)
        assert (ok == want_ok).all(), np.nonzero(ok != want_ok)[0][:10]
        assert want_ok.sum() > len(lens) // 2
        # verdicts of raw bytes: as the ingress kernel gives them on the frames without FCS
        d2 = torch.from_numpy(data).to(cuda)
        o2 = torch.from_numpy(np.stack([off[:-1], np.maximum(off[1:] - 4, off[:-1])], 1).reshape(-1)).to(cuda)
        v2 = L.ingress_verify_batch(d2, o2).cpu().numpy()[::2]
        assert (verdict == v2).all(), np.nonzero(verdict != v2)[0][:10]


def test_rx_verify_equals_the_two_kernels(cuda):
    """On 256 Ki x 1500-B UDP frames (bench.py --op rx_verify's shape): the one-pass
    results equal lnx_fcs_verify_batch + lnx_ingress_verify_batch on the frames
    without their FCS."""
    import torch
    import lneto_amd as L
    from lneto_amd import synth
    n, flen = 1 << 18, 1500
    rows = torch.from_numpy(_udp_rows(n, flen)).to(cuda)
    d = rows.reshape(-1)
    o = torch.arange(n + 1, dtype=torch.int64, device=cuda) * flen
    ok, verdict = L.rx_verify_batch(d, o)
    assert int(ok.sum()) == n and int((verdict == 0).sum()) == n
    d[(n // 2) * flen + 700] ^= 1
    ok, verdict = L.rx_verify_batch(d, o)
    assert int(ok.sum()) == n - 1 and int(ok[n // 2]) == 0 and int(verdict[n // 2]) == O.ERR_BAD_CRC
    ok2 = L.fcs_verify_batch(d, o)
    o3 = torch.stack([o[:-1], o[1:] - 4], 1).reshape(-1)
    v3 = L.ingress_verify_batch(d, o3)[::2]
    assert torch.equal(ok, ok2) and torch.equal(verdict, v3)


def _udp_rows(n, flen):
    """n UDP/IPv4 frames of flen bytes (FCS included) with valid sums and FCS."""
    from lneto_amd import synth
    rows = synth.bytes_np(n * flen, seed=123).reshape(n, flen)
    L = flen - 4
    rows[:, 0:14] = np.frombuffer(bytes.fromhex("c0ffee00dead4e8b3af9fb6b0800"), np.uint8)
    rows[:, 14:34] = np.frombuffer(bytes.fromhex("4500") + (L - 14).to_bytes(2, "big") +
                                   bytes.fromhex("0000400040110000c0a80a01c0a80a02"), np.uint8)
    rows[:, 34:42] = np.frombuffer(bytes.fromhex("14e90035") + (L - 34).to_bytes(2, "big") + b"\0\0", np.uint8)
    # header CRC (identical headers) then the UDP sums and the FCS on the host
    hdr = bytearray(rows[0, 14:34].tobytes())
    c = O.CRC791()
    c.write_even(bytes(hdr))
    rows[:, 24:26] = np.frombuffer(c.sum16().to_bytes(2, "big"), np.uint8)
    seed = O.ipv4_udp_pseudo(bytes(rows[0, 14:34]), L - 34).sum  # the same pseudo-header for every frame
    for i in range(n):
        fr = rows[i]
        s = O.c_payload_sum16(seed, fr[34:L].tobytes())
        fr[40:42] = np.frombuffer(O.never_zero_sum(s).to_bytes(2, "big"), np.uint8)
    fcs = O.crc32_frames(rows[:, :L].copy().reshape(-1), np.arange(n + 1, dtype=np.uint64) * L, threads=8)
    rows[:, L:flen] = fcs.view(np.uint8).reshape(n, 4)
    return rows


@pytest.mark.parametrize("n", [1, 2, 3, 5, 9, 52, 55, 57, 63, 64, 65, 897, 1000, 4097, 20000])
def test_rx_verify_batch_sizes(cuda, n):
    """Batches of every shape the launcher's group size takes (balanced_group:
    4 to 56 frames a group, the last group part-full) against the oracle."""
    base = _case_frames(G.frames(seed=70, count=400) + G.icmp_frames(seed=71, count=60), seed=72)
    frames = [base[i % len(base)] for i in range(n)]
    _cmp(_run(cuda, frames, n % 8), _want(frames), frames)
