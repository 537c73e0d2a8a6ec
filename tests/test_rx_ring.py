"""Receive ring: pinned slots -> H2D -> FCS verify + receive-path
verdicts -> D2H, the batch form of netdev.Stack.IngressPackets(bufs, offset)
(x/netdev/interface.go:82-89, x/xnet/netstack.go:103-111).

Every frame carries its LE FCS (internet/stack-ethernet.go:211-214).  Expected
values come from the oracle: fcs_ok = CRC32(frame) == residue (len >= 4), verdict
= oracle.ingress_verdict(frame without its FCS)."""
import struct

import numpy as np
import pytest

import lneto_amd as L
from oracle import oracle as O
from tests import framegen as G


def _with_fcs(f: bytes) -> bytes:
    return f + struct.pack("<I", O.crc32(f))


def _case_frames(seed: int, count: int):
    """Frames with FCS: valid ones, some with a flipped payload / FCS byte, short ones."""
    rng = np.random.default_rng(seed)
    out = []
    base = G.frames(seed=seed, count=count)
    for i, f in enumerate(base):
        b = bytearray(_with_fcs(f))
        r = rng.random()
        if r < 0.15 and len(b) > 4:
            b[rng.integers(0, len(b))] ^= 1 << int(rng.integers(0, 8))  # corrupt: FCS fails
        elif r < 0.18:
            b = b[: int(rng.integers(0, 4))]  # shorter than an FCS
        out.append(bytes(b))
    return out


def _expect(frames):
    ok = np.array([int(len(f) >= 4 and O.crc32(f) == L.CRC32_RESIDUE) for f in frames], dtype=np.uint8)
    verdict = np.array([O.ingress_verdict(f[:-4] if len(f) >= 4 else b"") for f in frames], dtype=np.uint8)
    return ok, verdict


def _ring(*a, **kw):
    """A ring whose batches all go to the GPU (host threshold 0), whatever their size."""
    kw.setdefault("host_threshold", 0)
    return L.RxRing(*a, **kw)


def _cap_for(frames, offset):
    """Slot capacity: the largest buffer, rounded up to 4 bytes."""
    return (max(len(f) for f in frames) + offset + 3) & ~3


def test_ring_requires_a_device():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(L.LnetoError):
        L.RxRing(16)


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [True, False])
@pytest.mark.parametrize("offset", [0, 2, 16])
def test_ring_slots_ingress(cuda, offset, zero_copy):
    frames = _case_frames(seed=11 + offset, count=1200)
    cap = _cap_for(frames, offset)
    ring = _ring(len(frames) + 7, slot_cap=cap, batch_slots=256, depth=3)
    try:
        ring.set_zero_copy(zero_copy)
        for i, f in enumerate(frames):
            ring.slots[i + 7, :offset] = 0xEE  # headroom before the frame
            ring.slots[i + 7, offset:offset + len(f)] = np.frombuffer(f, dtype=np.uint8)
            ring.lengths[i + 7] = offset + len(f)
        ok, verdict = ring.ingress(first=7, count=len(frames), offset=offset)
        want_ok, want_v = _expect(frames)
        assert np.array_equal(ok, want_ok)
        bad = np.flatnonzero(verdict != want_v)
        assert bad.size == 0, [(int(i), int(verdict[i]), int(want_v[i]), len(frames[i])) for i in bad[:20]]
        assert want_ok.sum() > 900 and (want_ok == 0).sum() > 150
        assert ring.stats()["zero_copy_frames"] == (len(frames) if zero_copy else 0)
    finally:
        ring.close()


@pytest.mark.gpu
def test_ring_evil_bit_flag(cuda):
    frames = _case_frames(seed=5, count=600)
    ring = _ring(len(frames), slot_cap=_cap_for(frames, 0), batch_slots=200, depth=2)
    try:
        ok, verdict = ring.ingress_packets(frames, offset=0, flags=L.VERIFY_EVIL_BIT)
        want_v = np.array([O.ingress_verdict(f[:-4] if len(f) >= 4 else b"", O.VERIFY_EVIL_BIT) for f in frames],
                          dtype=np.uint8)
        assert np.array_equal(verdict, want_v)
    finally:
        ring.close()


@pytest.mark.gpu
def test_ingress_packets_gather(cuda):
    """Caller-owned buffers, more frames than the ring has slots (several gather
    rounds over the stages), empty buffers and full-capacity buffers."""
    frames = _case_frames(seed=3, count=2500)
    rng = np.random.default_rng(9)
    offset = 4
    cap = _cap_for(frames, offset)
    frames += [b"", b"\x01\x02", bytes(rng.integers(0, 256, 1020, dtype=np.uint8))]
    frames.append(_with_fcs(bytes(rng.integers(0, 256, cap - offset - 4, dtype=np.uint8))))  # fills the slot
    bufs = [b"\xAA" * offset + f for f in frames]
    assert max(len(b) for b in bufs) == cap
    ring = _ring(600, slot_cap=cap, batch_slots=100, depth=3)
    try:
        ok, verdict = ring.ingress_packets(bufs, offset=offset)
    finally:
        ring.close()
    want_ok, want_v = _expect(frames)
    assert np.array_equal(ok, want_ok)
    assert np.array_equal(verdict, want_v)
    assert ok[-1] == 1


@pytest.mark.gpu
def test_ingress_packets_rejects_oversize(cuda):
    ring = _ring(8, slot_cap=64)
    try:
        with pytest.raises(L.LnetoError):
            ring.ingress_packets([b"x" * 65])
    finally:
        ring.close()


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [True, False])
def test_ring_mtu_batch_roundtrip(cuda, zero_copy):
    """64 Ki x 1500-byte frames with FCS through the pipelined ring: all pass;
    then one flipped byte per 1000 frames fails exactly those frames."""
    n, flen = 1 << 16, 1500
    ring = _ring(n, slot_cap=1536, batch_slots=8192, depth=3)
    try:
        ring.set_zero_copy(zero_copy)
        rng = np.random.default_rng(1)
        data = rng.integers(0, 256, (n, flen - 4), dtype=np.uint8)
        ring.slots[:, : flen - 4] = data
        crcs = np.array([O.crc32(r.tobytes()) for r in data[:256]], dtype=np.uint32)
        # FCS for all rows via the device CRC of the same bytes
        import torch
        d = torch.from_numpy(data.reshape(-1)).to(cuda)
        off = torch.arange(n + 1, dtype=torch.int64, device=cuda) * (flen - 4)
        fcs = L.crc32_batch(d, off).cpu().numpy().view(np.uint32)
        assert np.array_equal(fcs[:256], crcs)
        ring.slots[:, flen - 4: flen] = fcs.view(np.uint8).reshape(n, 4)
        ring.lengths[:] = flen
        ok, _ = ring.ingress(0, n)
        assert ok.all()
        bad = np.arange(0, n, 1000)
        ring.slots[bad, 77] ^= 0x10
        ok, _ = ring.ingress(0, n)
        assert np.array_equal(np.flatnonzero(ok == 0), bad)
    finally:
        ring.close()


@pytest.mark.gpu
@pytest.mark.parametrize("nslots", [1, 2, 3])
def test_ingress_packets_fewer_slots_than_stages(cuda, nslots):
    """A ring with fewer slots than pipeline stages (depth 3) gathers into its
    own slots only (the stage block used to run past the pool)."""
    frames = _case_frames(seed=40 + nslots, count=37)
    ring = _ring(nslots, slot_cap=_cap_for(frames, 0), depth=3)
    try:
        ok, verdict = ring.ingress_packets(frames, offset=0)
    finally:
        ring.close()
    want_ok, want_v = _expect(frames)
    assert np.array_equal(ok, want_ok)
    assert np.array_equal(verdict, want_v)


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [L.TX_CHECKSUM | L.TX_FCS, L.TX_FCS, L.TX_CHECKSUM])
def test_egress_packets_matches_oracle(cuda, flags):
    """netdev.Stack.EgressPackets(bufs, sizes, offset) (x/netdev/interface.go:85)
    for the device's part of the transmit path: checksum generate
    (oracle.tx_checksum), then pad + FCS (oracle.fcs_append), in place in
    caller-owned buffers, more frames than the ring has slots."""
    from tests.test_tx_checksum import tx_frames
    frames = [f for f in tx_frames(seed=60, count=1500) if len(f) <= 2000]
    offset, cap = 6, 2048
    rng = np.random.default_rng(61)
    bufs = []
    for f in frames:
        b = rng.integers(0, 256, offset + cap + 16, dtype=np.uint8)
        b[offset:offset + len(f)] = np.frombuffer(f, dtype=np.uint8)
        bufs.append(b)
    before = [b.copy() for b in bufs]
    ring = _ring(300, slot_cap=cap, batch_slots=128, depth=3)
    try:
        sizes, status = ring.egress_packets(bufs, [len(f) for f in frames], offset=offset, capacity=cap,
                                            flags=flags)
    finally:
        ring.close()
    bad = []
    for i, f in enumerate(frames):
        want, st = (O.tx_checksum(f) if flags & L.TX_CHECKSUM else (f, 0))
        st2 = 0
        if flags & L.TX_FCS:
            want, st2 = O.fcs_append(want, cap)
        got = bufs[i][offset:offset + int(sizes[i])].tobytes()
        if got != want or int(status[i]) != (st or st2):
            bad.append((i, len(f), int(sizes[i]), len(want), int(status[i]), st or st2))
        # bytes outside the finished frame are the caller's
        assert np.array_equal(bufs[i][:offset], before[i][:offset])
        assert np.array_equal(bufs[i][offset + len(want):], before[i][offset + len(want):])
    assert not bad, bad[:10]


@pytest.mark.gpu
def test_ring_icmp_flag(cuda):
    """IngressPackets with the ICMP clients attached (LNX_VERIFY_ICMP): ICMPv4 /
    ICMPv6 frames with their FCS, echo and other types, short and corrupted
    messages; the flag travels through the ring's stages to the verdict kernel."""
    frames = [_with_fcs(f) for f in G.icmp_frames(seed=21, count=1200)]
    flags = L.VERIFY_ICMP | L.VERIFY_EVIL_BIT
    ring = _ring(400, slot_cap=_cap_for(frames, 0), batch_slots=100, depth=3)
    try:
        ok, verdict = ring.ingress_packets(frames, offset=0, flags=flags)
    finally:
        ring.close()
    want_v = np.array([O.ingress_verdict(f[:-4], flags) for f in frames], dtype=np.uint8)
    assert ok.all()
    assert set(want_v.tolist()) >= {0, O.ERR_BAD_CRC, O.ERR_PACKET_DROP, O.ERR_TRUNCATED_FRAME}
    assert np.array_equal(verdict, want_v)


def _fill_ring(ring, frames, offset):
    for i, f in enumerate(frames):
        ring.slots[i, :offset] = 0xEE
        ring.slots[i, offset:offset + len(f)] = np.frombuffer(f, dtype=np.uint8)
        ring.lengths[i] = offset + len(f)


@pytest.mark.gpu
@pytest.mark.parametrize("dense", [True, False])
def test_ring_without_fcs(cuda, dense):
    """LNX_RX_NO_FCS: a device that strips the FCS (x/netdev/interface.go:34-40)
    — no FCS check, fcs_ok = 1, verdicts over the whole frame.  dense: frames
    that fill their slots (whole-slot copies), else a mix packed on the host."""
    if dense:
        base = [f for f in G.frames(seed=77, count=3000) if len(f) >= 1000][:400]
        frames = [f[:1000] for f in base]  # same length: every slot 1000 of 1000 bytes
    else:
        frames = G.frames(seed=78, count=1500)
    offset = 2
    cap = _cap_for(frames, offset)
    for how in ("slots", "packets"):
        ring = _ring(len(frames), slot_cap=cap, batch_slots=256, depth=3)
        try:
            if how == "slots":
                _fill_ring(ring, frames, offset)
                ok, verdict = ring.ingress(0, len(frames), offset=offset, flags=L.RX_NO_FCS)
            else:
                ok, verdict = ring.ingress_packets([b"\xEE" * offset + f for f in frames], offset=offset,
                                                   flags=L.RX_NO_FCS)
        finally:
            ring.close()
        want = np.array([O.ingress_verdict(f) for f in frames], dtype=np.uint8)
        assert ok.all(), how
        bad = np.flatnonzero(verdict != want)
        assert bad.size == 0, (how, [(int(i), int(verdict[i]), int(want[i])) for i in bad[:10]])


@pytest.mark.gpu
@pytest.mark.parametrize("no_fcs", [False, True])
def test_ring_filter_precedence(cuda, no_fcs):
    """lnx_rx_ring_set_filter: not-for-us frames (MAC, IPv4 / IPv6 address) and
    frames without a handler get ErrPacketDrop before or after the other checks
    as lneto orders them, with and without FCS; set_filter(None) restores accept-all."""
    from tests.test_rx_filter import _pair
    ofilt, cfilt = _pair("plain")
    frames = G.filter_frames(seed=91, count=1800)
    bufs = frames if no_fcs else [_with_fcs(f) for f in frames]
    flags = L.VERIFY_ICMP | (L.RX_NO_FCS if no_fcs else 0)
    ring = _ring(len(bufs), slot_cap=_cap_for(bufs, 0), batch_slots=512, depth=2)
    try:
        ring.set_filter(cfilt)
        ok, verdict = ring.ingress_packets(bufs, offset=0, flags=flags)
        _fill_ring(ring, bufs, 0)
        ok2, verdict2 = ring.ingress(0, len(bufs), offset=0, flags=flags)
        ring.set_filter(None)
        _, verdict3 = ring.ingress_packets(bufs, offset=0, flags=flags)
    finally:
        ring.close()
    want = np.array([O.ingress_verdict(f, L.VERIFY_ICMP, ofilt) for f in frames], dtype=np.uint8)
    want_all = np.array([O.ingress_verdict(f, L.VERIFY_ICMP) for f in frames], dtype=np.uint8)
    assert ok.all() and ok2.all()
    assert np.array_equal(verdict, want) and np.array_equal(verdict2, want)
    assert np.array_equal(verdict3, want_all)
    assert (want == O.ERR_PACKET_DROP).sum() > 400


@pytest.mark.gpu
@pytest.mark.parametrize("zero_copy", [True, False])
def test_ring_packed_zipf_lengths(cuda, zero_copy):
    """Zipf-mix frames (64-1500 B, mean ~246) in 1536-B slots: the batches are
    packed back to back (PCIe carries the frames, not the slots); every FCS and
    verdict as the oracle says, including corrupted and empty frames."""
    from lneto_amd import synth
    lens = synth.zipf_lengths(6000, seed=5)
    rng = np.random.default_rng(5)
    frames = []
    for i, l in enumerate(lens):
        f = G.ether(0x0800, G.ipv4(17, G.udp(rng.integers(0, 256, max(0, int(l) - 46), dtype=np.uint8).tobytes())))
        f = _with_fcs(f)
        if i % 97 == 0:
            f = _flip(f, int(rng.integers(0, len(f))))
        if i % 501 == 0:
            f = b""
        frames.append(f)
    ring = _ring(len(frames), slot_cap=1536, batch_slots=1024, depth=3)
    try:
        ring.set_zero_copy(zero_copy)
        _fill_ring(ring, frames, 0)
        ok, verdict = ring.ingress(0, len(frames))
        ok2, verdict2 = ring.ingress_packets(frames)
    finally:
        ring.close()
    want_ok, want_v = _expect(frames)
    assert np.array_equal(ok, want_ok) and np.array_equal(ok2, want_ok)
    assert np.array_equal(verdict, want_v) and np.array_equal(verdict2, want_v)
    assert (want_ok == 0).sum() >= 60


def _flip(f: bytes, i: int) -> bytes:
    b = bytearray(f)
    b[i] ^= 0x08
    return bytes(b)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [1, 8, 63, 64, 200])
def test_host_threshold_paths_agree(cuda, n):
    """Batches below the host threshold (LNX_HOST_BATCH_DEFAULT) run on the
    host with no launch, the others on the GPU; both equal the oracle, for
    ingress_packets, ring slots and egress_packets (netdev's Runner calls with
    n = 1, x/netdev/runner.go:432-433)."""
    frames = _case_frames(seed=900 + n, count=n)
    want_ok, want_v = _expect(frames)
    cap = max(1536, _cap_for(frames, 0) + 64)  # (room for the egress padding and FCS)
    for thr, where in ((L.HOST_BATCH_DEFAULT, "host" if n < L.HOST_BATCH_DEFAULT else "device"), (0, "device")):
        ring = L.RxRing(max(n, 1), slot_cap=cap, batch_slots=128, depth=2, host_threshold=thr)
        try:
            s0 = ring.stats()
            ok, verdict = ring.ingress_packets(frames)
            assert (ok == want_ok).all() and (verdict == want_v).all(), (thr, n)
            for i, f in enumerate(frames):
                ring.slots[i, :len(f)] = np.frombuffer(f, np.uint8)
                ring.lengths[i] = len(f)
            ok2, verdict2 = ring.ingress(0, n)
            assert (ok2 == want_ok).all() and (verdict2 == want_v).all(), (thr, n)
            s1 = ring.stats()
            if where == "host":
                assert s1["device_batches"] == s0["device_batches"] and s1["host_frames"] - s0["host_frames"] == 2 * n
            else:
                assert s1["device_batches"] > s0["device_batches"] and s1["device_frames"] - s0["device_frames"] == 2 * n
            # egress: the same frames (FCS stripped) finished in place, checked against the oracle
            bufs = [np.zeros(cap, dtype=np.uint8) for _ in frames]
            sizes = []
            for b, f in zip(bufs, frames):
                body = f[:-4] if len(f) >= 4 else f
                b[:len(body)] = np.frombuffer(body, np.uint8)
                sizes.append(len(body))
            lens, status = ring.egress_packets(bufs, sizes, offset=0, capacity=cap)
            for k, f in enumerate(frames):
                body = f[:-4] if len(f) >= 4 else f
                g, st = O.tx_checksum(body)
                fin, st2 = O.fcs_append(g, cap)
                assert int(status[k]) == (st or st2) and int(lens[k]) == len(fin), (thr, k)
                assert bufs[k][:len(fin)].tobytes() == fin, (thr, k)
        finally:
            ring.close()


@pytest.mark.gpu
@pytest.mark.parametrize("offset", [0, 6])
def test_packets_on_ring_slots(cuda, offset):
    """Zero copy at the netdev boundary: RunnerConfig.Buffers carved from the
    ring's slots (x/netdev/runner.go:92-94), so IngressPackets / EgressPackets
    get views of the ring's pinned memory and the kernels read (egress: patch)
    the frames in place.  Against the oracle, with the copying path on the same
    frames, with a buffer outside the ring (that batch is staged) and egress
    buffers out of slot order."""
    from tests.test_tx_checksum import tx_frames
    rx = _case_frames(seed=70 + offset, count=700)
    cap = max(1536, _cap_for(rx, offset))
    ring = _ring(1000, slot_cap=cap, batch_slots=256, depth=3)
    try:
        views = []
        for i, f in enumerate(rx):
            ring.slots[i, :offset] = 0xEE
            ring.slots[i, offset:offset + len(f)] = np.frombuffer(f, np.uint8)
            views.append(ring.slots[i, :offset + len(f)])
        s0 = ring.stats()["zero_copy_frames"]
        ok, verdict = ring.ingress_packets(views, offset=offset)
        assert ring.stats()["zero_copy_frames"] - s0 == len(rx)
        want_ok, want_v = _expect(rx)
        assert np.array_equal(ok, want_ok) and np.array_equal(verdict, want_v)
        # one buffer outside the ring: those batches are gathered, same results
        mixed = list(views)
        mixed[300] = np.frombuffer(b"\xEE" * offset + rx[300], np.uint8)
        ok2, verdict2 = ring.ingress_packets(mixed, offset=offset)
        assert np.array_equal(ok2, want_ok) and np.array_equal(verdict2, want_v)

        # egress in place: frames written by the "stack" into the slots, finished there
        tx = [f for f in tx_frames(seed=80 + offset, count=900) if len(f) <= cap - offset - 64][:700]
        capacity = cap - offset
        for order in ("slots", "reversed"):
            rng = np.random.default_rng(81)
            junk = rng.integers(0, 256, (len(tx), cap), dtype=np.uint8)
            ring.slots[:len(tx)] = junk
            for i, f in enumerate(tx):
                ring.slots[i, offset:offset + len(f)] = np.frombuffer(f, np.uint8)
            idx = list(range(len(tx))) if order == "slots" else list(range(len(tx)))[::-1]
            bufs = [ring.slots[i] for i in idx]
            s0 = ring.stats()["zero_copy_frames"]
            sizes, status = ring.egress_packets(bufs, [len(tx[i]) for i in idx], offset=offset, capacity=capacity)
            zc = ring.stats()["zero_copy_frames"] - s0
            assert zc == len(tx), (order, zc)  # slot buffers in any order are patched in place
            bad = []
            for k, i in enumerate(idx):
                want, st = O.tx_checksum(tx[i])
                want, st2 = O.fcs_append(want, capacity)
                got = ring.slots[i, offset:offset + int(sizes[k])].tobytes()
                if got != want or int(status[k]) != (st or st2):
                    bad.append((order, i, len(tx[i]), int(sizes[k]), len(want), int(status[k])))
                assert np.array_equal(ring.slots[i, :offset], junk[i, :offset])
                assert np.array_equal(ring.slots[i, offset + len(want):], junk[i, offset + len(want):]), (order, i)
            assert not bad, bad[:10]
    finally:
        ring.close()


@pytest.mark.gpu
@pytest.mark.parametrize("flags", [L.TX_CHECKSUM | L.TX_FCS, L.TX_FCS, L.TX_CHECKSUM])
@pytest.mark.parametrize("offset", [0, 3])
def test_egress_in_place_matches_oracle(cuda, flags, offset):
    """Zero-copy egress (tx_finish_kernel, rx_verify_kernel.hip): frames written
    into the ring's slots, finished in place by one kernel that reads each frame
    once -- checksum generate (oracle.tx_checksum) with the CRC corrected for
    the fields it writes, then the padding and FCS (oracle.fcs_append) -- for
    every protocol the step knows, runts, frames too short, and frames whose
    padded length does not fit `capacity` (ErrShortBuffer)."""
    from tests.test_tx_checksum import tx_frames
    cap = 2048
    frames = [f for f in tx_frames(seed=70 + offset, count=1400) if len(f) <= 1900]
    rng = np.random.default_rng(71)
    ring = _ring(len(frames), slot_cap=cap, batch_slots=256, depth=3)
    try:
        junk = rng.integers(0, 256, (len(frames), cap), dtype=np.uint8)
        ring.slots[:] = junk
        caps = []
        for i, f in enumerate(frames):
            ring.slots[i, offset:offset + len(f)] = np.frombuffer(f, np.uint8)
            caps.append(cap - offset)
        # FCS only: a capacity 2 bytes over the longest frame, which then does not fit
        capacity = cap - offset if flags != L.TX_FCS else max(len(f) for f in frames) + 2
        s0 = ring.stats()["zero_copy_frames"]
        sizes, status = ring.egress_packets([ring.slots[i] for i in range(len(frames))], [len(f) for f in frames],
                                            offset=offset, capacity=capacity, flags=flags)
        assert ring.stats()["zero_copy_frames"] - s0 == len(frames)
        bad = []
        for i, f in enumerate(frames):
            want, st = O.tx_checksum(f) if flags & L.TX_CHECKSUM else (f, 0)
            st2 = 0
            if flags & L.TX_FCS:
                want, st2 = O.fcs_append(want, capacity)
            got = ring.slots[i, offset:offset + int(sizes[i])].tobytes()
            if got != want or int(status[i]) != (st or st2):
                bad.append((i, len(f), int(sizes[i]), len(want), int(status[i]), st or st2))
            assert np.array_equal(ring.slots[i, :offset], junk[i, :offset])
            assert np.array_equal(ring.slots[i, offset + len(want):], junk[i, offset + len(want):]), i
        assert not bad, bad[:10]
        if flags == L.TX_FCS:
            assert (status == 6).sum() >= 1  # frames past the capacity stay unpadded
    finally:
        ring.close()
