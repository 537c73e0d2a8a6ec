"""The transmit tail in one read (lnx_tx_finish_batch, tx_finish_kernel in
lneto_amd/csrc/rx_verify_kernel.hip) on device-resident
frames against the oracle: the checksum step (oracle.tx_checksum: encapsulate4
/ encapsulate6 and the ICMP clients, internet/stack-ip4.go:202-228,
internet/stack-ip6.go:167-181) then the padding and FCS (oracle.fcs_append,
internet/stack-ethernet.go:200-214), with the CRC taken over the frame as
loaded and corrected for the fields the step writes.  Every protocol the
step knows, runts, frames too short, ErrShortBuffer, slots in shuffled order
and at odd addresses; and the same bytes as lnx_tx_checksum_batch followed by
lnx_fcs_append_batch."""
import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu

SLOT = 2048


def _layout(frames, lead, order, rng):
    """Frames in SLOT-byte slots (frame k in slot order[k], `lead` bytes in),
    random bytes around them; returns the buffer, the starts and the lengths."""
    buf = rng.integers(0, 256, SLOT * len(frames) + 64, dtype=np.uint8)
    starts = np.array([SLOT * int(order[k]) + lead for k in range(len(frames))], dtype=np.int64)
    for k, f in enumerate(frames):
        buf[starts[k]:starts[k] + len(f)] = np.frombuffer(f, np.uint8)
    return buf, starts, np.array([len(f) for f in frames], dtype=np.int32)


def _want(f, flags, capacity):
    want, st = O.tx_checksum(f) if flags & 1 else (f, 0)
    st2 = 0
    if flags & 2:
        want, st2 = O.fcs_append(want, capacity)
    return want, (st or st2)


@pytest.mark.parametrize("flags", [3, 2, 1])
@pytest.mark.parametrize("lead", [0, 5])
def test_tx_finish_matches_oracle(cuda, flags, lead):
    import torch
    import lneto_amd as L
    from tests.test_tx_checksum import tx_frames
    rng = np.random.default_rng(100 + 10 * flags + lead)
    frames = [f for f in tx_frames(seed=200 + lead, count=2100) if len(f) <= 1900]
    order = rng.permutation(len(frames))
    buf, starts, lens = _layout(frames, lead, order, rng)
    before = buf.copy()
    capacity = SLOT - lead - 8 if flags != 2 else max(len(f) for f in frames) + 2  # FCS only: the longest does not fit
    d = torch.from_numpy(buf).to(cuda)
    ds, dl = torch.from_numpy(starts).to(cuda), torch.from_numpy(lens).to(cuda)
    status = L.tx_finish_batch(d, ds, dl, capacity, flags=flags).cpu().numpy()
    out, newl = d.cpu().numpy(), dl.cpu().numpy()
    bad = []
    for k, f in enumerate(frames):
        want, st = _want(f, flags, capacity)
        s0 = int(starts[k])
        got = out[s0:s0 + int(newl[k])].tobytes()
        if got != want or int(status[k]) != st:
            bad.append((k, len(f), int(newl[k]), len(want), int(status[k]), st))
        # bytes outside the finished frame are untouched
        assert np.array_equal(out[s0 - lead:s0], before[s0 - lead:s0])
        assert np.array_equal(out[s0 + len(want):s0 - lead + SLOT], before[s0 + len(want):s0 - lead + SLOT]), k
    assert not bad, bad[:10]
    if flags == 2:
        assert (status == 6).sum() >= 1


def test_tx_finish_equals_the_two_calls(cuda):
    """4096 frames of every kind: lnx_tx_finish_batch leaves the same bytes,
    lengths and statuses as lnx_tx_checksum_batch then lnx_fcs_append_batch
    (whose slots are in increasing address order)."""
    import torch
    import lneto_amd as L
    from tests.test_tx_checksum import tx_frames
    rng = np.random.default_rng(7)
    frames = [f for f in tx_frames(seed=300, count=4400) if len(f) <= 1500][:4096]
    buf, starts, lens = _layout(frames, 2, np.arange(len(frames)), rng)
    cap = 1536
    a = torch.from_numpy(buf.copy()).to(cuda)
    b = torch.from_numpy(buf.copy()).to(cuda)
    ds = torch.from_numpy(starts).to(cuda)
    la, lb = torch.from_numpy(lens.copy()).to(cuda), torch.from_numpy(lens.copy()).to(cuda)
    st = L.tx_finish_batch(a, ds, la, cap, flags=3)
    c1 = L.tx_checksum_batch(b, ds, lb)
    c2 = L.fcs_append_batch(b, ds, lb, cap)
    assert torch.equal(a, b) and torch.equal(la, lb)
    assert torch.equal(st, torch.where(c1 != 0, c1, c2))


def test_tx_finish_mtu_round_trip(cuda):
    """64 Ki x 1496-byte UDP/IPv4 frames with garbled sums finished in place:
    every frame with its FCS folds to the CRC-32 residue and equals the valid
    frame it came from (tests/test_rx_verify.py _udp_rows)."""
    import torch
    import lneto_amd as L
    from tests.test_rx_verify import _udp_rows
    n, flen = 1 << 16, 1500
    rows = _udp_rows(n, flen)  # valid frames; their sums, lengths and FCS are then garbled
    body = rows[:, :flen - 4].copy()
    body[:, 24:26] = 0x5A
    body[:, 40:42] = 0xA5
    slots = np.zeros((n, 1536), dtype=np.uint8)
    slots[:, :flen - 4] = body
    d = torch.from_numpy(slots.reshape(-1)).to(cuda)
    ds = torch.arange(n, dtype=torch.int64, device=cuda) * 1536
    dl = torch.full((n,), flen - 4, dtype=torch.int32, device=cuda)
    st = L.tx_finish_batch(d, ds, dl, 1536, flags=3)
    assert int(st.max()) == 0 and bool((dl == flen).all())
    # every frame with its FCS folds to the residue, and equals the valid frame it came from
    seg = torch.full((n,), flen, dtype=torch.int32, device=cuda)
    crc = L.crc32_segments(d, ds, seg).cpu().numpy().view(np.uint32)
    assert (crc == O.CRC32_RESIDUE).all()
    assert np.array_equal(d.cpu().numpy().reshape(n, 1536)[:, :flen], rows)


def test_tx_finish_equals_the_two_calls_at_scale(cuda):
    """256 Ki frames (the generated ones of every kind, tiled in random order,
    at random leads in 2048-B slots taken in shuffled order): the same bytes, lengths and statuses as
    lnx_tx_checksum_batch then lnx_fcs_append_batch, over 5462 groups."""
    import torch
    import lneto_amd as L
    from tests.test_tx_checksum import tx_frames
    rng = np.random.default_rng(11)
    base = [f for f in tx_frames(seed=400, count=4400) if len(f) <= 1900]
    n = 1 << 18
    pick = rng.integers(0, len(base), n)
    lead = rng.integers(0, 16, n)
    # slots in shuffled order (round 5 had to keep them sorted: out-of-order
    # starts faulted the append entry, r6p; its workgroups now fold such a
    # slice frame by frame)
    buf = rng.integers(0, 256, SLOT * n + 64, dtype=np.uint8)
    starts = (rng.permutation(n).astype(np.int64) * SLOT + lead).astype(np.int64)
    lens = np.array([len(base[i]) for i in pick], dtype=np.int32)
    arrs = [np.frombuffer(f, np.uint8) for f in base]
    for k in range(n):
        s0 = int(starts[k])
        buf[s0:s0 + int(lens[k])] = arrs[pick[k]]
    cap = int(lens.max()) + 2  # the longest frames have no room for the FCS: status 6
    a = torch.from_numpy(buf).to(cuda)
    b = a.clone()
    ds = torch.from_numpy(starts).to(cuda)
    la, lb = torch.from_numpy(lens).to(cuda), torch.from_numpy(lens.copy()).to(cuda)
    st = L.tx_finish_batch(a, ds, la, cap, flags=3)
    c1 = L.tx_checksum_batch(b, ds, lb)
    c2 = L.fcs_append_batch(b, ds, lb, cap)
    assert torch.equal(la, lb)
    assert torch.equal(st, torch.where(c1 != 0, c1, c2))
    assert torch.equal(a, b)
    assert int((st == 6).sum()) >= 1 and int((st == 0).sum()) > n // 4


@pytest.mark.parametrize("flags", [3, 2])
def test_tx_finish_exact_fit_at_the_buffer_end(cuda, flags):
    """Frames whose padded length + FCS is exactly their capacity, and one byte
    more (status 6, left unpadded), each in a buffer that ends exactly where
    its capacity does (a load or store past it would fault): lengths 0..80 and
    MTU, the capacity from the frame's own needs."""
    import torch
    import lneto_amd as L
    from tests.test_tx_checksum import tx_frames
    rng = np.random.default_rng(21)
    frames = [f for f in tx_frames(seed=500, count=300) if len(f) <= 1500]
    frames += [bytes(rng.integers(0, 256, n, dtype=np.uint8)) for n in (0, 1, 13, 14, 33, 59, 60, 61, 80)]
    for f in frames:
        want_fit, _ = _want(f, flags, 1 << 20)
        fit = len(want_fit) if flags & 2 else len(f)
        for cap, slack in ((fit, 0), (max(fit - 1, len(f)), 1)):
            buf = np.zeros(cap, dtype=np.uint8)
            buf[:len(f)] = np.frombuffer(f, np.uint8)
            d = torch.from_numpy(buf).to(cuda)
            ds = torch.zeros(1, dtype=torch.int64, device=cuda)
            dl = torch.tensor([len(f)], dtype=torch.int32, device=cuda)
            st = int(L.tx_finish_batch(d, ds, dl, cap, flags=flags).cpu()[0])
            want, wst = _want(f, flags, cap)
            got = d.cpu().numpy()[:int(dl.cpu()[0])].tobytes()
            assert (got, st) == (want, wst), (len(f), cap, slack, st, wst)


@pytest.mark.parametrize("n", [1, 3, 5, 61, 64, 65, 1000, 3073])
def test_tx_finish_batch_sizes(cuda, n):
    """Batches of every shape the launcher's group size takes (4 to 64 frames a
    group, the last group part-full): the bytes, lengths and statuses of the two
    calls."""
    import torch
    import lneto_amd as L
    from tests.test_tx_checksum import tx_frames
    rng = np.random.default_rng(n)
    base = [f for f in tx_frames(seed=600, count=700) if len(f) <= 1500]
    frames = [base[i % len(base)] for i in range(n)]
    buf, starts, lens = _layout(frames, 3, np.arange(n), rng)
    cap = 1536
    a = torch.from_numpy(buf.copy()).to(cuda)
    b = torch.from_numpy(buf.copy()).to(cuda)
    ds = torch.from_numpy(starts).to(cuda)
    la, lb = torch.from_numpy(lens.copy()).to(cuda), torch.from_numpy(lens.copy()).to(cuda)
    st = L.tx_finish_batch(a, ds, la, cap, flags=3)
    c1 = L.tx_checksum_batch(b, ds, lb)
    c2 = L.fcs_append_batch(b, ds, lb, cap)
    assert torch.equal(a, b) and torch.equal(la, lb)
    assert torch.equal(st, torch.where(c1 != 0, c1, c2))
