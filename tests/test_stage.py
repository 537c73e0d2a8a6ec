"""The staged lane streams (lneto_amd/csrc/stage_kernel.hip)
and the round-5 dispatch behind the plain entries (dispatch.hpp, §3.10) on the
GPU against the C oracle (Go hash/crc32 IEEE restated; the arithmetic of
ethernet.CRC32, lneto ethernet/crc.go:19-21).

Product entries, each case run through both: "auto" = lnx_crc32_batch /
lnx_fcs_verify_batch (rows and staged kernels, each slice's kernel picked on
the device), "short" = the _ex forms with LNX_BATCH_SHORT_FRAMES (every slice
that fits goes to the staged kernel).  Cases: the Zipf mix, every length
0..700 at odd lead-ins, tiny and empty frames (the byte-serial halves), frames
longer than a stretch (the carry chain), jumbo and 3 MiB frames, tiny batches,
FCS verify with flipped bytes, offsets out of order, batches whose slices go
to different kernels, configs[3]'s whole 16 M-frame batch (offsets past 2^31),
and giant slices (a 2.2 GB frame among short ones: the byte pieces).

The round-4 research forms (stage_research.hip, liblneto_amd_research.so)
keep one parity test each.  The schedule's algebra is pinned on the host in
tests/test_stage_algebra.py."""
import ctypes
import time

import numpy as np
import pytest

MODES = ["auto", "short"]
# research forms (stage_research.hip): slicing-by-2 / 16-column Z_4 / slicing-by-8 fold, 766-frame blocks,
# deferred correction, patched boundary word (the product's fold), two chains per half, 190- / 254-frame
# blocks, offsets a block ahead, 510-frame blocks, 6 waves; verify form = var + 1
RESEARCH_VARS = [300, 302, 308, 310, 312, 314, 316, 318, 320, 322, 324, 326]


def _research():
    import lneto_amd as L
    f = L.research_lib().lnx__crc32_variant
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    return f


def _run(cuda, data, off, mode, verify=False):
    """Results of the product entry (mode "auto" / "short") or research variant (int)."""
    import torch
    import lneto_amd as L
    n = len(off) - 1
    d = data if isinstance(data, torch.Tensor) else torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(np.asarray(off).astype(np.int64)).to(cuda)
    if isinstance(mode, int):
        out = torch.full((max(n, 1),), -1, dtype=torch.int32, device=cuda)
        rc = _research()(mode + int(verify), d.data_ptr(), o.data_ptr(), n, out.data_ptr(),
                         torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)[:n]
        return got.view(np.uint8)[:n] if verify else got
    if verify:
        return L.fcs_verify_batch(d, o, short_frames=mode == "short").cpu().numpy()
    return L.crc32_batch(d, o, short_frames=mode == "short").cpu().numpy().view(np.uint32)


def _check(cuda, off, seed, name, mode):
    from lneto_amd import synth
    from oracle import oracle as O
    off = np.asarray(off, dtype=np.uint64)
    data = synth.bytes_np(int(off.max()) + 8, seed=seed)
    got = _run(cuda, data, off, mode)
    want = O.crc32_frames(data, off, threads=8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{name}: wrong at frames {bad[:8]} (lens {np.diff(off.astype(np.int64))[bad[:8]]}) of {len(off) - 1}"


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_stage_zipf(cuda, mode):
    from lneto_amd import synth
    for n, seed in ((1 << 16, 11), (1 << 20, 12), (300_001, 13)):
        _check(cuda, synth.offsets_from_lengths(synth.zipf_lengths(n, seed=seed)), seed, f"zipf {n}", mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_stage_all_lengths(cuda, mode):
    from lneto_amd import synth
    rng = np.random.default_rng(9)
    for lead in (0, 1, 2, 3, 5, 64, 127):
        lens = rng.permutation(np.arange(0, 701))
        off = np.concatenate([[0], synth.offsets_from_lengths(lens) + lead])
        _check(cuda, off, 100 + lead, f"lengths lead {lead}", mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_stage_tiny_and_empty(cuda, mode):
    """Several boundaries in one 64-byte half: the byte-serial path."""
    from lneto_amd import synth
    rng = np.random.default_rng(21)
    for trial in range(4):
        lens = rng.choice([0, 0, 1, 2, 3, 4, 5, 7, 9, 15, 16, 17, 33, 64, 200], size=20000 + 977 * trial)
        off = np.concatenate([[0], synth.offsets_from_lengths(lens) + trial * 37])
        _check(cuda, off, 200 + trial, f"tiny {trial}", mode)
    lens = np.concatenate([np.full(50000, 64), synth.zipf_lengths(50000, seed=5), np.full(3000, 1)])
    _check(cuda, synth.offsets_from_lengths(lens), 300, "mixed", mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_stage_long_frames(cuda, mode):
    """Frames longer than a stretch (the carry runs through stretches without
    a boundary), jumbo frames, a 3 MiB frame among short ones."""
    from lneto_amd import synth
    rng = np.random.default_rng(31)
    lens = rng.choice([9000, 1500, 64, 0, 100_000], size=3000)
    _check(cuda, synth.offsets_from_lengths(lens), 400, "long", mode)
    lens = np.array([60] * 500 + [3 << 20] + [60] * 500 + [1500] * 2000)
    _check(cuda, synth.offsets_from_lengths(lens), 401, "3 MiB", mode)
    _check(cuda, synth.offsets_from_lengths(np.full(20000, 9000)), 402, "jumbo", mode)
    _check(cuda, synth.offsets_from_lengths(np.full(100000, 1500)), 403, "mtu", mode)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_stage_small_batches(cuda, mode):
    from lneto_amd import synth
    rng = np.random.default_rng(41)
    for n in (1, 2, 3, 63, 64, 65, 381, 382, 383, 765, 1000):
        lens = rng.integers(0, 400, size=n)
        for lead in (0, 13, 127):
            _check(cuda, np.concatenate([[0], synth.offsets_from_lengths(lens) + lead]), n + lead, f"n {n} lead {lead}",
                   mode)


def _verify_case():
    """200 000 Zipf frames carrying their LE FCS; a third get one flipped
    byte; runts under 4 bytes fail."""
    from lneto_amd import synth
    from oracle import oracle as O
    lens = synth.zipf_lengths(200_000, seed=7)
    lens[::997] = 3
    off = synth.offsets_from_lengths(lens)
    data = synth.bytes_np(int(off[-1]) + 8, seed=8)
    for i in range(len(lens)):
        s, e = int(off[i]), int(off[i + 1])
        if e - s >= 4:
            data[e - 4:e] = np.frombuffer(int(O.c_crc32(data[s:e - 4].tobytes())).to_bytes(4, "little"), np.uint8)
    rng = np.random.default_rng(9)
    flip = rng.random(len(lens)) < 0.33
    for i in np.nonzero(flip)[0]:
        s, e = int(off[i]), int(off[i + 1])
        if e > s:
            data[s + int(rng.integers(0, e - s))] ^= 0x40
    want = np.array([int(int(off[i + 1]) - int(off[i]) >= 4 and O.c_crc32(data[int(off[i]):int(off[i + 1])].tobytes())
                         == 0x2144DF1C) for i in range(len(lens))], dtype=np.uint8)
    assert want.sum() > 100_000 and (want == 0).sum() > 50_000
    return data, off, want


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_stage_verify(cuda, mode):
    data, off, want = _verify_case()
    got = _run(cuda, data, off, mode, verify=True)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_offsets_out_of_order(cuda, mode):
    """Offsets outside the contract (an end below its start): such a frame is
    empty, the others are CRC32(bytes[off[i]:off[i+1]]) whichever kernel folds
    them (off = [0, 8, 4, 12]); in a long staged slice the block
    with the reversed pair is folded one lane per frame (ooo_block)."""
    from lneto_amd import synth
    _check(cuda, np.array([0, 8, 4, 12]), 70, "0 8 4 12", mode)
    off = synth.offsets_from_lengths(synth.zipf_lengths(100_000, seed=71)).astype(np.int64)
    for i in (5, 777, 40_001, 99_990):
        off[i] = off[i + 1] + 3  # frame i - 1 runs long, frame i is empty (end below start)
    _check(cuda, off.astype(np.uint64), 72, "zipf with reversed pairs", mode)


@pytest.mark.gpu
def test_gpu_dispatch_mixed_slices(cuda):
    """One batch whose slices go to different kernels under the default entry
    (uniform 1500 B, 256 B and 9000 B slices to the rows kernel; Zipf, 64 B and
    uniform-random slices to the staged one), every frame against the oracle."""
    from lneto_amd import synth
    rng = np.random.default_rng(81)
    parts = [np.full(300_000, 1500), synth.zipf_lengths(400_000, seed=82), np.full(200_000, 256),
             np.full(300_000, 64), np.full(20_000, 9000), rng.integers(64, 1500, 150_000), np.full(70_000, 1024)]
    lens = np.concatenate(parts)
    _check(cuda, np.concatenate([[0], synth.offsets_from_lengths(lens) + 3]), 83, "mixed slices", "auto")


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_configs3_full_batch(cuda, mode):
    """configs[3] whole: 16 M Zipf frames, 4.13 GB, offsets past 2^31, frame by frame against the C oracle (16 threads, Go's amd64 path)."""
    import torch
    from lneto_amd import synth
    from oracle import oracle as O
    off = synth.offsets_from_lengths(synth.zipf_lengths(1 << 24))
    assert int(off[-1]) > (3 << 30)  # 4.13 GB: offsets past 2^31, up to 0.96 x 2^32
    d = synth.bytes_torch(int(off[-1]), cuda)
    got = _run(cuda, d, off, mode)
    want = O.crc32_frames(d.cpu().numpy(), off, threads=16, amd64=O.has_clmul())
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]
    del d
    torch.cuda.empty_cache()


def _giant_batch(lead, giant, nshort, at, seed=91):
    """nshort short Zipf frames with one frame of `giant` bytes at index `at`,
    the first starting `lead` bytes into the buffer."""
    from lneto_amd import synth
    lens = synth.zipf_lengths(nshort, seed=seed).astype(np.int64)
    lens = np.insert(lens, at, giant)
    return (synth.offsets_from_lengths(lens) + lead).astype(np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_giant_frame(cuda, mode):
    """a 2.2 GB frame among 2000 short ones with a nonzero
    lead-in.  Its slice does not fit 31-bit offsets: every workgroup of the
    staged launch folds 16 KiB pieces of it and joins the parts (giant_pieces).
    CRC and FCS verify against the C oracle, and the launch time."""
    import torch
    from lneto_amd import synth
    from oracle import oracle as O
    import lneto_amd as L
    giant = 2_200_000_000
    off = _giant_batch(5, giant, 2000, 1234)
    d = synth.bytes_torch(int(off[-1]) + 8, cuda, seed=92)
    host = d.cpu().numpy()
    want = O.crc32_frames(host, off, threads=16, amd64=O.has_clmul())
    got = _run(cuda, d, off, mode)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]
    # the giant frame carries its FCS: it verifies, a flipped byte in its middle fails it
    s, e = int(off[1234]), int(off[1235])
    d[e - 4:e] = torch.tensor(list(int(O.crc32_frames(host, np.array([s, e - 4], np.uint64), amd64=O.has_clmul())[0])
                                   .to_bytes(4, "little")), dtype=torch.uint8, device=cuda)
    ok = _run(cuda, d, off, mode, verify=True)
    assert ok[1234] == 1 and (ok[:1234] == ((want[:1234] == 0x2144DF1C) & (np.diff(off.astype(np.int64))[:1234] >= 4))).all()
    d[s + giant // 2 + 7] ^= 1
    ok = _run(cuda, d, off, mode, verify=True)
    assert ok[1234] == 0
    # the launch: HIP events around the entry on the current stream
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    c = torch.empty(len(off) - 1, dtype=torch.int32, device=cuda)
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        L.crc32_batch(d, o, out=c, short_frames=mode == "short")
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    print(f"giant frame {giant} B among 2000: {ms:.3f} ms ({int(off[-1]) / ms / 1e6:.0f} GB/s)")
    assert ms < 50.0, ts
    del d, host
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_gpu_giant_slices_edges(cuda):
    """Giant slices with frames ending exactly on 16 KiB piece bounds, empty
    frames at a giant slice's start and end, two giant frames in one slice and
    a giant slice beside ordinary ones (3 000 frames: 47 slices)."""
    import torch
    from lneto_amd import synth
    from oracle import oracle as O
    P = 16384
    rng = np.random.default_rng(93)
    lens = list(rng.integers(0, 3000, 1350))  # (the group below: frames 1350-1362, all in slice 21 = [1344, 1408))
    lens += [0, 0, P - 100, P, 3 * P, 1, 1_150_000_000, 0, 7, 1_100_000_000 + 13, 2 * P, 0, 0]
    lens += list(rng.integers(0, 3000, 1637))
    off = np.concatenate([[0], synth.offsets_from_lengths(np.array(lens)) + 100]).astype(np.uint64)
    d = synth.bytes_torch(int(off[-1]) + 8, cuda, seed=94)
    want = O.crc32_frames(d.cpu().numpy(), off, threads=16, amd64=O.has_clmul())
    for mode in MODES:
        got = _run(cuda, d, off, mode)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, (mode, bad[:10])
    del d
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_gpu_short_frames_entry_host(cuda):
    """lnx_crc32_batch_host (the plain entry's dispatch behind pinned copies)
    against the oracle."""
    import lneto_amd as L
    from lneto_amd import synth
    from oracle import oracle as O
    rng = np.random.default_rng(51)
    cases = [synth.offsets_from_lengths(synth.zipf_lengths(300_001, seed=3)),
             np.concatenate([[0], synth.offsets_from_lengths(rng.permutation(np.arange(0, 701))) + 5]),
             np.array([0, 8, 4, 12])]
    for k, off in enumerate(cases):
        off = np.asarray(off, dtype=np.uint64)
        data = synth.bytes_np(int(off.max()) + 8, seed=60 + k)
        want = O.crc32_frames(data, off, threads=8)
        host = np.zeros(len(off) - 1, dtype=np.uint32)
        assert L.lib.lnx_crc32_batch_host(data.ctypes.data, data.size, off.ctypes.data, len(off) - 1,
                                          host.ctypes.data, 0) == 0
        assert (host == want).all(), k


@pytest.mark.gpu
@pytest.mark.parametrize("var", RESEARCH_VARS)
def test_gpu_research_stage_form(cuda, var):
    """One parity test per round-4 research form: the Zipf mix, all lengths at
    a lead-in, tiny frames, and its FCS verify form."""
    from lneto_amd import synth
    _check(cuda, synth.offsets_from_lengths(synth.zipf_lengths(1 << 16, seed=11)), 11, "zipf", var)
    rng = np.random.default_rng(9)
    _check(cuda, np.concatenate([[0], synth.offsets_from_lengths(rng.permutation(np.arange(0, 701))) + 5]), 105,
           "lengths", var)
    _check(cuda, synth.offsets_from_lengths(rng.choice([0, 1, 3, 17, 64, 65, 3000], size=20000)), 106, "tiny", var)
    data, off, want = _verify_case()
    got = _run(cuda, data, off, var, verify=True)
    assert (got == want).all(), np.nonzero(got != want)[0][:10]


def _place(lens, at, big):
    """lens with the frames of `big` (bytes) written over indices `at`."""
    lens = np.asarray(lens, dtype=np.int64).copy()
    for i, b in zip(at, big):
        lens[i] = b
    return lens


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_ooo_block_long_frames(cuda, mode):
    """VERDICT r5 "Next" 3: a reversed pair in the same staged block as a
    3 MiB and a 40 MiB frame (and ~230 frames over the 16 KiB lane limit).
    ooo_block folds frames up to 16 KiB one lane each and every longer one with
    the whole wave (wave_fold): every frame gets its true CRC, through the plain
    and the short-frames entries.  The background frames average 30 KB, so the
    slice (320 frames) is not giant by the skew rule and stays staged."""
    import torch
    from lneto_amd import synth
    from oracle import oracle as O
    rng = np.random.default_rng(77)
    n = 80_000
    lens = _place(rng.integers(0, 60_000, n), (3250, 3300), (3 << 20, 40 << 20))
    off = (synth.offsets_from_lengths(lens) + 5).astype(np.int64)
    off[3400] = off[3401] + 3  # frame 3399 runs long, frame 3400 is empty (end below start)
    off = off.astype(np.uint64)
    d = synth.bytes_torch(int(off.max()) + 8, cuda, seed=78)
    want = O.crc32_frames(d.cpu().numpy(), off, threads=16, amd64=O.has_clmul())
    got = _run(cuda, d, off, mode)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]
    assert want[3400] == 0 and want[3300] != 0
    del d
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_giant_slice_out_of_order(cuda, mode):
    """giant slices whose offsets decrease somewhere.  64
    frames of 1 MiB (giant by mean) with one decreasing offset, and a 40 MiB
    and a 3 MiB frame with a reversed pair among Zipf frames (giant by the
    skew rule): the workgroups find the decreasing pair, give that slice no
    pieces and fold its frames one per wave, so every frame gets its true CRC
    (the empty one 0), nothing faults, and a correct giant call on the same
    stream afterwards is still exact (the pieces' scratch stayed clean)."""
    import torch
    from lneto_amd import synth
    from oracle import oracle as O
    cases = []
    off = synth.offsets_from_lengths(np.full(64, 1 << 20)).astype(np.int64)
    off[20] = off[21] - (3 << 20)  # 18 MiB: frame 19 = [19, 18) MiB is empty, frame 20 = [18, 21) MiB overlaps 18
    cases.append(off.astype(np.uint64))
    lens = _place(synth.zipf_lengths(100_000, seed=79), (40_500, 40_600), (40 << 20, 3 << 20))
    off = (synth.offsets_from_lengths(lens) + 3).astype(np.int64)
    off[40_700] = off[40_701] + 1
    cases.append(off.astype(np.uint64))
    good = synth.offsets_from_lengths(np.full(64, (1 << 20) + 3))  # in order, giant by mean
    for k, off in enumerate(cases):
        d = synth.bytes_torch(int(off.max()) + 8, cuda, seed=80 + k)
        want = O.crc32_frames(d.cpu().numpy(), off, threads=16, amd64=O.has_clmul())
        for verify in (False, True):
            got = _run(cuda, d, off, mode, verify=verify)
            w = ((want == 0x2144DF1C) & (np.diff(off.astype(np.int64)) >= 4)).astype(np.uint8) if verify else want
            bad = np.nonzero(got != w)[0]
            assert bad.size == 0, (k, verify, bad[:10])
        d2 = synth.bytes_torch(int(good[-1]) + 8, cuda, seed=90 + k)
        want2 = O.crc32_frames(d2.cpu().numpy(), good, threads=16, amd64=O.has_clmul())
        assert (_run(cuda, d2, good, mode) == want2).all(), k
        del d, d2
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("mode", MODES)
def test_gpu_large_frames_among_zipf(cuda, mode):
    """VERDICT r5 "Next" 6 (the large-frame cliff): a 1.9 GB and a 300 MB frame
    among configs[3]'s 16 M Zipf frames.  Neither slice is giant by span or by
    mean; the skew rule (>= 16 MiB at 8x the batch mean, dispatch.hpp) sends
    both to the giant pieces instead of one wave each.  Every frame against
    the C oracle, and the launch takes <= 10 ms."""
    import torch
    import lneto_amd as L
    from lneto_amd import synth
    from oracle import oracle as O
    n = 1 << 24
    lens = _place(synth.zipf_lengths(n), (5_000_000, 12_345_678), (1_900_000_000, 300_000_000))
    off = synth.offsets_from_lengths(lens).astype(np.uint64)
    d = synth.bytes_torch(int(off[-1]) + 8, cuda, seed=95)
    want = O.crc32_frames(d.cpu().numpy(), off, threads=16, amd64=O.has_clmul())
    got = _run(cuda, d, off, mode)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    c = torch.empty(n, dtype=torch.int32, device=cuda)
    ts = []
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        L.crc32_batch(d, o, out=c, short_frames=mode == "short")
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b))
    ms = float(np.median(ts))
    print(f"1.9 GB + 300 MB frames among 16 M Zipf ({int(off[-1]) / 1e9:.2f} GB): {ms:.3f} ms")
    assert ms <= 10.0, ts
    del d, o, c
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_gpu_frame_past_4gib(cuda):
    """One 4.5 GB frame (positions inside it past 2^32) between short ones:
    the giant pieces' 64-bit positions and Z_d shifts for d up to 2^33 (the
    HBM image's nibble tables m = 31..39), CRC through both entries against the
    C oracle, then its FCS appended verifies and a flipped byte past 2^32 fails it."""
    import torch
    from lneto_amd import synth
    from oracle import oracle as O
    big = 4_500_000_000
    lens = np.array([100, 7, big, 1500, 0, 64], dtype=np.int64)
    off = (synth.offsets_from_lengths(lens) + 9).astype(np.uint64)
    d = synth.bytes_torch(int(off[-1]) + 8, cuda, seed=97)
    host = d.cpu().numpy()
    want = O.crc32_frames(host, off, threads=8, amd64=O.has_clmul())
    for mode in MODES:
        got = _run(cuda, d, off, mode)
        assert (got == want).all(), (mode, got, want)
    s, e = int(off[2]), int(off[3])
    fcs = int(O.crc32_frames(host, np.array([s, e - 4], np.uint64), amd64=O.has_clmul())[0])
    del host
    d[e - 4:e] = torch.tensor(list(fcs.to_bytes(4, "little")), dtype=torch.uint8, device=cuda)
    for mode in MODES:
        assert _run(cuda, d, off, mode, verify=True)[2] == 1, mode
    d[s + (1 << 32) + 12345] ^= 4
    for mode in MODES:
        assert _run(cuda, d, off, mode, verify=True)[2] == 0, mode
    del d
    torch.cuda.empty_cache()
