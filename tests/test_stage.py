"""Staged lane streams (lneto_amd/csrc/stage_kernel.hip) on the
GPU against the C oracle (Go hash/crc32 IEEE restated; the arithmetic of
ethernet.CRC32, lneto ethernet/crc.go:19-21): the Zipf mix, every length
0..700 at odd lead-ins (variants 300 / 302: the two folds), tiny and empty frames (the byte-serial halves),
frames longer than a stretch (the carry chain), jumbo and gigantic frames,
tiny batches, and FCS verify (variants 301 / 303) with one flipped byte per frame
for a third of the frames.  The schedule's algebra is pinned on the host in
tests/test_stage_algebra.py."""
import ctypes

import numpy as np
import pytest


CRC_VARS = [300, 302, 308, 310, 312, 314, 316, 318, 320, 322, 324, 326]  # slicing-by-2 / 16-column Z_4 / slicing-by-8 fold, 766-frame blocks, deferred correction, patched boundary word, two chains per half, 190- / 254-frame blocks, offsets a block ahead, 510-frame blocks, 6 waves


def _lib():
    import lneto_amd as L
    f = L.research_lib().lnx__crc32_variant
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
    return f


def _run(cuda, data, off, var=300):
    import torch
    n = len(off) - 1
    d = torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    out = torch.full((max(n, 1),), -1, dtype=torch.int32, device=cuda)
    rc = _lib()(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(), torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)[:n]
    return got if var % 2 == 0 else got.view(np.uint8)[:n]


def _check(cuda, off, seed, name, var=300):
    from lneto_amd import synth
    from oracle import oracle as O
    off = np.asarray(off, dtype=np.uint64)
    data = synth.bytes_np(int(off[-1]) + 8, seed=seed)
    got = _run(cuda, data, off, var)
    want = O.crc32_frames(data, off, threads=8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{name}: wrong at frames {bad[:8]} (lens {np.diff(off)[bad[:8]]}) of {len(off) - 1}"


@pytest.mark.gpu
@pytest.mark.parametrize("var", CRC_VARS)
def test_gpu_stage_zipf(cuda, var):
    from lneto_amd import synth
    for n, seed in ((1 << 16, 11), (1 << 20, 12), (300_001, 13)):
        _check(cuda, synth.offsets_from_lengths(synth.zipf_lengths(n, seed=seed)), seed, f"zipf {n}", var)


@pytest.mark.gpu
@pytest.mark.parametrize("var", CRC_VARS)
def test_gpu_stage_all_lengths(cuda, var):
    from lneto_amd import synth
    rng = np.random.default_rng(9)
    for lead in (0, 1, 2, 3, 5, 64, 127):
        lens = rng.permutation(np.arange(0, 701))
        off = np.concatenate([[0], synth.offsets_from_lengths(lens) + lead])
        _check(cuda, off, 100 + lead, f"lengths lead {lead}", var)


@pytest.mark.gpu
@pytest.mark.parametrize("var", CRC_VARS)
def test_gpu_stage_tiny_and_empty(cuda, var):
    """Several boundaries in one 64-byte half: the byte-serial path."""
    from lneto_amd import synth
    rng = np.random.default_rng(21)
    for trial in range(4):
        lens = rng.choice([0, 0, 1, 2, 3, 4, 5, 7, 9, 15, 16, 17, 33, 64, 200], size=20000 + 977 * trial)
        off = np.concatenate([[0], synth.offsets_from_lengths(lens) + trial * 37])
        _check(cuda, off, 200 + trial, f"tiny {trial}", var)
    lens = np.concatenate([np.full(50000, 64), synth.zipf_lengths(50000, seed=5), np.full(3000, 1)])
    _check(cuda, synth.offsets_from_lengths(lens), 300, "mixed", var)


@pytest.mark.gpu
@pytest.mark.parametrize("var", CRC_VARS)
def test_gpu_stage_long_frames(cuda, var):
    """Frames longer than a stretch (the carry runs through stretches without
    a boundary), jumbo frames, a 3 MiB frame among short ones."""
    from lneto_amd import synth
    rng = np.random.default_rng(31)
    lens = rng.choice([9000, 1500, 64, 0, 100_000], size=3000)
    _check(cuda, synth.offsets_from_lengths(lens), 400, "long", var)
    lens = np.array([60] * 500 + [3 << 20] + [60] * 500 + [1500] * 2000)
    _check(cuda, synth.offsets_from_lengths(lens), 401, "3 MiB", var)
    _check(cuda, synth.offsets_from_lengths(np.full(20000, 9000)), 402, "jumbo", var)
    _check(cuda, synth.offsets_from_lengths(np.full(100000, 1500)), 403, "mtu", var)


@pytest.mark.gpu
@pytest.mark.parametrize("var", CRC_VARS)
def test_gpu_stage_small_batches(cuda, var):
    from lneto_amd import synth
    rng = np.random.default_rng(41)
    for n in (1, 2, 3, 63, 64, 65, 381, 382, 383, 765, 1000):
        lens = rng.integers(0, 400, size=n)
        for lead in (0, 13, 127):
            _check(cuda, np.concatenate([[0], synth.offsets_from_lengths(lens) + lead]), n + lead, f"n {n} lead {lead}", var)


@pytest.mark.gpu
@pytest.mark.parametrize("var", [301, 303, 309, 311, 313, 315, 317, 319, 321, 323, 325, 327])
def test_gpu_stage_verify(cuda, var):
    """Variant 301: FCS verify (residue) over frames carrying their LE FCS;
    a third get one flipped byte; runts under 4 bytes fail."""
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
    got = _run(cuda, data, off, var=var)
    want = np.array([int(int(off[i + 1]) - int(off[i]) >= 4 and O.c_crc32(data[int(off[i]):int(off[i + 1])].tobytes())
                         == 0x2144DF1C) for i in range(len(lens))], dtype=np.uint8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]
    assert want.sum() > 100_000 and (want == 0).sum() > 50_000


@pytest.mark.gpu
def test_gpu_short_frames_entry(cuda):
    """The product entry (lnx_crc32_batch_ex / lnx_fcs_verify_batch_ex with
    LNX_BATCH_SHORT_FRAMES, and lnx_crc32_batch_host, which picks the staged
    kernel itself for a short mix) against the oracle."""
    import torch
    import lneto_amd as L
    from lneto_amd import synth
    from oracle import oracle as O
    rng = np.random.default_rng(51)
    cases = [synth.offsets_from_lengths(synth.zipf_lengths(300_001, seed=3)),
             np.concatenate([[0], synth.offsets_from_lengths(rng.permutation(np.arange(0, 701))) + 5]),
             np.concatenate([[0], synth.offsets_from_lengths(rng.choice([0, 1, 3, 17, 64, 65], size=30000)) + 1])]
    for k, off in enumerate(cases):
        off = np.asarray(off, dtype=np.int64)
        data = synth.bytes_np(int(off[-1]) + 8, seed=60 + k)
        want = O.crc32_frames(data, off.astype(np.uint64), threads=8)
        d = torch.from_numpy(data).to(cuda)
        o = torch.from_numpy(off).to(cuda)
        got = L.crc32_batch(d, o, short_frames=True).cpu().numpy().view(np.uint32)
        assert (got == want).all(), (k, np.nonzero(got != want)[0][:8])
        ok = L.fcs_verify_batch(d, o, short_frames=True).cpu().numpy()
        lens = np.diff(off)
        assert (ok == ((want == 0x2144DF1C) & (lens >= 4))).all(), k
        host = np.zeros(len(off) - 1, dtype=np.uint32)
        assert L.lib.lnx_crc32_batch_host(data.ctypes.data, data.size, off.astype(np.uint64).ctypes.data,
                                          len(off) - 1, host.ctypes.data, 0) == 0
        assert (host == want).all(), k
