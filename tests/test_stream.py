"""Streaming rows (lneto_amd/csrc/stream_rows.hpp) and lane
streams (lneto_amd/csrc/stream_lanes.hpp, §3.8).

CPU: the schedule's algebra, restated in tests/stream_algebra.py, equals
zlib's CRC-32 (Go hash/crc32 IEEE, the arithmetic of ethernet/crc.go:19-21) on
frames of every small length, empty frames and frames inside one 16-byte lane
piece (its slow path); the lane streams' algebra likewise, with several
frames inside one superstep.  GPU: the kernel (profiling variants 150 / 153:
the product dispatch with 8- / 4-lane streaming rows for the narrow rows'
workgroups; 160: with lane streams) is bit-exact
against the C oracle on the Zipf mix, every length 0..700, runs of tiny and
empty frames, and workgroup slices ending at every line offset."""
import ctypes
import random
import zlib

import numpy as np
import pytest

from tests import stream_algebra as SA


def test_stream_algebra_matches_zlib():
    rnd = random.Random(7)
    for _ in range(200):
        lens = [rnd.choice([0, 1, 2, 3, 4, 5, 7, 12, 15, 16, 17, 31, 60, 63, 64, 65, 100, 127, 128, 129, 250, 1500])
                for _ in range(rnd.randint(1, 10))]
        frames = [bytes(rnd.getrandbits(8) for _ in range(n)) for n in lens]
        SA.check(frames, lead=rnd.randint(0, 300), RL=4)
        SA.check(frames, lead=rnd.randint(0, 300), RL=8)


def test_lane_stream_algebra_matches_zlib():
    rnd = random.Random(8)
    for _ in range(200):
        lens = [rnd.choice([0, 1, 2, 3, 4, 5, 7, 12, 15, 16, 17, 31, 60, 63, 64, 65, 100, 127, 128, 129, 250, 1500])
                for _ in range(rnd.randint(1, 10))]
        frames = [bytes(rnd.getrandbits(8) for _ in range(n)) for n in lens]
        SA.check_lanes(frames, lead=rnd.randint(0, 300), SB=64)
        SA.check_lanes(frames, lead=rnd.randint(0, 300), SB=16)


def test_lane_stream_operators():
    # the reset identity: Z_{64-4k}(e) ^ Z_{64-cb}(~0) == Z_{64-cb}(Z_c(e) ^ ~0), cb = 4k + c
    rnd = random.Random(4)
    for _ in range(50):
        e = rnd.getrandbits(32)
        k, c = rnd.randrange(16), rnd.randrange(4)
        cb = 4 * k + c
        assert SA.Z(64 - 4 * k, e) ^ SA.Z(64 - cb, 0xFFFFFFFF) == SA.Z(64 - cb, SA.Z(c, e) ^ 0xFFFFFFFF)


def test_stream_algebra_operators():
    # the injection identity the kernel relies on: Z_{128-4k}(O) ^ Z_d(~0) == Z_d(~Z_c(O)), d = 128 - 4k - c
    rnd = random.Random(3)
    for _ in range(50):
        O = rnd.getrandbits(32)
        k, c = rnd.randrange(4), rnd.randrange(4)
        d = 128 - 4 * k - c
        assert SA.Z(128 - 4 * k, O) ^ SA.Z(d, 0xFFFFFFFF) == SA.Z(d, SA.Z(c, O) ^ 0xFFFFFFFF)
    assert SA.Zt(4, 0x12345678) == SA.Z(4, 0x12345678)
    assert zlib.crc32(b"123456789") == 0xCBF43926


def _lib():
    import lneto_amd as L
    L.research_lib().lnx__crc32_variant.restype = ctypes.c_int
    L.research_lib().lnx__crc32_variant.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                         ctypes.c_void_p, ctypes.c_void_p]
    return L


def _run(cuda, var, data, off):
    import torch
    L = _lib()
    n = len(off) - 1
    d = torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    out = torch.empty(max(n, 1), dtype=torch.int32, device=cuda)
    rc = L.research_lib().lnx__crc32_variant(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)[:n]


VARS = [150, 153, 160, 164, 165]  # streaming rows of 8 lanes (128-byte row steps), of 4 lanes (64-byte), lane streams (164: reset in the fold)


def _check(cuda, off, seed, name, var):
    from lneto_amd import synth
    from oracle import oracle as O
    data = synth.bytes_np(int(off[-1]) + 8, seed=seed)
    got = _run(cuda, var, data, off)
    want = O.crc32_frames(data, off, threads=8)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"{name} (variant {var}): wrong at frames {bad[:8]} (lens {np.diff(off)[bad[:8]]}) of {len(off) - 1}"


@pytest.mark.gpu
@pytest.mark.parametrize("var", VARS)
def test_gpu_stream_zipf(cuda, var):
    from lneto_amd import synth
    for n, seed in ((1 << 16, 11), (1 << 20, 12), (300_001, 13)):
        _check(cuda, synth.offsets_from_lengths(synth.zipf_lengths(n, seed=seed)), seed, f"zipf {n}", var)


@pytest.mark.gpu
@pytest.mark.parametrize("var", VARS)
def test_gpu_stream_all_lengths(cuda, var):
    from lneto_amd import synth
    rng = np.random.default_rng(9)
    for lead in (0, 1, 2, 3, 5, 64, 127):
        lens = rng.permutation(np.arange(0, 701))
        off = (synth.offsets_from_lengths(lens) + lead).astype(np.uint64)
        off = np.concatenate([[0], off]).astype(np.uint64)
        _check(cuda, off, 100 + lead, f"lengths lead {lead}", var)


@pytest.mark.gpu
@pytest.mark.parametrize("var", VARS)
def test_gpu_stream_tiny_and_empty(cuda, var):
    """Frames inside one lane piece (the same-piece slow path), empty frames,
    and 8+ frame ends in one line (the offset-block stall path)."""
    from lneto_amd import synth
    rng = np.random.default_rng(21)
    for trial in range(4):
        lens = rng.choice([0, 0, 1, 2, 3, 4, 5, 7, 9, 15, 16, 17, 33, 64, 200], size=20000 + 977 * trial)
        off = synth.offsets_from_lengths(lens) + trial * 37
        off = np.concatenate([[0], off]).astype(np.uint64)
        _check(cuda, off, 200 + trial, f"tiny {trial}", var)
    # mixed: long runs of 64-byte frames (two events per line), then Zipf
    lens = np.concatenate([np.full(50000, 64), synth.zipf_lengths(50000, seed=5), np.full(3000, 1)])
    _check(cuda, synth.offsets_from_lengths(lens), 300, "mixed", var)


@pytest.mark.gpu
@pytest.mark.parametrize("var", VARS)
def test_gpu_stream_slice_ends(cuda, var):
    """Small batches: rows with zero or one frame, slices ending at every offset mod 128."""
    from lneto_amd import synth
    for n in (1, 2, 7, 127, 128, 129, 1000):
        for pad in (0, 13, 64, 127):
            lens = synth.zipf_lengths(n, seed=n + pad)
            off = (synth.offsets_from_lengths(lens) + pad).astype(np.uint64)
            off = np.concatenate([[0], off]).astype(np.uint64)
            _check(cuda, off, n * 7 + pad, f"n {n} pad {pad}", var)
