"""Every CRC kernel configuration the dispatcher can pick, forced on every
workgroup, is bit-exact against the oracle.

The product dispatch (lnx_crc32_batch) chooses the row width per workgroup from
its frames' mean length, so a given test batch exercises only some of the
compiled configurations.  The profiling entry point lnx__crc32_variant forces
one configuration for the whole launch (ids in crc32_kernel.hip launch_rows).
"""
import ctypes

import numpy as np
import pytest

import lneto_amd as L
from lneto_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu

# 10..16: forced 32-lane rows (line-aligned windows, nt loads), (KS, S) = (13, 1), (13, 2),
#   (14, 1), (13, 1) with 2- and 8-frame chunks, (24, 1), (18, 1);
# 17/21: forced one-word 16-lane rows, (KS, S) = (24, 1), (12, 3);
# 18/19/28/29/40/41/42: forced two-word 16-lane rows (line windows, dwordx2 nt loads),
#   (13, 1), (13, 2), (14, 1), (24, 1), (13, 1) with 8- and 16-frame chunks, (12, 2);
# 22..25, 60, 63: forced 4-lane rows (16, 2) with 32-frame chunks, (8, 3), (12, 2), (6, 3), (16, 2) with 16, (16, 2) with 32;
# 50..52: forced lean line rows (lines_body), KSL = 13, 14, 12;
# 56: the product dispatch with one-word 16-lane rows instead of lean rows;
# 70: forced lean rows on 32 lanes x one word;
# 125: the product dispatch with 4-lane and one-word 16-lane rows loading every step of an item (r2),
#   120/124/126: loading runs of 2 / 1 / 6 steps (the product: 4)
# 130/138/139/140: the product dispatch with 4-lane rows of four words per lane (dwordx4, 64-byte row
#   steps, the RL = 16 image): 4 / 4 (16-frame chunks) / 3 / 5 steps per item
# 150 / 153: the product dispatch with streaming rows (stream_rows.hpp) of 8 / 4 lanes for the narrow rows' frames
FORCED = [10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 21, 22, 23, 24, 25, 28, 29, 40, 41, 42, 50, 51, 52, 56, 57, 60, 63, 70, 90, 92, 93, 97, 43, 44,
          120, 124, 125, 126, 130, 138, 139, 140, 150, 153, 160]

L.research_lib().lnx__crc32_variant.restype = ctypes.c_int
L.research_lib().lnx__crc32_variant.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                     ctypes.c_void_p, ctypes.c_void_p]


def _run(var, d, o, n):
    import torch
    out = torch.empty(n, dtype=torch.int32, device=d.device)
    rc = L.research_lib().lnx__crc32_variant(var, d.data_ptr(), o.data_ptr(), n, out.data_ptr(),
                                  torch.cuda.current_stream().cuda_stream)
    assert rc == 0
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def _batches(cuda):
    import torch
    rng = np.random.default_rng(5)
    # every length 0..700 shuffled, after a 3-byte pad: all lead-ins, all end alignments
    lens = rng.permutation(np.arange(0, 701))
    off = synth.offsets_from_lengths(lens) + 3
    off = np.concatenate([[0], off]).astype(np.uint64)  # frame 0 is the 3-byte pad
    yield "lengths", off
    yield "zipf", synth.offsets_from_lengths(synth.zipf_lengths(1 << 15, seed=77))
    yield "long", synth.offsets_from_lengths(np.array([1, 2, 3, 5, 4097, 9001, 65537, 1500, 1499, 1498, 1497]))


@pytest.mark.parametrize("var", FORCED)
def test_forced_configuration_parity(cuda, var):
    import torch
    for name, off in _batches(cuda):
        n = len(off) - 1
        data = synth.bytes_np(int(off[-1]) + 8, seed=0xC0FFEE + n)
        d = torch.from_numpy(data).to(cuda)
        o = torch.from_numpy(off.astype(np.int64)).to(cuda)
        got = _run(var, d, o, n)
        want = O.crc32_frames(data, off, threads=8)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, f"{name}: variant {var} wrong at frames {bad[:8]} (lens {np.diff(off)[bad[:8]]})"


@pytest.mark.parametrize("var", [0, 50, 18, 10, 70])
def test_range_end_alignments(cuda, var):
    """The last frame of a workgroup's range ends at every offset mod 128: the
    whole-line layouts load qwords / lines that straddle the end of the range
    descriptor (rounded up to 4 bytes); the bytes inside must still count."""
    import torch
    for pad in range(0, 128, 1):
        lens = np.array([1500, 1500, 1500, 1497 + (pad % 8)])
        off = synth.offsets_from_lengths(lens) + pad
        off = np.concatenate([[0], off]).astype(np.uint64)
        n = len(off) - 1
        data = synth.bytes_np(int(off[-1]), seed=pad)
        d = torch.from_numpy(data).to(cuda)
        o = torch.from_numpy(off.astype(np.int64)).to(cuda)
        got = _run(var, d, o, n)
        want = O.crc32_frames(data, off)
        assert np.array_equal(got, want), f"pad {pad}: variant {var} wrong at {np.nonzero(got != want)[0]}"
