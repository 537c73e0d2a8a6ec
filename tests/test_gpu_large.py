"""GPU parity at BASELINE.json's full per-GPU sizes (VERDICT r2 "Next" item 1).

* configs[4]'s per-GPU slice: 16 M x 1500 B (24 GB, the slice bench.py's
  mtu1500_x8 workload runs on every rank), synthesized on the device.  Frame
  offsets run past 2^32, and the kernels keep only the low offset dword per
  frame (the workgroup's byte range is addressed relative to its first frame),
  so the frames straddling 2^31, 2^32 and 2^34 are sampled on purpose.
* more than 4 GiB of frames checked frame by frame against the C oracle;
* configs[2]'s 9000-B frames at a batch size where every CU claims chunks;
* lnx_crc32_batch_multi (the in-process per-GPU partition of SURVEY.md §8(e))
  on one GPU named twice, against the single call.

Reference semantics: ethernet.CRC32 (ethernet/crc.go:19-21); the FCS is
stored little-endian after the frame (internet/stack-ethernet.go:211-214), so
CRC32(frame || FCS) is the CRC-32 residue for every frame."""
import numpy as np
import pytest

import lneto_amd as L
from lneto_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _frame_at(byte: int, flen: int) -> int:
    return byte // flen


def test_configs4_slice_16m_frames_past_4gib(cuda):
    import torch
    n, flen = 1 << 24, 1500
    d = synth.bytes_torch(n * flen, cuda, seed=synth.SEED + 0x4000)
    fr = d.view(n, flen)
    starts = torch.arange(n, dtype=torch.int64, device=cuda) * flen
    lens = torch.full((n,), flen - 4, dtype=torch.int32, device=cuda)
    fcs = L.crc32_segments(d, starts, lens)           # segment mode: CRC of each frame's first 1496 B
    fr[:, flen - 4:] = fcs.view(torch.uint8).view(n, 4)  # LE FCS after the data
    off = torch.arange(n + 1, dtype=torch.int64, device=cuda) * flen
    assert int(off[-1]) > (1 << 34)
    # every frame: the FCS verifies (offsets mode, residue test) and the full-frame CRC is the residue
    ok = L.fcs_verify_batch(d, off)
    assert int(ok.sum()) == n
    crc = L.crc32_batch(d, off)
    assert bool((crc == O.CRC32_RESIDUE).all())  # 0x2144DF1C < 2^31: the same int32
    # >= 4096 sampled frames against the oracle, including the ones holding byte 2^31, 2^32, 3*2^31, 2^34
    rng = np.random.default_rng(4)
    special = [_frame_at(b, flen) + k for b in (1 << 31, 1 << 32, 3 << 31, 1 << 34) for k in (-1, 0, 1)]
    idx = np.unique(np.concatenate([rng.choice(n, 4096, replace=False), special, [0, n - 1]]))
    assert (_frame_at(1 << 32, flen) * flen < (1 << 32) < (_frame_at(1 << 32, flen) + 1) * flen)
    host = fr[torch.from_numpy(idx).to(cuda)].cpu().numpy()
    got = fcs.cpu().numpy().view(np.uint32)[idx]
    for j, i in enumerate(idx):
        assert int(got[j]) == O.crc32(host[j, :flen - 4].tobytes()), f"frame {i}"
        assert int.from_bytes(host[j, flen - 4:].tobytes(), "little") == int(got[j])
    # one flipped byte in the frame straddling 2^32: exactly that frame fails
    i32 = _frame_at(1 << 32, flen)
    d[(1 << 32) + 1] ^= 0x20
    ok = L.fcs_verify_batch(d, off)
    assert int(ok.sum()) == n - 1 and int(ok[i32]) == 0
    del d, fr, fcs, ok, crc
    torch.cuda.empty_cache()


def test_over_4gib_against_c_oracle(cuda):
    """3 M x 1500 B (4.5 GB) frame by frame against the C oracle (16 threads)."""
    import torch
    n, flen = 3 << 20, 1500
    d = synth.bytes_torch(n * flen + 8, cuda, seed=synth.SEED + 0x4501)
    off_np = synth.fixed_offsets(n, flen) + np.uint64(3)  # odd base: every alignment class
    off = torch.from_numpy(off_np.astype(np.int64)).to(cuda)
    got = L.crc32_batch(d, off).cpu().numpy().view(np.uint32)
    host = d.cpu().numpy()
    want = O.crc32_frames(host, off_np, threads=16, amd64=O.has_clmul())
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]
    del d
    torch.cuda.empty_cache()


@pytest.mark.parametrize("base", [0, 5])
def test_jumbo_9000_every_cu(cuda, base):
    """configs[2]'s frame size at 64 Ki frames (256 workgroups, each claiming
    many 4-frame chunks of the 16-lane or 32-lane rows) against the C oracle."""
    import torch
    n, flen = 1 << 16, 9000
    d = synth.bytes_torch(n * flen + base + 8, cuda, seed=synth.SEED + 0x9000 + base)
    off_np = synth.fixed_offsets(n, flen) + np.uint64(base)
    off = torch.from_numpy(off_np.astype(np.int64)).to(cuda)
    got = L.crc32_batch(d, off).cpu().numpy().view(np.uint32)
    want = O.crc32_frames(d.cpu().numpy(), off_np, threads=16, amd64=O.has_clmul())
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]


def test_multi_entry_two_slices_one_gpu(cuda):
    """lnx_crc32_batch_multi(ngpu=2, devices=[0, 0]): the two halves of a
    1 M x 1500 B batch, each in its own buffer with local offsets, equal the
    single call over the whole batch."""
    import torch
    n, flen = 1 << 20, 1500
    d = synth.bytes_torch(n * flen, cuda, seed=synth.SEED + 0x3311)
    off = torch.arange(n + 1, dtype=torch.int64, device=cuda) * flen
    whole = L.crc32_batch(d, off)
    h = n // 2 + 7  # uneven split
    parts = [(d[: h * flen].contiguous(), off[: h + 1].contiguous()),
             (d[h * flen:].clone(), (off[h:] - off[h]).contiguous())]
    got = L.crc32_batch_multi(parts, [cuda.index or 0, cuda.index or 0])
    assert torch.equal(torch.cat(got), whole)
    with pytest.raises(L.LnetoError):
        L.crc32_batch_multi(parts, [0])


@pytest.mark.parametrize("base", [0, 5])
def test_configs2_jumbo_full_size(cuda, base):
    """configs[2] at its size (VERDICT r5 "Next" 1): 1 M x 9000 B = 9.4 GB,
    offsets past 2^33, through the default entry (the >= 4096-B mean takes the
    32-lane whole-line rows).  CRC of every frame against the C oracle (16
    threads, Go's amd64 path); then each frame gets its LE FCS (the oracle's
    CRC of its first 8996 bytes), all verify, and one flipped byte just past
    2^33 fails exactly its frame (ethernet/crc.go:19-21)."""
    import torch
    n, flen = 1 << 20, 9000
    d = synth.bytes_torch(n * flen + base + 8, cuda, seed=synth.SEED + 0x9009 + base)
    off_np = synth.fixed_offsets(n, flen) + np.uint64(base)
    assert int(off_np[-1]) > (1 << 33)
    off = torch.from_numpy(off_np.astype(np.int64)).to(cuda)
    got = L.crc32_batch(d, off).cpu().numpy().view(np.uint32)
    host = d.cpu().numpy()
    want = O.crc32_frames(host, off_np, threads=16, amd64=O.has_clmul())
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, bad[:10]
    # the FCS of each frame's first 8996 bytes: frames [s, s + 8996) and the 4-byte gaps, interleaved
    inner = np.empty(2 * n + 1, dtype=np.uint64)
    inner[0::2] = off_np
    inner[1::2] = off_np[:-1] + np.uint64(flen - 4)
    fcs = O.crc32_frames(host, inner, threads=16, amd64=O.has_clmul())[0::2].astype("<u4")
    del host
    pos = torch.from_numpy((off_np[:-1].astype(np.int64) + flen - 4)[:, None] + np.arange(4)).to(cuda)
    d[pos.reshape(-1)] = torch.from_numpy(fcs.view(np.uint8).copy()).to(cuda)
    ok = L.fcs_verify_batch(d, off)
    assert int(ok.sum()) == n
    crc = L.crc32_batch(d, off)
    assert bool((crc == O.CRC32_RESIDUE).all())
    at = (1 << 33) + 1
    d[at] ^= 0x10
    ok = L.fcs_verify_batch(d, off)
    i = (at - base) // flen
    assert int(ok.sum()) == n - 1 and int(ok[i]) == 0
    del d, off, ok, crc, pos
    torch.cuda.empty_cache()
