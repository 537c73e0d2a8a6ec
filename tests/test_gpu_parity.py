"""GPU parity of the HIP batch path against the oracle (bit-exact).

Every test calls through the C-ABI (lneto_amd -> liblneto_amd.so) on cuda:0
and compares with oracle/ (zlib + crc.go restatement, or the C oracle) or the
frozen golden vectors.  Edge cases follow the reference's tests:
ethernet/crc_test.go (empty, short, CRC appended LE), lneto_test.go (real
IPv4/TCP frames), x/xnet/xnet_test.go:1015-1110 (trailing FCS accepted,
flipped byte rejected).
"""
import struct

import numpy as np
import pytest

import lneto_amd as L
from lneto_amd import synth
from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _pack(frames, base_pad=0):
    """Pack byte strings back to back after `base_pad` filler bytes.

    Returns (data, off) with the N+1 offsets of the batch ABI: frame i is
    data[off[i]:off[i+1]], so frames are contiguous by construction.
    """
    parts, offs, pos = [b"\xAA" * base_pad], [base_pad], base_pad
    for f in frames:
        parts.append(f)
        pos += len(f)
        offs.append(pos)
    return np.frombuffer(b"".join(parts) + b"\0" * 8, dtype=np.uint8).copy(), np.array(offs, dtype=np.uint64)


def _pack_segments(segs, gaps, base_pad=0):
    """Segments with filler gaps between them: (data, starts) for the (off, len) ABI of sum16."""
    parts, starts, pos = [b"\xAA" * base_pad], [], base_pad
    for s, g in zip(segs, gaps):
        parts.append(b"\x55" * int(g))
        pos += int(g)
        starts.append(pos)
        parts.append(s)
        pos += len(s)
    return np.frombuffer(b"".join(parts) + b"\0" * 8, dtype=np.uint8).copy(), np.array(starts, dtype=np.uint64)


def _dev(cuda, data, off):
    import torch
    return (torch.from_numpy(data).to(cuda), torch.from_numpy(off.astype(np.int64)).to(cuda))


def _crc_gpu(cuda, data, off):
    d, o = _dev(cuda, data, off)
    out = L.crc32_batch(d, o)
    import torch
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


def test_golden_vectors(cuda, golden):
    frames = [bytes.fromhex(v["data"]) for v in golden["crc32_vectors"]]
    frames.append(bytes.fromhex(golden["crc32_check"]["data"]))
    want = [v["crc"] for v in golden["crc32_vectors"]] + [golden["crc32_check"]["crc"]]
    data, off = _pack(frames)
    got = _crc_gpu(cuda, data, off)
    assert [int(x) for x in got] == want


def test_lneto_frames_fcs(cuda, golden):
    frames = [bytes.fromhex(f["frame"]) for f in golden["lneto_tcp_frames"]]
    data, off = _pack(frames)
    got = _crc_gpu(cuda, data, off)
    assert [int(x) for x in got] == [f["fcs"] for f in golden["lneto_tcp_frames"]]


@pytest.mark.parametrize("base_pad", [0, 1, 2, 3])
def test_every_length_every_alignment(cuda, base_pad):
    """Lengths 0..1100 in shuffled order after a 0-3 byte pad: every lead-in length
    and every start/end alignment occurs."""
    rng = np.random.default_rng(7 + base_pad)
    lens = list(range(0, 1101))
    blob = synth.bytes_np(sum(lens) + 64, seed=0xA11 + base_pad)
    frames, pos = [], 0
    for n in lens:
        frames.append(blob[pos:pos + n].tobytes())
        pos += n
    rng.shuffle(frames)
    data, off = _pack(frames, base_pad=base_pad)
    got = _crc_gpu(cuda, data, off)
    want = O.crc32_frames(data, off)
    bad = np.nonzero(got != want)[0]
    assert bad.size == 0, f"mismatch at lengths {[len(frames[i]) for i in bad[:10]]}"


def test_long_frames(cuda):
    lens = [2047, 2048, 2049, 4095, 9000, 9018, 65535, 65536, 65539, 262147, 1 << 20]
    blob = synth.bytes_np(sum(lens), seed=0xB16)
    frames, pos = [], 0
    for n in lens:
        frames.append(blob[pos:pos + n].tobytes())
        pos += n
    data, off = _pack(frames, base_pad=3)
    got = _crc_gpu(cuda, data, off)
    assert list(got) == list(O.crc32_frames(data, off))


def test_slice_over_2gib_takes_the_generic_path(cuda):
    """A workgroup slice of more than 2 GiB does not fit the 31-bit buffer
    offsets of the pipelined bodies and is folded by rows_generic
    (crc32_kernel.hip: static per-wave ranges, byte loads): 16 frames of
    ~136 MB in one slice, the first starting at an odd offset."""
    import torch
    lens = np.array([136_000_001 + 17 * i for i in range(16)], dtype=np.int64)
    off = (synth.offsets_from_lengths(lens) + 5).astype(np.uint64)
    assert int(off[-1] - off[0]) > (1 << 31)
    d = synth.bytes_torch(int(off[-1]) + 8, cuda, seed=0x2619)
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    got = L.crc32_batch(d, o).cpu().numpy().view(np.uint32)
    host = d.cpu().numpy()
    want = O.crc32_frames(host, off, threads=8)
    assert np.array_equal(got, want), np.nonzero(got != want)[0]
    # FCS verify through the same path: frame 3 gets its LE FCS in its last 4 bytes
    s3, e3 = int(off[3]), int(off[4])
    fcs = O.crc32(host[s3:e3 - 4].tobytes())
    d[e3 - 4:e3] = torch.tensor(list(int(fcs).to_bytes(4, "little")), dtype=torch.uint8, device=cuda)
    ok = L.fcs_verify_batch(d, o).cpu().numpy()
    assert list(ok) == [1 if i == 3 else 0 for i in range(16)], list(ok)


def test_empty_batch_and_empty_frames(cuda):
    import torch
    d = torch.zeros(16, dtype=torch.uint8, device=cuda)
    o = torch.zeros(1, dtype=torch.int64, device=cuda)
    assert L.crc32_batch(d, o).numel() == 0
    data, off = _pack([b"", b"", b"x", b""])
    assert [int(x) for x in _crc_gpu(cuda, data, off)] == [0, 0, O.crc32(b"x"), 0]
    # a frame whose end offset is below its start is treated as empty
    off_bad = np.array([0, 8, 4, 12], dtype=np.uint64)
    data = np.arange(16, dtype=np.uint8)
    got = _crc_gpu(cuda, data, off_bad)
    assert int(got[1]) == 0 and int(got[0]) == O.crc32(data[:8].tobytes())


def test_fcs_verify(cuda, golden):
    """Residue check == CRC32(f[:-4]) == LE32(f[-4:]) (x/xnet/xnet_test.go:1015-1110 shape)."""
    import torch
    rng = np.random.default_rng(11)
    frames, want = [], []
    for i in range(600):
        n = int(rng.integers(0, 1600))
        payload = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        f = payload + struct.pack("<I", O.crc32(payload))
        kind = i % 4
        if kind == 1 and n > 0:       # flipped payload byte -> reject
            b = bytearray(f)
            b[int(rng.integers(0, n))] ^= 0x01
            f = bytes(b)
        elif kind == 2:               # flipped FCS bit -> reject
            b = bytearray(f)
            b[-1] ^= 0x80
            f = bytes(b)
        elif kind == 3:               # truncated below 4 bytes -> reject
            f = f[: int(rng.integers(0, 4))]
        frames.append(f)
        ok = len(f) >= 4 and O.crc32(f[:-4]) == struct.unpack("<I", f[-4:])[0]
        want.append(1 if ok else 0)
    data, off = _pack(frames, base_pad=1)
    d, o = _dev(cuda, data, off)
    got = L.fcs_verify_batch(d, o)
    torch.cuda.synchronize()
    assert got.cpu().numpy().tolist() == want


def test_misaligned_base_pointer(cuda):
    """d_bytes itself not 4-byte aligned (a view into a larger allocation)."""
    import torch
    off = synth.offsets_from_lengths(np.array([60, 61, 62, 63, 1500, 1, 2, 3, 4, 5, 9000]))
    data = synth.bytes_np(int(off[-1]) + 8, seed=3)
    want = O.crc32_frames(data, off)
    for shift in (1, 2, 3):
        big = torch.zeros(len(data) + 8, dtype=torch.uint8, device=cuda)
        big[shift:shift + len(data)] = torch.from_numpy(data).to(cuda)
        view = big[shift:shift + len(data)]
        o = torch.from_numpy(off.astype(np.int64)).to(cuda)
        got = L.crc32_batch(view, o)
        torch.cuda.synchronize()
        assert np.array_equal(got.cpu().numpy().view(np.uint32), want)


def test_mtu_batch_full_parity(cuda):
    """64 Ki x 1500-byte frames generated on device == C oracle on host."""
    import torch
    n = 1 << 16
    off = synth.fixed_offsets(n, 1500)
    d = synth.bytes_torch(int(off[-1]), cuda)
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    got = L.crc32_batch(d, o).cpu().numpy().view(np.uint32)
    want = O.crc32_frames(d.cpu().numpy(), off, threads=8)
    assert np.array_equal(got, want)


def test_zipf_batch_parity(cuda):
    import torch
    off = synth.offsets_from_lengths(synth.zipf_lengths(1 << 17))
    d = synth.bytes_torch(int(off[-1]), cuda)
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    got = L.crc32_batch(d, o).cpu().numpy().view(np.uint32)
    want = O.crc32_frames(d.cpu().numpy(), off, threads=8)
    assert np.array_equal(got, want)


def test_full_size_fcs_roundtrip(cuda):
    """BASELINE configs[1] size (1 M x 1500 B): append each frame's CRC as its
    FCS on device, then every frame must pass the residue verify and a sample
    must match the oracle.  Size-independent property (encode -> verify)."""
    import torch
    n, L0 = 1 << 20, 1500
    d = synth.bytes_torch(n * L0, cuda)
    o = torch.arange(n + 1, dtype=torch.int64, device=cuda) * L0
    crc = L.crc32_batch(d, o)
    framed = torch.empty((n, L0 + 4), dtype=torch.uint8, device=cuda)
    framed[:, :L0] = d.view(n, L0)
    framed[:, L0:] = crc.view(torch.uint8).view(n, 4)
    o2 = torch.arange(n + 1, dtype=torch.int64, device=cuda) * (L0 + 4)
    ok = L.fcs_verify_batch(framed.view(-1), o2)
    assert int(ok.sum()) == n
    idx = np.random.default_rng(5).choice(n, 512, replace=False)
    host = d.view(n, L0)[torch.from_numpy(idx).to(cuda)].cpu().numpy()
    got = crc.cpu().numpy().view(np.uint32)[idx]
    assert all(int(got[k]) == O.crc32(host[k].tobytes()) for k in range(len(idx)))
    # corrupt one byte in 1000 frames -> exactly those fail
    bad = torch.from_numpy(np.random.default_rng(6).choice(n, 1000, replace=False)).to(cuda)
    framed[bad, 100] ^= 0x10
    ok = L.fcs_verify_batch(framed.view(-1), o2)
    assert int(ok.sum()) == n - 1000
    assert int(ok[bad].sum()) == 0


# ------------------------------------------------------------ internet checksum
def _sum_gpu(cuda, data, off, lens, seeds):
    import torch
    d = torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(np.asarray(off, dtype=np.int64)).to(cuda)
    ln = torch.from_numpy(np.asarray(lens, dtype=np.uint32).view(np.int32)).to(cuda)
    sd = None if seeds is None else torch.from_numpy(np.asarray(seeds, dtype=np.uint32).view(np.int32)).to(cuda)
    out = L.sum16_batch(d, o, ln, sd)
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint16)


def test_sum16_golden(cuda, golden):
    segs = [bytes.fromhex(v["data"]) for v in golden["sum16_vectors"]]
    data, starts = _pack_segments(segs, gaps=[i % 3 for i in range(len(segs))], base_pad=1)
    got = _sum_gpu(cuda, data, starts, [len(s) for s in segs], [v["seed"] for v in golden["sum16_vectors"]])
    assert [int(x) for x in got] == [v["sum16"] for v in golden["sum16_vectors"]]


def test_sum16_lneto_tcp_kat(cuda, golden):
    """lneto_test.go:119-160 through the GPU: IPv4 header sum and TCP sum with pseudo-header."""
    segs, seeds, want = [], [], []
    for fr in golden["lneto_tcp_frames"]:
        f = bytearray.fromhex(fr["frame"])
        ip = f[14:]
        # IPv4 header checksum: zero the field, sum the 20-byte header (ipv4/frame.go:138-146)
        hdr = bytearray(ip[:20])
        hdr[10:12] = b"\0\0"
        segs.append(bytes(hdr)); seeds.append(0); want.append(fr["ipv4_sum_want"])
        # TCP: pseudo-header seed (ipv4/frame.go:154-158), checksum field zeroed
        seed = O.ipv4_tcp_pseudo(bytes(ip)).sum
        tcp = bytearray(ip[20:])
        tcp[16:18] = b"\0\0"
        segs.append(bytes(tcp)); seeds.append(seed); want.append(fr["tcp_sum_want"])
    data, starts = _pack_segments(segs, gaps=[1, 0, 3, 2])
    got = _sum_gpu(cuda, data, starts, [len(s) for s in segs], seeds)
    assert [int(x) for x in got] == want


def test_sum16_random_segments(cuda):
    rng = np.random.default_rng(21)
    n = 5000
    blob = synth.bytes_np(1 << 22, seed=77)
    lens = rng.integers(0, 1600, size=n).astype(np.uint32)
    lens[:8] = [0, 1, 2, 3, 4, 5, 20, 9000]
    starts = rng.integers(0, len(blob) - 10000, size=n).astype(np.uint64)
    seeds = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    seeds[:4] = [0, 0xFFFFFFFF, 0xFFFF0000, 0x0001FFFE]
    got = _sum_gpu(cuda, blob, starts, lens, seeds)
    want = O.sum16_segments(blob, starts, lens, seeds)
    assert np.array_equal(got, want)
    got0 = _sum_gpu(cuda, blob, starts, lens, None)
    assert np.array_equal(got0, O.sum16_segments(blob, starts, lens, None))


def test_host_convenience(cuda):
    off = synth.offsets_from_lengths(np.array([60, 1500, 9000, 7, 0, 33]))
    data = synth.bytes_np(int(off[-1]), seed=9)
    got = L.crc32_batch_host(data, off, device=0)
    assert np.array_equal(got, O.crc32_frames(data, off))


def test_sum16_kernel_variants_agree(cuda):
    """The sum16 kernels (line rows with default-policy edge lines = product,
    half-line rows = r1c, line rows with the default cache policy, line rows
    with 8 and 16 lines in flight, line rows all nt) on random segments at every start alignment
    mod 128, lengths 0..2000, 8192 segments (more workgroups than CUs), three
    launches each."""
    import ctypes
    import torch
    L.research_lib().lnx__sum16_variant.restype = ctypes.c_int
    L.research_lib().lnx__sum16_variant.argtypes = [ctypes.c_int] + [ctypes.c_void_p] * 4 + [ctypes.c_uint64] + \
        [ctypes.c_void_p] * 2
    rng = np.random.default_rng(23)
    n = 8192
    blob = synth.bytes_np(1 << 21, seed=78)
    lens = rng.integers(0, 2001, size=n).astype(np.uint32)
    starts = (rng.integers(0, (len(blob) - 4096) // 128, size=n) * 128 + np.arange(n) % 128).astype(np.uint64)
    seeds = rng.integers(0, 1 << 32, size=n, dtype=np.uint64).astype(np.uint32)
    want = O.sum16_segments(blob, starts, lens, seeds)
    d = torch.from_numpy(blob).to(cuda)
    o = torch.from_numpy(starts.astype(np.int64)).to(cuda)
    ln = torch.from_numpy(lens.view(np.int32)).to(cuda)
    sd = torch.from_numpy(seeds.view(np.int32)).to(cuda)
    for var in (0, 1, 2, 3, 4, 5) * 3:
        out = torch.empty(n, dtype=torch.int16, device=cuda)
        assert L.research_lib().lnx__sum16_variant(var, d.data_ptr(), o.data_ptr(), ln.data_ptr(), sd.data_ptr(), n,
                                        out.data_ptr(), torch.cuda.current_stream().cuda_stream) == 0
        torch.cuda.synchronize()
        bad = np.nonzero(out.cpu().numpy().view(np.uint16) != want)[0]
        assert bad.size == 0, f"sum16 variant {var}: {bad.size} wrong, first {bad[:8]}"
