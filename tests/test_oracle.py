"""Pin the oracle before trusting it (CPU only).

The oracle's CRC-32 and internet-checksum restatements are checked against
  - the reference's own known answers: lneto_test.go:119-160 (IPv4 header and
    TCP checksums of two real SYN frames) and ethernet/crc_test.go:8-100
    (CRC32Search cases, CRC appended little-endian);
  - the CRC-32/ISO-HDLC check value 0xCBF43926 (Go hash/crc32 IEEE);
  - each other (zlib, bit-serial Python, C slicing-by-8, C byte-table).
"""
import struct

import numpy as np
import pytest

from oracle import oracle as O


def test_check_value(golden):
    d = bytes.fromhex(golden["crc32_check"]["data"])
    assert O.crc32(d) == O.CRC32_CHECK == golden["crc32_check"]["crc"]
    assert O.crc32_bitwise(d) == O.CRC32_CHECK
    assert O.c_crc32(d) == O.CRC32_CHECK
    assert O.c_crc32_simple(d) == O.CRC32_CHECK


def test_crc32_nil_is_zero():
    # CRC32(nil) == 0: ethernet/crc_test.go:79-88 relies on it.
    assert O.crc32(b"") == 0 and O.c_crc32(b"") == 0 and O.crc32_bitwise(b"") == 0


def test_crc_test_go_search_cases(golden):
    """ethernet/crc_test.go:8-100 subtests, via the Python and C restatements."""
    for case in golden["crc32_search_cases"]:
        d = bytes.fromhex(case["data"])
        assert O.crc32_search(d, case["min_off"]) == case["want"], case
        assert O.c_crc32_search(d, case["min_off"]) == case["want"], case


def test_crc_test_go_payload_values():
    """The crc_test.go payloads (data[i] = byte(i)) — values cross-checked by three restatements."""
    for n, want in [(100, 0x58C932F5), (50, 0xB50C79FF), (20, 0x3BDDFFA4)]:
        d = bytes(i & 0xFF for i in range(n))
        assert O.crc32(d) == want
        assert O.crc32_bitwise(d) == want
        assert O.c_crc32(d) == want


def test_restatements_agree(golden):
    for v in golden["crc32_vectors"]:
        d = bytes.fromhex(v["data"])
        assert O.crc32(d) == v["crc"]
        assert O.c_crc32(d) == v["crc"]
        assert O.c_crc32_simple(d) == v["crc"]
        if len(d) <= 300:
            assert O.crc32_bitwise(d) == v["crc"]


def test_update_composes():
    """crc32.Update(Update(0, a), b) == Checksum(a+b): the CRC32Update hook contract."""
    rng = np.random.default_rng(1)
    for _ in range(50):
        a = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        b = rng.integers(0, 256, int(rng.integers(0, 300)), dtype=np.uint8).tobytes()
        assert O.crc32_update(O.crc32_update(0, a), b) == O.crc32(a + b)


def test_residue_equivalence():
    """CRC32(f[:-4]) == LE32(f[-4:])  <=>  CRC32(f) == 0x2144DF1C (used by FCS verify)."""
    rng = np.random.default_rng(2)
    for n in list(range(0, 40)) + [1500, 9000]:
        m = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        f = m + struct.pack("<I", O.crc32(m))
        assert O.crc32(f) == O.CRC32_RESIDUE
        bad = bytearray(f)
        bad[int(rng.integers(0, len(f)))] ^= 1 << int(rng.integers(0, 8))
        assert O.crc32(bytes(bad)) != O.CRC32_RESIDUE


def test_lneto_tcp_kat(golden):
    """lneto_test.go:119-160: the IPv4 header and TCP checksums stored in two real frames."""
    for fr in golden["lneto_tcp_frames"]:
        f = bytearray.fromhex(fr["frame"])
        ip = f[14:]
        assert (ip[10] << 8 | ip[11]) == fr["ipv4_sum_want"]
        hdr = bytearray(ip[:20])
        hdr[10:12] = b"\0\0"
        assert O.ipv4_header_sum16(bytes(hdr)) == fr["ipv4_sum_want"]
        # verify form: the unzeroed header sums to 0 (internet/stack-ip4.go:128)
        assert O.ipv4_header_sum16(bytes(ip[:20])) == 0
        tcp = bytearray(ip[20:])
        assert (tcp[16] << 8 | tcp[17]) == fr["tcp_sum_want"]
        crc = O.ipv4_tcp_pseudo(bytes(ip))
        assert crc.payload_sum16(bytes(ip[20:])) == 0  # verify (internet/stack-ip4.go:145)
        tcp[16:18] = b"\0\0"
        assert crc.payload_sum16(bytes(tcp)) == fr["tcp_sum_want"]
        assert O.crc32(bytes(f)) == fr["fcs"]


def test_sum16_restatements(golden):
    for v in golden["sum16_vectors"]:
        d = bytes.fromhex(v["data"])
        assert O.payload_sum16(v["seed"], d) == v["sum16"]
        assert O.c_payload_sum16(v["seed"], d) == v["sum16"]


def test_sum16_wraparound_is_uint32():
    """crc.go:25 adds into a uint32 with wrap-around (not one's-complement carry)."""
    d = b"\xff\xff" * 4
    s = 0xFFFFFFF0
    assert O.sum_write_even(s, d) == (s + 4 * 0xFFFF) & 0xFFFFFFFF


def test_never_zero_and_crc791_methods():
    assert O.never_zero_sum(0) == 0xFFFF and O.never_zero_sum(5) == 5
    c = O.CRC791()
    c.add_uint32(0x12345678)
    assert c.sum == 0x1234 + 0x5678
    c.add_uint16(0xFFFF)
    assert c.sum16() == O.sum16(0x1234 + 0x5678 + 0xFFFF)
    c.reset()
    assert c.sum == 0
    with pytest.raises(IndexError):
        c.write_even(b"\x01\x02\x03")


def test_frames_batch_helper_threads():
    from lneto_amd import synth
    off = synth.offsets_from_lengths(synth.zipf_lengths(3000))
    data = synth.bytes_np(int(off[-1]))
    one = O.crc32_frames(data, off, threads=1)
    many = O.crc32_frames(data, off, threads=8)
    assert np.array_equal(one, many)
    assert all(int(one[i]) == O.crc32(data[int(off[i]):int(off[i + 1])].tobytes()) for i in range(0, 3000, 97))


def test_amd64_fast_path_matches_table_form():
    """Go's amd64 fast path restated (PCLMULQDQ folding for >= 64 bytes over the
    largest multiple of 16, slicing-by-8 tail: crc32_amd64.go archUpdateIEEE)
    equals the table form and zlib for every length 0..300, long random inputs
    and any starting register; the CPU baseline runs this form."""
    import zlib
    if not O.has_clmul():
        pytest.skip("no PCLMULQDQ on this CPU")
    rng = np.random.default_rng(11)
    lens = list(range(0, 301)) + [int(x) for x in rng.integers(301, 20000, size=100)]
    for n in lens:
        b = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        c = int(rng.integers(0, 1 << 32))
        assert O.c_crc32_update_amd64(0, b) == zlib.crc32(b)
        assert O.c_crc32_update_amd64(c, b) == zlib.crc32(b, c)
    off = np.concatenate([[0], np.cumsum(rng.integers(0, 3000, size=500))]).astype(np.uint64)
    data = rng.integers(0, 256, size=int(off[-1]), dtype=np.uint8)
    assert np.array_equal(O.crc32_frames(data, off, threads=4, amd64=True), O.crc32_frames(data, off, threads=4))
