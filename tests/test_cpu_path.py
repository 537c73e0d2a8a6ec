"""Per-frame host functions of liblneto_amd.so (exact Go semantics) vs the oracle.

These mirror the reference's single-frame tests: ethernet/crc_test.go:8-100
(CRC32Search) and lneto_test.go:119-160 (CRC791 through the pseudo-headers).
No GPU needed: the per-frame API never launches a kernel.
"""
import numpy as np

import lneto_amd as L
from oracle import oracle as O


def test_crc32_check_and_nil(golden):
    assert L.crc32(bytes.fromhex(golden["crc32_check"]["data"])) == O.CRC32_CHECK
    assert L.crc32(b"") == 0


def test_crc32_vectors(golden):
    for v in golden["crc32_vectors"]:
        assert L.crc32(bytes.fromhex(v["data"])) == v["crc"], v["len"]


def test_crc32_update_hook_contract():
    """StackEthernet calls crcupdate(0, frame) (internet/stack-ethernet.go:211-214)."""
    rng = np.random.default_rng(3)
    for n in [0, 1, 15, 16, 17, 60, 1500]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert L.crc32_update(0, d) == O.crc32(d)
        for cut in {0, n // 3, n}:
            assert L.crc32_update(L.crc32_update(0, d[:cut]), d[cut:]) == O.crc32(d)


def test_crc32_search_cases(golden):
    for case in golden["crc32_search_cases"]:
        d = bytes.fromhex(case["data"])
        assert L.crc32_search(d, case["min_off"]) == case["want"], case


def test_crc32_search_random():
    rng = np.random.default_rng(4)
    for _ in range(60):
        n = int(rng.integers(0, 200))
        d = bytearray(rng.integers(0, 256, n + 4, dtype=np.uint8).tobytes())
        if rng.random() < 0.7:
            d[n:n + 4] = O.crc32(bytes(d[:n])).to_bytes(4, "little")
        m = int(rng.integers(-3, n + 3))
        assert L.crc32_search(bytes(d), m) == O.crc32_search(bytes(d), m)


def test_min64_frame_plumbing():
    """BASELINE configs[0]: 60 data bytes + LE FCS as StackEthernet.Encapsulate emits
    (padding internet/stack-ethernet.go:203-207, FCS :211-214); CRC32Search finds 60."""
    from lneto_amd import synth
    data = synth.bytes_np(60 * 64)
    for i in range(64):
        f = data[60 * i:60 * (i + 1)].tobytes()
        fr = f + L.crc32(f).to_bytes(4, "little")
        assert len(fr) == 64
        assert L.crc32_search(fr, 0) == 60
        assert L.crc32(fr) == O.CRC32_RESIDUE


def test_crc791(golden):
    for v in golden["sum16_vectors"]:
        assert L.payload_sum16(v["seed"], bytes.fromhex(v["data"])) == v["sum16"]
    for fr in golden["lneto_tcp_frames"]:
        ip = bytes.fromhex(fr["frame"])[14:]
        c = L.CRC791()
        c.WriteEven(ip[:20])
        assert c.Sum16() == 0                      # stored checksum verifies
        seed = O.ipv4_tcp_pseudo(ip).sum
        c = L.CRC791()
        c.WriteEven(ip[12:20])
        c.AddUint16(((ip[2] << 8) | ip[3]) - (ip[0] & 0xF) * 4)
        c.AddUint16(ip[9])
        assert c.sum == seed
        assert c.PayloadSum16(ip[20:]) == 0
    assert L.never_zero_sum(0) == 0xFFFF and L.never_zero_sum(0x1234) == 0x1234
    assert L.sum16(0x0001FFFE) == O.sum16(0x0001FFFE)


def test_crc791_random_vs_oracle():
    rng = np.random.default_rng(5)
    for _ in range(200):
        n = int(rng.integers(0, 3000))
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        s = int(rng.integers(0, 1 << 32))
        assert L.payload_sum16(s, d) == O.payload_sum16(s, d)
        even = d[: n & ~1]
        assert L.sum_write_even(s, even) == O.sum_write_even(s, even)
