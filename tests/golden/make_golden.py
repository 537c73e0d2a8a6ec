"""Generate tests/golden/vectors.json — frozen checksum vectors for the parity tests.

Run from the repo root:  python tests/golden/make_golden.py

Sources of truth, in order of authority:
  1. The reference's own known answers, copied as data:
     - lneto_test.go:120-131  two Ethernet+IPv4+TCP SYN frames; their IPv4 header
       checksums (0xa3aa, 0xaa6a) and TCP checksums (0x62bc, 0xde02) are the
       values stored in the frames and asserted at lneto_test.go:145-157.
     - ethernet/crc_test.go:8-100  CRC32Search cases (payload, minOff -> offset).
  2. The CRC-32/ISO-HDLC check value 0xCBF43926 (Go hash/crc32 IEEE is that CRC).
  3. Everything else is computed by the oracle (oracle/oracle.py: zlib + the
     crc.go restatement) and frozen here so the GPU box, which has no Python
     reference, compares against fixed data.
"""
from __future__ import annotations

import json
import os
import struct
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

from oracle import oracle as O  # noqa: E402
from lneto_amd import synth  # noqa: E402

OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "vectors.json")

# lneto_test.go:120-131 (frame bytes, verbatim data)
LNETO_TCP_FRAMES = [
    "c0ffee00dead4e8b3af9fb6b08004500003c01be40004006a3aac0a80a01c0a80a02e70a00504060d5cc"
    "00000000a002faf062bc0000020405b40402080abbac9bca0000000001030307",
    "c0ffee00dead4e8b3af9fb6b08004500003cfafd40004006aa6ac0a80a01c0a80a02e70e00509cdcfe05"
    "00000000a002faf0de020000020405b40402080abbac9bca0000000001030307",
]
LNETO_IPV4_WANT = [0xA3AA, 0xAA6A]
LNETO_TCP_WANT = [0x62BC, 0xDE02]


def crc_test_go_cases():
    """ethernet/crc_test.go:8-100, as (data_hex, min_off, want_off) triples."""
    def make(payload_len):
        d = bytearray(i & 0xFF for i in range(payload_len)) + bytearray(4)
        struct.pack_into("<I", d, payload_len, O.crc32(bytes(d[:payload_len])))
        return bytes(d)
    cases = []
    d100 = make(100)
    cases += [(d100, 0, 100), (d100, 50, 100), (d100, 100, 100), (d100, 101, -1)]   # :20-50
    cases.append((bytes(i & 0xFF for i in range(100)), 0, -1))                       # :52-61
    cases.append((bytes([1, 2, 3]), 0, -1))                                          # :63-69
    cases.append((make(20), -5, 20))                                                 # :71-77
    z = bytearray(4)
    struct.pack_into("<I", z, 0, O.crc32(b""))
    cases.append((bytes(z), 0, 0))                                                   # :79-88
    cases.append((make(50) + bytes(50), 0, 50))                                      # :90-99
    return [{"data": d.hex(), "min_off": m, "want": w} for d, m, w in cases]


def main():
    vec = {"_doc": __doc__.strip().splitlines()[0]}
    vec["crc32_check"] = {"data": b"123456789".hex(), "crc": O.CRC32_CHECK}
    vec["crc32_search_cases"] = crc_test_go_cases()

    frames = []
    for hx, ipw, tcpw in zip(LNETO_TCP_FRAMES, LNETO_IPV4_WANT, LNETO_TCP_WANT):
        f = bytes.fromhex(hx)
        assert len(f) == 74, len(f)
        frames.append({"frame": hx, "ipv4_off": 14, "ipv4_sum_want": ipw, "tcp_sum_want": tcpw,
                       "fcs": O.crc32(f)})
    vec["lneto_tcp_frames"] = frames

    # CRC-32 over synthetic bytes, all lengths 0..64 plus boundary lengths.
    lens = list(range(0, 65)) + [127, 128, 129, 255, 256, 257, 1499, 1500, 1514, 1518, 9000, 9018]
    blob = synth.bytes_np(sum(lens) + 16, seed=0x5EED)
    crc_vecs, pos = [], 0
    for n in lens:
        d = blob[pos:pos + n].tobytes()
        crc_vecs.append({"len": n, "data": d.hex(), "crc": O.crc32(d)})
        pos += n
    vec["crc32_vectors"] = crc_vecs

    # Internet checksum over synthetic segments with pseudo-header-like seeds.
    sum_vecs = []
    blob2 = synth.bytes_np(4096, seed=0xC0FFEE)
    for i, n in enumerate([0, 1, 2, 3, 7, 8, 19, 20, 21, 60, 61, 1479, 1480, 1481]):
        start = (i * 37) % 512
        d = blob2[start:start + n].tobytes()
        seed = (0x12345 * (i + 1)) & 0xFFFFFFFF
        sum_vecs.append({"data": d.hex(), "seed": seed, "sum16": O.payload_sum16(seed, d)})
    # uint32 wrap-around case (crc.go:25): seed close to 2^32
    d = bytes([0xFF]) * 40
    sum_vecs.append({"data": d.hex(), "seed": 0xFFFFFF00, "sum16": O.payload_sum16(0xFFFFFF00, d)})
    vec["sum16_vectors"] = sum_vecs

    with open(OUT, "w") as fh:
        json.dump(vec, fh, indent=1)
    print(f"wrote {OUT}")


if __name__ == "__main__":
    main()
