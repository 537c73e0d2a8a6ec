"""The CRC algebra of the fused receive kernel (lneto_amd/csrc/rx_verify_kernel.hip,
DESIGN.md §3.12) restated on the host and checked against zlib (the arithmetic of
ethernet.CRC32, lneto ethernet/crc.go:19-21): 16 lanes fold the interleaved
8-byte chunks of a window that starts at the qword holding the frame's first
byte, r <- Z_128(r ^ w0) ^ Z_124(w1) per 128-byte line; the first line masked
to the frame with the init on its first four bytes, the later lines unmasked
(the last qword's bytes past the frame removed again by the lane that holds
it); then R = Z_{-b}(XOR_p Z_{-8(p + a)}(r_p)).  Every length 0..300 and long
frames, at every base alignment mod 8, with garbage before and after the
frame."""
import zlib

import numpy as np

POLY = 0xEDB88320


def _zbit(r):
    return (r >> 1) ^ np.where(r & 1, np.uint32(POLY), np.uint32(0)).astype(np.uint32)


def _unzbit(r):
    b = r >> 31
    t = np.where(b == 1, r ^ np.uint32(POLY), r).astype(np.uint32)
    return ((t << 1) | b).astype(np.uint32)


def _z(r, k):
    r = np.asarray(r, dtype=np.uint32).copy()
    for _ in range(8 * abs(k)):
        r = _zbit(r) if k > 0 else _unzbit(r)
    return r


E = np.arange(256, dtype=np.uint32)
NIB = np.array([v << (4 * i) for i in range(8) for v in range(16)], dtype=np.uint32)
T = [_z(E << np.uint32(8 * k), 128) for k in range(4)] + [_z(E << np.uint32(8 * k), 124) for k in range(4)]
F = [_z(NIB, -8 * q).reshape(8, 16) for q in range(32)]
B = [_z(NIB, -b).reshape(8, 16) for b in range(8)]


def _unit(v0, v1):
    r = 0
    for k in range(4):
        r ^= int(T[k][(v0 >> (8 * k)) & 0xFF]) ^ int(T[4 + k][(v1 >> (8 * k)) & 0xFF])
    return r


def _nib(tab, v):
    r = 0
    for i in range(8):
        r ^= int(tab[i][(v >> (4 * i)) & 15])
    return r


def _range(o0, a, b):
    """rv_range: byte mask of the frame offsets [a, b) in the word whose byte 0 is at o0."""
    m = 0
    for j in range(4):
        if a <= o0 + j < b:
            m |= 0xFF << (8 * j)
    return m


def _fused_crc_register(buf: bytes, mis: int, Lt: int) -> int:
    """The kernel's register after the frame buf[mis : mis + Lt] (buf 8-aligned at index 0)."""
    QE = (Lt + mis + 7) >> 3
    le = lambda q, h: int.from_bytes(buf[8 * q + 4 * h: 8 * q + 4 * h + 4], "little") if 0 <= q < QE else 0
    NL = (QE + 15) >> 4
    lastq = QE - 1
    ie = min(Lt, 4)
    keep = lambda k: (0xFFFFFFFF << (8 * min(max(k, 0), 4))) & 0xFFFFFFFF
    regs = []
    for p in range(16):
        r = 0
        for line in range(NL):
            q = p + 16 * line
            c0, c1 = le(q, 0), le(q, 1)
            if line == 0:  # unit 0: the frame's bytes only, the CRC init on its first four
                o0 = 8 * q - mis
                c0 = (c0 & _range(o0, 0, Lt)) ^ _range(o0, 0, ie)
                c1 = (c1 & _range(o0 + 4, 0, Lt)) ^ _range(o0 + 4, 0, ie)
            r = _unit(r ^ c0, c1)
        # the last qword's bytes past the frame went in unmasked (lines >= 1): the
        # lane that holds it takes their part out again (it was that lane's last unit)
        if lastq >= 16 and (lastq & 15) == p:
            ol = 8 * lastq - mis
            r ^= _unit(le(lastq, 0) & keep(Lt - ol), le(lastq, 1) & keep(Lt - ol - 4))
        regs.append(r)
    pad = 128 * NL - mis - Lt
    a, b = pad >> 3, pad & 7
    assert 0 <= a < 16
    x = 0
    for p in range(16):
        x ^= _nib(F[p + a], regs[p])
    return _nib(B[b], x)


def test_fused_crc_algebra_all_lengths_and_alignments():
    rng = np.random.default_rng(5)
    lengths = list(range(0, 301)) + [1499, 1500, 1518, 1536, 1537, 3000, 9018]
    for Lt in lengths:
        for mis in range(8):
            buf = rng.integers(0, 256, mis + Lt + 24, dtype=np.uint8).tobytes()
            R = _fused_crc_register(buf, mis, Lt)
            frame = buf[mis:mis + Lt]
            if Lt >= 4:
                assert (~R & 0xFFFFFFFF) == zlib.crc32(frame), (Lt, mis)
            else:  # the kernel only tests the residue, which needs 4 bytes; the fold itself:
                assert ((~R ^ (0xFFFFFFFF >> (8 * Lt))) & 0xFFFFFFFF) == zlib.crc32(frame), (Lt, mis)


def test_fused_residue_of_frames_with_fcs():
    rng = np.random.default_rng(6)
    for Lt in (64, 65, 66, 67, 100, 1518):
        for mis in range(8):
            body = rng.integers(0, 256, Lt - 4, dtype=np.uint8).tobytes()
            frame = body + zlib.crc32(body).to_bytes(4, "little")
            buf = bytes(rng.integers(0, 256, mis, dtype=np.uint8)) + frame + bytes(rng.integers(0, 256, 16, dtype=np.uint8))
            assert (~_fused_crc_register(buf, mis, Lt) & 0xFFFFFFFF) == 0x2144DF1C
