"""CPU emulation of the segment-lane CRC32Search kernels' algebra
(lneto_amd/csrc/search_kernel.hip: crc32_search_seg_kernel, 64 lanes x 24 B,
six-step scan; crc32_search_half_kernel / crc32_search_u_kernel, 32 lanes x 48 B
per capture, five-step scan, pass A all through Z_4, and the r2 product's pass B
by word checks, WB).

The kernels answer ethernet.CRC32Search (ethernet/crc.go:28-47) for one
capture per wave (or half-wave), in blocks of LANES lane segments of SEG bytes:
  pass A  l_j  = segment j folded from register 0 (lane 0 also Z_SEG(carry)),
          its first kSearchZWords words through Z_4, the rest byte by byte,
  scan    P_j  = XOR_{i<=j} Z_{SEG*(j-i)}(l_i) by log2(LANES) doubling steps with the
               Z_{SEG*2^k} tables,
  pass B  from P_{j-1} (lane 0: the carry) the register after every byte,
          tested against the residue register 0xDEBB20E3.
This restates that schedule in Python, with the kernel's segment size and its
treatment of bytes past the capture end, and checks it against the
Go-semantics oracle. It pins the scan identity and the block carry on the CPU;
tests/test_search.py checks the kernel itself on the GPU.
"""
import struct

import numpy as np
import pytest

from oracle import oracle as O

RESIDUE = 0xDEBB20E3
# (SEG, LANES, KZ): kSearchSeg / 64 lanes / kSearchZWords, and kHalfSeg / 32 lanes / all 12 words
SCHEDULES = [(24, 64, 2, False), (48, 32, 12, False), (48, 32, 12, True)]

_T = []
for _e in range(256):
    _c = _e
    for _ in range(8):
        _c = (_c >> 1) ^ (0xEDB88320 if _c & 1 else 0)
    _T.append(_c)


def _byte_step(r, b):
    return _T[(r ^ b) & 0xFF] ^ (r >> 8)


def _zshift(x, nbytes):
    """Z_n: the register after n zero bytes from register x (linear in x)."""
    for _ in range(nbytes):
        x = _byte_step(x, 0)
    return x


def _zshift_table(nbytes):
    """Z_n through its four byte tables, as the kernel's LDS image holds it."""
    tabs = [[_zshift(e << (8 * m), nbytes) for e in range(256)] for m in range(4)]
    return lambda x: tabs[0][x & 0xFF] ^ tabs[1][(x >> 8) & 0xFF] ^ tabs[2][(x >> 16) & 0xFF] ^ tabs[3][x >> 24]


_Z4 = _zshift_table(4)
_ZLEVELS = {}


# Word-check pass B (r2 product): the register after k = 1..4 bytes of a word
# is Z_k(r ^ (w & lo_k)) and Z_k is a bijection, so it is the residue register
# exactly when r ^ (w & lo_k) == Z_{-k}(RESIDUE): four compares against
# constants per word, then r <- Z_4(r ^ w).
def _zback(x, nbytes):
    for _ in range(8 * nbytes):
        b = x >> 31
        t = (x ^ 0xEDB88320) if b else x
        x = ((t << 1) & 0xFFFFFFFF) | b
    return x


RESIDUE_BACK = [None] + [_zback(RESIDUE, k) for k in range(1, 5)]


def seg_search(data: bytes, min_off: int, SEG: int = 24, LANES: int = 64, KZ: int = 2, WB: bool = False) -> int:
    nlev = LANES.bit_length() - 1
    if SEG not in _ZLEVELS:
        _ZLEVELS[SEG] = [_zshift_table(SEG << k) for k in range(6)]
    _ZLEVEL = _ZLEVELS[SEG]
    L = len(data)
    m = max(min_off, 0)
    if L < m + 4:
        return -1
    carry = 0xFFFFFFFF
    for B in range(0, L, LANES * SEG):
        segs = []
        for j in range(LANES):
            seg = data[B + SEG * j: B + SEG * (j + 1)]
            segs.append(seg + bytes(SEG - len(seg)))   # past the end: any bytes (zeros here)
        # pass A: the first KZ words with Z_4, the rest byte by byte
        l = []
        for j, seg in enumerate(segs):
            v = 0
            for wi, w in enumerate(struct.unpack("<%dI" % (SEG // 4), seg)):
                if wi < KZ:
                    v = _Z4(v ^ w)
                else:
                    for q in range(4):
                        v = _byte_step(v, (w >> (8 * q)) & 0xFF)
            if j == 0:
                v ^= _ZLEVEL[0](carry)
            l.append(v)
        # scan: P holds lanes (j - 2^k, j] after step k
        P = list(l)
        for k in range(nlev):
            d = 1 << k
            P = [P[j] ^ (_ZLEVEL[k](P[j - d]) if j >= d else 0) for j in range(LANES)]
        # pass B: first valid hit in (lane, byte) order
        for j, seg in enumerate(segs):
            r = carry if j == 0 else P[j - 1]
            base = B + SEG * j
            if WB:
                for wi, w in enumerate(struct.unpack("<%dI" % (SEG // 4), seg)):
                    for kk in range(1, 5):
                        k = base + 4 * wi + kk
                        lo = 0xFFFFFFFF >> (32 - 8 * kk)
                        if r ^ (w & lo) == RESIDUE_BACK[kk] and m + 4 <= k <= L:
                            return k - 4
                    r = _Z4(r ^ w)
                continue
            for i, b in enumerate(seg):
                r = _byte_step(r, b)
                k = base + i + 1   # bytes consumed
                if r == RESIDUE and m + 4 <= k <= L:
                    return k - 4
        carry = P[LANES - 1]
    return -1


def oct_search(data: bytes, min_off: int) -> int:
    """crc32_search_o_kernel (research, LNX_PROF_SEARCH=o): 8 lanes x 192 bytes
    per 1536-byte block; each lane folds four 48-byte chains from 0 (la_c),
    joins them by Horner with Z_48, the 3-level scan uses Z_{192*2^k}, pass B
    enters chain c + 1 at Z_48(r_c) ^ la_c and checks words; each lane keeps its
    smallest valid hit byte and the first lane with a hit answers."""
    SEG, LANES, CW = 192, 8, 12
    if SEG not in _ZLEVELS:
        _ZLEVELS[SEG] = [_zshift_table(SEG << k) for k in range(3)]
    zl = _ZLEVELS[SEG]
    z48 = _ZLEVELS.setdefault("z48", _zshift_table(48))
    L = len(data)
    m = max(min_off, 0)
    if L < m + 4:
        return -1
    carry = 0xFFFFFFFF
    for B in range(0, L, LANES * SEG):
        words, la, l = [], [], []
        for j in range(LANES):
            seg = data[B + SEG * j: B + SEG * (j + 1)]
            w = struct.unpack("<48I", seg + bytes(SEG - len(seg)))
            words.append(w)
            las = []
            for ch in range(4):
                x = w[CW * ch]
                for i in range(CW - 1):
                    x = _Z4(x) ^ w[CW * ch + i + 1]
                las.append(_Z4(x))
            p = las[0]
            for ch in range(1, 4):
                p = z48(p) ^ las[ch]
            if j == 0:
                p ^= zl[0](carry)
            la.append(las)
            l.append(p)
        P = list(l)
        for k in range(3):
            d = 1 << k
            P = [P[j] ^ (zl[k](P[j - d]) if j >= d else 0) for j in range(LANES)]
        for j in range(LANES):
            base = B + SEG * j
            r = [carry if j == 0 else P[j - 1]]
            for ch in range(1, 4):
                r.append(z48(r[ch - 1]) ^ la[j][ch - 1])
            best = None
            for i in range(CW):
                for ch in range(4):
                    wi = CW * ch + i
                    w = words[j][wi]
                    for kk in range(1, 5):
                        lo = 0xFFFFFFFF >> (32 - 8 * kk)
                        bi = 4 * wi + kk - 1
                        if r[ch] ^ (w & lo) == RESIDUE_BACK[kk] and m + 4 <= base + bi + 1 <= L:
                            best = bi if best is None else min(best, bi)
                    r[ch] = _Z4(r[ch] ^ w)
            if best is not None:
                return base + best + 1 - 4
        carry = P[LANES - 1]
    return -1


def test_oct_schedule_matches_oracle():
    rng = np.random.default_rng(37)
    cases = []
    for n in [0, 3, 4, 5, 47, 48, 49, 191, 192, 193, 1499, 1536, 1537, 3100]:
        body = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        cases.append((body, 0))
        cases.append((body + struct.pack("<I", O.crc32(body)), 0))
        cases.append((body + struct.pack("<I", O.crc32(body)) + body[:40], n))
        cases.append((body + struct.pack("<I", O.crc32(body)) + body[:40], n + 1))
    cases.append((b"\0\0\0\0" + bytes(100), 0))
    # hits straddling chains, lane segments and the block edge
    for cut in [44, 45, 46, 47, 92, 140, 141, 188, 189, 190, 191, 380, 1532, 1533, 1534, 1535, 1536, 3068]:
        body = rng.integers(0, 256, size=cut, dtype=np.uint8).tobytes()
        cases.append((body + struct.pack("<I", O.crc32(body)) + bytes(9), 0))
    for data, mo in cases:
        assert oct_search(data, mo) == O.crc32_search(data, mo), (len(data), mo)


def test_split_chain_identity():
    """crc32_search_u_kernel<NC, SPLIT>: a 48-byte segment folded as two
    24-byte chains joins as Z_24(la) ^ lb, and pass B's second chain starts from
    Z_24(r0) ^ la (la, lb: the halves folded from register 0)."""
    rng = np.random.default_rng(5)
    z24 = _zshift_table(24)
    for _ in range(200):
        seg = rng.integers(0, 256, size=48, dtype=np.uint8).tobytes()
        w = struct.unpack("<12I", seg)
        r0 = int(rng.integers(0, 1 << 32))
        la = lb = 0
        for x in w[:6]:
            la = _Z4(la ^ x)
        for x in w[6:]:
            lb = _Z4(lb ^ x)
        full = 0
        for x in w:
            full = _Z4(full ^ x)
        assert z24(la) ^ lb == full
        r = r0
        for x in w[:6]:
            r = _Z4(r ^ x)
        assert z24(r0) ^ la == r


def test_residue_back_constants():
    for k in range(1, 5):
        assert _zshift(RESIDUE_BACK[k], k) == RESIDUE


@pytest.mark.parametrize("seg,lanes,kz,wb", SCHEDULES)
def test_seg_schedule_matches_oracle(seg, lanes, kz, wb):
    rng = np.random.default_rng(31)
    cases = []
    for n in [0, 3, 4, 5, 23, 24, 25, 1499, 1536, 1537, 3100]:
        body = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        cases.append((body, 0))
        cases.append((body + struct.pack("<I", O.crc32(body)), 0))
        cases.append((body + struct.pack("<I", O.crc32(body)) + body[:40], n))
        cases.append((body + struct.pack("<I", O.crc32(body)) + body[:40], n + 1))
    cases.append((b"\0\0\0\0" + bytes(100), 0))
    # hits straddling lane segments and the 1536-byte block edge
    for cut in [20, 21, 22, 23, 44, 45, 46, 47, 92, 1532, 1533, 1534, 1535, 1536, 3068]:
        body = rng.integers(0, 256, size=cut, dtype=np.uint8).tobytes()
        cases.append((body + struct.pack("<I", O.crc32(body)) + bytes(9), 0))
    for data, mo in cases:
        assert seg_search(data, mo, seg, lanes, kz, wb) == O.crc32_search(data, mo), (len(data), mo)
