"""CPU restatement of the staged lane-stream CRC-32 schedule (stage_kernel.hip;
DESIGN.md §3.9).  Test infrastructure: it checks the algebra the kernel uses,
on the host, against zlib (= Go hash/crc32 IEEE, the arithmetic of
ethernet.CRC32, lneto ethernet/crc.go:19-21).

A wave takes a BLOCK of BF consecutive frames, bytes [A, E).  From
A_al = A rounded down to 128 it cuts 64 STRETCHES of Q bytes (Q a multiple of
128, 64 Q >= E - A_al); lane k folds stretch k, [S_k, S_k + Q), serially, one
dword at a time, from register 0:

    r <- Z4(r ^ w)                                   (no boundary in the dword)

The block's boundaries are x_j = off[f0 + j], j = 0..BF: x_j ends frame
f0 + j - 1 (j >= 1) and starts frame f0 + j (j < BF).  At a boundary in the
dword at 4d, byte c = x - 4d:

    e  = r ^ (w & lomask(c))          the ending frame's state is S = Z_c(e)
    r <- Z4((w & ~lomask(c)) ^ K_c)   K_c = Z_{-c}(0xFFFFFFFF): the new frame's
                                      state after the dword, from the CRC init

so a frame that starts and ends in one stretch has CRC ~S with no length
operator.  The fast path takes one boundary per 64-byte half; a half where
some lane has two or more (frames under 64 bytes, empty frames) runs byte by
byte (r <- Z1(r ^ b), r = ~0 at a frame start).

A stretch starts inside a frame: its first boundary's S is local (from 0 at
S_k).  After the block, with E_k the register at the stretch end and P_k the
true register at S_k of the frame open there,

    P_k = E_{k-1}                      if stretch k-1 has a boundary
          Z_Q(P_{k-1}) ^ E_{k-1}       else (a frame longer than a stretch)
    S  <- S ^ Z_d(P_k),  d = x - S_k   (Z_d: binary powers Z_{2^m})
"""
from __future__ import annotations

import zlib

POLY = 0xEDB88320
MASK = 0xFFFFFFFF
LINE = 128
HALF = 64

T1 = []
for _n in range(256):
    _c = _n
    for _ in range(8):
        _c = (_c >> 1) ^ (POLY if _c & 1 else 0)
    T1.append(_c)


def z1(v: int) -> int:
    return (v >> 8) ^ T1[v & 0xFF]


def zc(c: int, v: int) -> int:
    for _ in range(c):
        v = z1(v)
    return v


def z4(v: int) -> int:
    return z1(z1(z1(z1(v))))


def unz1(r: int) -> int:
    """Inverse of z1 (one zero byte backwards)."""
    for _ in range(8):
        b = r >> 31
        t = r ^ POLY if b else r
        r = ((t << 1) & MASK) | b
    return r


K = [MASK]
for _c in range(1, 4):
    K.append(unz1(K[-1]))  # K_c = Z_{-c}(~0)


def zpow(d: int, v: int) -> int:
    """Z_d(v) by binary powers, as the kernel's carry step."""
    m = 0
    while d >> m:
        if (d >> m) & 1:
            v = zc(1 << m, v)
        m += 1
    return v


def lomask(c: int) -> int:
    return (1 << (8 * c)) - 1


def stage_block(data: bytes, off, f0: int, bf: int, q: int, force_slow: bool = False, out=None):
    """CRCs of frames f0 .. f0 + bf - 1 (into `out`, a dict frame -> crc)."""
    out = {} if out is None else out
    a, e = off[f0], off[f0 + bf]
    a_al = a - (a % LINE)
    assert q % LINE == 0 and 64 * q > e - a_al
    bnd = [off[f0 + j] - a_al for j in range(bf + 1)] + [MASK]  # relative, sentinel
    nbytes = len(data)

    def word(p):  # little-endian dword at relative position p (0 past the buffer)
        g = a_al + p
        return int.from_bytes(data[g:g + 4].ljust(4, b"\0"), "little") if g < nbytes else 0

    def byte(p):
        g = a_al + p
        return data[g] if g < nbytes else 0

    lanes = []
    for k in range(64):
        s_k = k * q
        j = next(i for i, x in enumerate(bnd) if x >= s_k)
        r, first, rec, has_b = 0, True, None, False

        def end(jj, st):
            nonlocal first, rec
            if jj == 0:
                first = False
                return
            if first:
                rec = (jj, st, bnd[jj] - s_k)
                first = False
            else:
                out[f0 + jj - 1] = st ^ MASK

        for p in range(s_k, s_k + q, HALF):
            nb = sum(1 for x in bnd if p <= x < p + HALF)
            if nb >= 2 or force_slow:
                for b in range(HALF):
                    while bnd[j] == p + b:
                        has_b = True
                        end(j, r)
                        if j < bf:
                            r = MASK
                        j += 1
                    r = z1(r ^ byte(p + b))
                continue
            kb = c = -1
            if nb == 1:
                kb, c = (bnd[j] - p) >> 2, (bnd[j] - p) & 3
            ecap = 0
            for d in range(16):
                w = word(p + 4 * d)
                if d == kb:
                    ecap = r ^ (w & lomask(c))
                    r = z4((w & ~lomask(c) & MASK) ^ K[c]) if j < bf else z4(r ^ w)
                else:
                    r = z4(r ^ w)
            if nb == 1:
                has_b = True
                end(j, zc(c, ecap))
                j += 1
        lanes.append((r, has_b, rec))
    # carries
    p_in = [0] * 64
    for k in range(1, 64):
        e_prev, hb_prev, _ = lanes[k - 1]
        p_in[k] = e_prev if hb_prev else zpow(q, p_in[k - 1]) ^ e_prev
    for k in range(64):
        rec = lanes[k][2]
        if rec:
            jj, st, d = rec
            out[f0 + jj - 1] = (st ^ zpow(d, p_in[k])) ^ MASK
    return out


def stage_crcs(data: bytes, off, bf: int = 512, force_slow: bool = False):
    """Every frame's CRC by the staged schedule: blocks of bf frames, each with
    the smallest Q (a multiple of 128) that covers it."""
    n = len(off) - 1
    out = {}
    for f0 in range(0, n, bf):
        b = min(bf, n - f0)
        a, e = off[f0], off[f0 + b]
        span = e - (a - a % LINE)
        q = max(LINE, -(-span // 64 // LINE) * LINE) if span else LINE
        while 64 * q <= span:  # the last boundary (at span) must lie inside a stretch
            q += LINE
        stage_block(data, off, f0, b, q, force_slow, out)
    return [out[i] for i in range(n)]


def zlib_crcs(data: bytes, off):
    return [zlib.crc32(data[off[i]:off[i + 1]]) for i in range(len(off) - 1)]
