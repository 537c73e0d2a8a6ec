"""CPU restatement of the streaming-row CRC-32 schedule (crc32_kernel.hip
stream_body).  Test infrastructure: it checks the algebra the
kernel's streaming rows use, on the host, against zlib (= Go hash/crc32 IEEE,
the arithmetic of ethernet.CRC32, lneto ethernet/crc.go:19-21).

A row of RL = 8 lanes streams a contiguous run of frames one 128-byte line per
step; lane p holds the 16 bytes [L + 16p, L + 16p + 16) of line L.  Each lane
keeps ONE register r, its share of the running CRC state of the row's byte
stream, positioned at the start of its next piece: per step

    y0 = r ^ w0,  y1 = Z4(y0) ^ w1,  y2 = Z4(y1) ^ w2,  y3 = Z4(y2) ^ w3,
    ra = Z116(y3)                        (116 = the 112 bytes of the other lanes + 4)

Frame boundaries ("events") are positions x inside the line.  The stream's
state at x is combined from the lanes (rel = x - L, p_e = rel >> 4, k = (rel >> 2)
& 3, c = rel & 3):

    lane p <  p_e : ra   (its piece is before x)   column n = 4((p - p_e) & 7) - k
    lane p >  p_e : r    (its piece is after x)    column n = 4(p - p_e) - k
    lane p == p_e : y_k ^ (w_k & ~lomask(c))       column 0 (identity)

    O = XOR_p Z_{-4 n_p}(value_p)       (the state at X = L + 16 p_e + 4k, with the
                                          c data bytes [X, x) XOR-ed in)
    S = Z_c(O)                          (the state at x)

An event that ends a frame stores CRC = ~S.  An event that starts a frame
injects V = ~S at x: lane p_e's ra gets Z_{128 - (rel & 15)}(V) = Z_{128-4k}(O) ^
Z_{128 - (rel & 15)}(0xFFFFFFFF), after which the stream's state at x is
0xFFFFFFFF, the CRC init; so the next frame's CRC needs no per-frame length
operator, and junk before a row's first frame cancels.

Two events in one lane piece (frames shorter than 16 bytes): the later one
uses the chain values from before the earlier one's injection; a row-uniform
accumulator P (the injections of this piece, positioned at the last event)
adds Z_{x - x_prev}(P) to its state.
"""
from __future__ import annotations

import zlib

POLY = 0xEDB88320
MASK = 0xFFFFFFFF


def zbit(r: int) -> int:
    return (r >> 1) ^ (POLY if r & 1 else 0)


def unzbit(r: int) -> int:
    b = r >> 31
    t = r ^ POLY if b else r
    return ((t << 1) & MASK) | b


def Z(k: int, r: int) -> int:
    """Advance the reflected CRC register over k zero bytes (k < 0: back)."""
    if k >= 0:
        for _ in range(8 * k):
            r = zbit(r)
    else:
        for _ in range(-8 * k):
            r = unzbit(r)
    return r


_ZC: dict = {}


def Zt(k: int, r: int) -> int:
    """Z_k through byte tables (as the kernel's LDS tables would), cached per k."""
    t = _ZC.get(k)
    if t is None:
        t = [[Z(k, e << (8 * m)) for e in range(256)] for m in range(4)]
        _ZC[k] = t
    return t[0][r & 255] ^ t[1][(r >> 8) & 255] ^ t[2][(r >> 16) & 255] ^ t[3][r >> 24]


def lomask(c: int) -> int:
    return (1 << (8 * c)) - 1


def stream_row(data: bytes, events: list[int], RL: int = 8) -> list[int]:
    """CRCs of the frames [events[i], events[i+1]) of one row, by the streaming
    schedule with RL lanes per row (row steps of LINE = 16 RL bytes: 8 lanes,
    one 128-byte line; 4 lanes, a 64-byte half line).  data: the whole buffer
    (reads past its end are 0)."""
    LINE = 16 * RL
    m = len(events) - 1
    out = []
    if m < 0:
        return out
    L = events[0] & ~(LINE - 1)
    r = [0] * RL
    k = 0
    last = events[-1]

    def word(pos: int) -> int:
        b = data[pos:pos + 4]
        b = b + bytes(4 - len(b)) if len(b) < 4 else b
        return int.from_bytes(b, "little")

    while k <= m:
        w = [[word(L + 16 * p + 4 * i) for i in range(4)] for p in range(RL)]
        y = [[0] * 4 for _ in range(RL)]
        ra = [0] * RL
        for p in range(RL):
            y[p][0] = r[p] ^ w[p][0]
            y[p][1] = Zt(4, y[p][0]) ^ w[p][1]
            y[p][2] = Zt(4, y[p][1]) ^ w[p][2]
            y[p][3] = Zt(4, y[p][2]) ^ w[p][3]
            ra[p] = Zt(LINE - 12, y[p][3])
        piece_prev = -1  # lane piece of the previous event in this line
        x_prev = 0
        P = 0
        while k <= m and events[k] < L + LINE:
            x = events[k]
            rel = x - L
            pe, ke, c = rel >> 4, (rel >> 2) & 3, rel & 3
            O = 0
            for p in range(RL):
                if p < pe:
                    v, n = ra[p], 4 * ((p - pe) % RL) - ke
                elif p > pe:
                    v, n = r[p], 4 * (p - pe) - ke
                else:
                    v, n = y[p][ke] ^ (w[p][ke] & ~lomask(c) & MASK), 0
                O ^= Z(-4 * n, v)
            if piece_prev == pe:  # slow path: an earlier event in this piece
                O ^= Z(-c, Z(x - x_prev, P))  # (S gets Z_{x - x_prev}(P) after Z_c below)
            S = Z(c, O)
            if k >= 1:
                out.append(S ^ MASK)
            if k < m:
                V = S ^ MASK
                d = LINE - (rel & 15)
                G = Z(LINE - 4 * ke, O) ^ Z(d, MASK)
                if piece_prev == pe:
                    G = Z(d, V)  # Z_{128-4k}(O) no longer equals Z_d(S) on this path
                ra[pe] ^= G
                P = (Z(x - x_prev, P) if piece_prev == pe else 0) ^ V
                piece_prev, x_prev = pe, x
            k += 1
        r = ra
        L += LINE
        if L > last + LINE:
            break
    return out


def check(frames: list[bytes], lead: int = 0, RL: int = 8) -> None:
    buf = bytes(range(256)) * ((lead + 255) // 256)
    data = bytearray(buf[:lead])
    ev = [lead]
    for f in frames:
        data += f
        ev.append(len(data))
    data += bytes(range(7)) * 40  # junk after the run
    got = stream_row(bytes(data), ev, RL)
    want = [zlib.crc32(f) for f in frames]
    assert got == want, (got, want)


def lane_stream(data: bytes, events: list[int], SB: int = 64) -> list[int]:
    """CRCs of the frames [events[i], events[i+1]) by the lane-stream schedule
    (stream_lanes.hpp): ONE lane folds the run serially, SB bytes (the kernel:
    64) per superstep at q (SB-aligned), with no cross-lane combination:

        y0 = r ^ w0, y_i = Z4(y_{i-1}) ^ w_i (i < SB/4), r' = Z4(y_last)

    An event x in [q, q + SB) (cb = x - q, k = cb >> 2, c = cb & 3) reads the
    chain's uncorrected state there from e = y_k ^ (w_k & ~lomask(c)):
    S = Z_c(e); a frame start at x makes r' ^= Z_{SB-4k}(e) ^ Z_{SB-cb}(~0)
    (= Z_{SB-cb}(S ^ ~0): the stream's state at x becomes ~0).  Only the last
    start of a superstep corrects r' (the reset makes the earlier ones moot); a
    later event of the same superstep corrects its S by Z_{x - x'}(S' ^ ~0), S'
    the previous event's uncorrected state."""
    m = len(events) - 1
    out = []
    if m < 0:
        return out

    def word(pos: int) -> int:
        b = data[pos:pos + 4]
        b = b + bytes(4 - len(b)) if len(b) < 4 else b
        return int.from_bytes(b, "little")

    q = events[0] & ~63  # the lane's first superstep: 64-byte aligned
    r = 0
    k = 0
    nw = SB // 4
    while k <= m:
        w = [word(q + 4 * i) for i in range(nw)]
        y = [r ^ w[0]]
        for i in range(1, nw):
            y.append(Zt(4, y[i - 1]) ^ w[i])
        rn = Zt(4, y[-1])
        fix = 0
        first = True
        Sp = 0
        xp = 0
        while k <= m and events[k] < q + SB:
            x = events[k]
            cb = x - q
            kk, c = cb >> 2, cb & 3
            e = y[kk] ^ (w[kk] & ~lomask(c) & MASK)
            S = Zt(c, e) if c else e
            corr = Zt(SB - 4 * kk, e) ^ Z(SB - cb, MASK)
            St = S if first else S ^ Z(x - xp, Sp ^ MASK)
            if k >= 1:
                out.append(St ^ MASK)
            if k < m:
                fix = corr
            Sp, xp, first = S, x, False
            k += 1
        r = rn ^ fix
        q += SB
    return out


def check_lanes(frames: list[bytes], lead: int = 0, SB: int = 64) -> None:
    buf = bytes(range(256)) * ((lead + 255) // 256)
    data = bytearray(buf[:lead])
    ev = [lead]
    for f in frames:
        data += f
        ev.append(len(data))
    data += bytes(range(7)) * 40
    got = lane_stream(bytes(data), ev, SB)
    want = [zlib.crc32(f) for f in frames]
    assert got == want, (got, want)


if __name__ == "__main__":
    import random

    rnd = random.Random(1)
    for trial in range(300):
        lens = [rnd.choice([0, 1, 2, 3, 4, 5, 7, 15, 16, 17, 31, 63, 64, 65, 100, 127, 128, 129, 200, 1500])
                for _ in range(rnd.randint(1, 12))]
        frames = [bytes(rnd.getrandbits(8) for _ in range(n)) for n in lens]
        check(frames, lead=rnd.randint(0, 300), RL=rnd.choice([4, 8]))
        check_lanes(frames, lead=rnd.randint(0, 300), SB=rnd.choice([16, 64]))
    print("ok")
