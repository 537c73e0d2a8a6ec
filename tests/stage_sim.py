"""Wave-level simulation of crc32_stage_kernel (stage_kernel.hip), statement by
statement: the wave-uniform choice between the fast and the byte-serial path
per half, the boundary registers (x, x1, xprev, j), end_at / advance, the held
results and their flushes, the stretch carries with the Jacobi sweep, and the
16-byte range check of the loads.  Test infrastructure (tests/stage_algebra.py
restates the algebra per lane; this follows the kernel's control flow)."""
from __future__ import annotations

from tests.stage_algebra import K, MASK, z1, z4, zpow

NONE = 0xFFFFFFFF


def stage_block_sim(data: bytes, off, f0: int, bf: int, base_mod128: int = 0, out=None):
    out = {} if out is None else out
    A, E = off[f0], off[f0 + bf]
    adj = (base_mod128 + A) & 127
    span = E - A + adj if E > A else adj
    sp = span
    Q = ((sp + 64) // 64 + 127) & ~127  # 64 Q > sp
    Q = max(Q, 128)
    rounds = Q // 128
    rng_end = (sp + 15) & ~15  # the descriptor's range
    lst = [NONE] * 384
    for j in range(384):
        if j <= bf:
            o = off[f0 + j]
            lst[j] = (o - A) + adj if o > A else adj
    a_al = A - adj
    nbytes = len(data)

    def word(rel):  # the loaded dword at relative byte rel (4-aligned)
        if rel + 4 > rng_end:
            return 0
        g = a_al + rel
        return int.from_bytes(data[g:g + 4].ljust(4, b"\0"), "little") if g < nbytes else 0

    class Lane:
        pass

    lanes = []
    for k in range(64):
        L = Lane()
        L.Sk = k * Q
        lo, hi = 0, bf + 1
        while lo < hi:
            mid = (lo + hi) >> 1
            if lst[min(mid, 383)] >= L.Sk:
                hi = mid
            else:
                lo = mid + 1
        L.jstart = L.j = lo
        L.x, L.x1 = lst[L.j], lst[min(L.j + 1, 383)]
        L.xprev = lst[L.j - 1] if L.j > 0 else 0
        L.r = 0
        L.first = True
        L.rec = False
        L.rec_j = L.rec_S = L.rec_d = 0
        L.hold = [None, None]
        lanes.append(L)

    def end_at(L, ev, S, xe, h):
        is_first = ev and L.first and L.j > 0
        if is_first:
            L.rec_j, L.rec_S, L.rec_d, L.rec = L.j, S, (xe - L.Sk) & MASK, True
        res = ev and not L.first and L.j > 0
        if ev:
            L.first = False
        if res:
            fr = f0 + L.j - 1
            if h == 2:
                out[fr] = S ^ MASK
            else:
                L.hold[h] = (fr, S ^ MASK)

    def advance(L, ev):
        if ev:
            L.xprev = L.x
            L.j += 1
            L.x = L.x1
        x2 = lst[min(L.j + 1, 383)]
        if ev:
            L.x1 = x2

    def flush():
        for L in lanes:
            for h in range(2):
                if L.hold[h] is not None:
                    fr, v = L.hold[h]
                    out[fr] = v
                    L.hold[h] = None

    for rr in range(rounds):
        flush()
        for h in range(2):
            P = [L.Sk + 128 * rr + 64 * h for L in lanes]
            if any(((L.x1 - P[k]) & MASK) < 64 for k, L in enumerate(lanes)):
                for b in range(64):
                    for k, L in enumerate(lanes):
                        w = word(P[k] + (b & ~3))
                        pos = P[k] + b
                        while L.x == pos:
                            end_at(L, True, L.r, L.x, 2)
                            L.r = MASK
                            advance(L, True)
                        L.r = z1(L.r ^ ((w >> (8 * (b & 3))) & 0xFF))
                continue
            for k, L in enumerate(lanes):
                rel = (L.x - P[k]) & MASK
                inn = rel < 64
                kb, c = (rel >> 2 if inn else 99), rel & 3
                lm = ((1 << (8 * c)) - 1) if inn else 0
                Kc = K[c]
                ecap = 0
                for d in range(16):
                    w = word(P[k] + 4 * d)
                    at = d == kb
                    if at:
                        ecap = L.r ^ (w & lm)
                        v = (w & ~lm & MASK) ^ Kc
                    else:
                        v = L.r ^ w
                    L.r = z4(v)
                if inn:
                    S = ecap
                    for s in range(3):
                        if s < c:
                            S = z1(S)
                    end_at(L, True, S, L.x, h)
                    advance(L, True)
    flush()
    # carries
    E1 = [L.r for L in lanes]
    hb = [L.j > L.jstart for L in lanes]
    Ep = [E1[(k + 63) & 63] for k in range(64)]
    hbp = [k == 0 or hb[(k + 63) & 63] for k in range(64)]
    Pk = list(Ep)
    if any(L.rec and not hbp[k] for k, L in enumerate(lanes)):
        for _ in range(64):
            Pp = [Pk[(k + 63) & 63] for k in range(64)]
            Pn = [Ep[k] if hbp[k] else zpow(Q, Pp[k]) ^ Ep[k] for k in range(64)]
            ch = any(Pn[k] != Pk[k] for k in range(64))
            Pk = Pn
            if not ch:
                break
    for k, L in enumerate(lanes):
        if L.rec:
            out[f0 + L.rec_j - 1] = (L.rec_S ^ zpow(L.rec_d, Pk[k])) ^ MASK
    return out
