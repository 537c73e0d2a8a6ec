"""The staged lane-stream schedule (tests/stage_algebra.py, the restatement of
stage_kernel.hip) against zlib on the host: resets by select, the ending
frame's Z_c, the byte-by-byte half for short and empty frames, and the carry
of frames that cross stretches (also frames longer than a stretch)."""
import random

import pytest

from tests import stage_algebra as S


def _case(seed, lens, lead):
    rng = random.Random(seed)
    off = [lead]
    for l in lens:
        off.append(off[-1] + l)
    return bytes(rng.getrandbits(8) for _ in range(off[-1] + 200)), off


def _lens(kind, rng):
    if kind == "zipf":
        from lneto_amd import synth
        return [int(x) for x in synth.zipf_lengths(400, seed=rng.randint(0, 99))]
    if kind == "tiny":
        return [rng.choice([0, 1, 2, 3, 4, 5, 7, 8, 13, 60, 64]) for _ in range(400)]
    if kind == "mixed":
        return [rng.randint(0, 2000) for _ in range(150)]
    return [rng.choice([5000, 9000, 64, 3, 0]) for _ in range(40)]  # frames longer than a stretch


@pytest.mark.parametrize("kind", ["zipf", "tiny", "mixed", "long"])
@pytest.mark.parametrize("lead", [0, 1, 3, 127])
def test_stage_schedule_matches_zlib(kind, lead):
    rng = random.Random(hash((kind, lead)) & 0xFFFF)
    data, off = _case(lead + 7, _lens(kind, rng), lead)
    want = S.zlib_crcs(data, off)
    for bf in (5, 64, 512):
        assert S.stage_crcs(data, off, bf=bf) == want, bf
    assert S.stage_crcs(data, off, bf=33, force_slow=True) == want


def test_reset_constants():
    """K_c = Z_{-c}(~0): c zero bytes forward give the CRC init back."""
    for c in range(4):
        assert S.zc(c, S.K[c]) == 0xFFFFFFFF


def test_block_ending_on_a_stretch_multiple():
    """A block whose span is exactly 64 Q under `64 Q >= span` left its last
    boundary outside every stretch (the 1 M Zipf GPU run lost one frame that
    way): Q is now the smallest line multiple with 64 Q > span."""
    from tests import stage_sim as SIM
    for lens, lead in (([128] * 64, 0), ([100] * 80 + [192], 0), ([64] * 127 + [64 + 127], 1)):
        data, off = _case(5, lens, lead)
        want = S.zlib_crcs(data, off)
        assert S.stage_crcs(data, off, bf=len(lens)) == want
        got = SIM.stage_block_sim(data, off, 0, len(lens), 0)
        assert [got.get(i) for i in range(len(lens))] == want


@pytest.mark.parametrize("kind", ["zipf", "tiny", "long"])
def test_wave_simulation_matches_zlib(kind):
    """tests/stage_sim.py follows the kernel's control flow (wave-uniform slow
    halves, held results, carries) and must give every frame of the block."""
    from tests import stage_sim as SIM
    rng = random.Random(len(kind))
    lens = _lens(kind, rng)[:120]
    data, off = _case(11, lens, 37)
    want = S.zlib_crcs(data, off)
    got = SIM.stage_block_sim(data, off, 0, len(lens), 0)
    assert [got.get(i) for i in range(len(lens))] == want


def test_slicing_by_8_unit_algebra():
    """FOLD 8 (variants 310 / 311): an 8-byte unit (w0, w1) entered with r
    leaves XOR_k T8_k[byte k of v0] ^ XOR_k T8_{4+k}[byte k of v1], T8_k[e] =
    Z_{8-k}(e), with v0 = r ^ w0 (or the reset value when a frame starts in w0)
    and v1 = w1 (or the reset value, the r side then dropped); the ending
    frame's pre-Z_c state is r ^ (w0 & lm) in w0 and Z_4(r ^ w0) ^ (w1 & lm) in
    w1; Z_c(e) = (e >> 8c) ^ XOR_{i<c} T8_{8-c+i}[byte i of e]."""
    rng = random.Random(88)
    T8 = [[S.zc(8 - k, e) for e in range(256)] for k in range(8)]

    def half(v, h):
        out = 0
        for k in range(4):
            out ^= T8[4 * h + k][(v >> (8 * k)) & 0xFF]
        return out

    for _ in range(3000):
        r, w0, w1 = (rng.getrandbits(32) for _ in range(3))
        # plain unit = two Z_4 steps
        assert half(r ^ w0, 0) ^ half(w1, 1) == S.z4(S.z4(r ^ w0) ^ w1)
        for where in (0, 1):
            c = rng.randrange(4)
            lm = (1 << (8 * c)) - 1
            w = w0 if where == 0 else w1
            vr = (w & ~lm & S.MASK) ^ S.K[c]
            if where == 0:
                got = half(vr, 0) ^ half(w1, 1)
                want = S.z4(S.z4(vr) ^ w1)
                e = r ^ (w0 & lm)
                e_ref = r ^ (w0 & lm)
            else:
                got = half(w1 if False else vr, 1)
                want = S.z4(vr)
                e = half(r ^ w0, 1) ^ (w1 & lm)
                e_ref = S.z4(r ^ w0) ^ (w1 & lm)
            assert got == want and e == e_ref
            zc = (e >> (8 * c)) if c else e
            for i in range(c):
                zc ^= T8[8 - c + i][(e >> (8 * i)) & 0xFF]
            assert zc == S.zc(c, e)


def test_deferred_boundary_correction():
    """Variants 312 / 313: a 64-byte half folded with no boundary select ends
    at r_plain; with a frame starting at byte c of dword d the true end state
    is r_plain ^ Z_{64-4d}(e ^ K_c), e = r_d ^ (w_d & lomask(c)) the ending
    frame's pre-Z_c state (r_d: the state before dword d)."""
    rng = random.Random(312)
    for _ in range(2000):
        r0 = rng.getrandbits(32)
        w = [rng.getrandbits(32) for _ in range(16)]
        d, c = rng.randrange(16), rng.randrange(4)
        lm = (1 << (8 * c)) - 1
        r, rd = r0, None
        for i in range(16):
            if i == d:
                rd = r
            r = S.z4(r ^ w[i])
        plain = r
        e = rd ^ (w[d] & lm)
        r = r0
        for i in range(16):
            r = S.z4(((w[i] & ~lm & S.MASK) ^ S.K[c]) if i == d else (r ^ w[i]))
        assert r == plain ^ S.zpow(64 - 4 * d, e ^ S.K[c])


def test_patched_boundary_word_half():
    """Variants 314 / 315: the boundary word patched once per half, p = (w_kb &
    ~lm) ^ K_c; unit u = kb >> 1 enters (p, w1) for a boundary in w0 and (0, p)
    for one in w1 (Z_8(0) = 0 drops r), every other unit (r ^ w0, w1).  The
    half's end state equals the dword-serial fold with the reset at dword kb,
    and the ending frame's pre-Z_c state comes from the captured r and the
    unit's two words re-read from the line."""
    rng = random.Random(314)
    T8 = [[S.zc(8 - k, e) for e in range(256)] for k in range(8)]

    def half(v, h):
        out = 0
        for k in range(4):
            out ^= T8[4 * h + k][(v >> (8 * k)) & 0xFF]
        return out

    for _ in range(2000):
        r0 = rng.getrandbits(32)
        w = [rng.getrandbits(32) for _ in range(16)]
        kb, c = rng.randrange(16), rng.randrange(4)
        lm = (1 << (8 * c)) - 1
        odd, ub = kb & 1, kb >> 1
        p = (w[kb] & ~lm & S.MASK) ^ S.K[c]
        r, rc = r0, 0
        for u in range(8):
            w0, w1 = w[2 * u], w[2 * u + 1]
            au = u == ub
            rc = r if au else rc
            v0 = (0 if odd else p) if au else r ^ w0
            v1 = p if (au and odd) else w1
            r = half(v0, 0) ^ half(v1, 1)
        # the dword-serial fold with the reset at dword kb
        rs, e_ref = r0, None
        for i in range(16):
            if i == kb:
                e_ref = rs ^ (w[i] & lm)
                rs = S.z4(p)
            else:
                rs = S.z4(rs ^ w[i])
        assert r == rs
        wx, wy = w[2 * ub], w[2 * ub + 1]
        e = (half(rc ^ wx, 1) ^ (wy & lm)) if odd else rc ^ (wx & lm)
        assert e == e_ref


def test_two_chain_half():
    """Variants 316 / 317: the half as chain A (units 0-3, from r) and chain B
    (units 4-7, from 0), r = Z_32(A) ^ B, or B alone when the boundary lies in
    B; a boundary in B captures B's local state, the true one adds
    Z_{8(u-4)}(A)."""
    rng = random.Random(316)
    T8 = [[S.zc(8 - k, e) for e in range(256)] for k in range(8)]

    def half(v, h):
        out = 0
        for k in range(4):
            out ^= T8[4 * h + k][(v >> (8 * k)) & 0xFF]
        return out

    def unit(r, w0, w1, au, odd, p):
        v0 = (0 if odd else p) if au else r ^ w0
        return half(v0, 0) ^ half(p if (au and odd) else w1, 1)

    for _ in range(2000):
        r0 = rng.getrandbits(32)
        w = [rng.getrandbits(32) for _ in range(16)]
        kb, c = rng.randrange(16), rng.randrange(4)
        lm = (1 << (8 * c)) - 1
        odd, ub = kb & 1, kb >> 1
        p = (w[kb] & ~lm & S.MASK) ^ S.K[c]
        ra, rb, rc = r0, 0, 0
        for u in range(4):
            if u == ub:
                rc = ra
            elif u + 4 == ub:
                rc = rb
            ra = unit(ra, w[2 * u], w[2 * u + 1], u == ub, odd, p)
            rb = unit(rb, w[8 + 2 * u], w[9 + 2 * u], u + 4 == ub, odd, p)
        inb = ub >= 4
        r = rb if inb else S.zpow(32, ra) ^ rb
        rct = rc ^ S.zpow(8 * (ub - 4), ra) if inb else rc
        rs, e_ref = r0, None
        for i in range(16):
            if i == kb:
                e_ref = rs ^ (w[i] & lm)
                rs = S.z4(p)
            else:
                rs = S.z4(rs ^ w[i])
        assert r == rs
        wx, wy = w[2 * ub], w[2 * ub + 1]
        e = (half(rct ^ wx, 1) ^ (wy & lm)) if odd else rct ^ (wx & lm)
        assert e == e_ref
