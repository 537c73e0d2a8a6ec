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
