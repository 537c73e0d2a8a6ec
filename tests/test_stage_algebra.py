"""The staged lane-stream schedule (tests/stage_algebra.py, the restatement of
crc32_stage.hip) against zlib on the host: resets by select, the ending
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
