"""Batched ethernet.CRC32Search (ethernet/crc.go:28-47), SURVEY.md §8(f).4:
lnx_crc32_search_batch against the golden cases (ethernet/crc_test.go shapes)
and the Go-semantics oracle on random captures with embedded FCS."""
import struct

import numpy as np
import pytest

from oracle import oracle as O

pytestmark = pytest.mark.gpu


def _run(cuda, caps, mins):
    import torch
    import lneto_amd as L
    offs = np.zeros(len(caps) + 1, dtype=np.int64)
    offs[1:] = np.cumsum([len(c) for c in caps])
    data = np.frombuffer(b"".join(caps) + b"\0" * 8, dtype=np.uint8).copy()
    d = torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(offs).to(cuda)
    m = torch.tensor(mins, dtype=torch.int64, device=cuda)
    return L.crc32_search_batch(d, o, m).cpu().numpy().tolist()


def test_golden_search_cases(cuda, golden):
    cases = golden["crc32_search_cases"]
    got = _run(cuda, [bytes.fromhex(c["data"]) for c in cases], [c["min_off"] for c in cases])
    assert got == [c["want"] for c in cases]


def test_random_captures(cuda):
    rng = np.random.default_rng(21)
    caps, mins = [], []
    for i in range(3000):
        kind = i % 6
        n = int(rng.integers(0, 2100))
        body = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        if kind in (0, 1, 2):  # a frame with its FCS, then trailing capture garbage
            cut = int(rng.integers(0, n + 1))
            cap = body[:cut] + struct.pack("<I", O.crc32(body[:cut])) + body[cut:cut + int(rng.integers(0, 64))]
        elif kind == 3:        # two valid FCS positions: the first one wins
            a = body[: n // 3]
            f1 = a + struct.pack("<I", O.crc32(a))
            cap = f1 + struct.pack("<I", O.crc32(f1)) + body[:10]
        elif kind == 4:        # leading zeros: off 0 matches CRC32(nil) == 0
            cap = b"\0\0\0\0" + body[:200]
        else:                  # no FCS anywhere (almost surely)
            cap = body
        caps.append(cap)
        mins.append(int(rng.choice([0, -5, 1, 3, len(cap) // 2, len(cap) - 4, len(cap) - 3, len(cap) + 10])))
    got = _run(cuda, caps, mins)
    want = [O.crc32_search(c, m) for c, m in zip(caps, mins)]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, [(i, len(caps[i]), mins[i], got[i], want[i]) for i in bad[:10]]


def test_long_captures_many_blocks(cuda):
    """Captures spanning several lane blocks (the register carried from block to
    block), hits in any block, including on block boundaries."""
    rng = np.random.default_rng(22)
    caps, mins = [], []
    for i in range(400):
        n = int(rng.integers(1500, 12000))
        body = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        if i % 4 == 3:  # FCS ending exactly on a multiple of 512 bytes
            cut = max(0, (int(rng.integers(0, n)) // 512) * 512 - 4)
        else:
            cut = int(rng.integers(0, n + 1))
        cap = body[:cut] + struct.pack("<I", O.crc32(body[:cut])) + body[cut:cut + int(rng.integers(0, 3000))]
        caps.append(cap)
        mins.append(int(rng.choice([0, 0, cut // 2, cut, cut + 1])))
    got = _run(cuda, caps, mins)
    want = [O.crc32_search(c, m) for c, m in zip(caps, mins)]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, [(i, len(caps[i]), mins[i], got[i], want[i]) for i in bad[:10]]


def test_two_captures_per_wave_pairs(cuda):
    """Captures share a wave (the r2 kernels fold one or two per 32-lane half,
    crc32_search_u_kernel<2> four per wave): pair a long capture (several 1536-byte blocks, hit
    late or never) with a short or empty one, in both orders, hits on the
    1536-byte block edges, and an odd capture count (the last wave's second
    half has no capture)."""
    rng = np.random.default_rng(23)
    caps, mins = [], []
    for i in range(301):
        long_first = i % 2 == 0
        n_long = int(rng.integers(3000, 9000))
        body = rng.integers(0, 256, size=n_long, dtype=np.uint8).tobytes()
        cut = (int(rng.integers(1, n_long // 1536 + 1)) * 1536 - 4) if i % 3 == 0 else int(rng.integers(0, n_long))
        long_cap = body[:cut] + struct.pack("<I", O.crc32(body[:cut])) + body[cut:]
        if i % 5 == 4:
            long_cap = body  # no hit: every block scanned
        short = rng.integers(0, 256, size=int(rng.integers(0, 80)), dtype=np.uint8).tobytes()
        if i % 7 == 0:
            short = short + struct.pack("<I", O.crc32(short))
        pair = [long_cap, short] if long_first else [short, long_cap]
        for c in pair:
            caps.append(c)
            mins.append(int(rng.choice([0, 2, len(c) // 3])))
    caps.append(b"\x01\x02\x03")
    mins.append(0)
    assert len(caps) % 2 == 1
    got = _run(cuda, caps, mins)
    want = [O.crc32_search(c, m) for c, m in zip(caps, mins)]
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, [(i, len(caps[i]), mins[i], got[i], want[i]) for i in bad[:10]]


def test_decreasing_offsets_take_the_guarded_loads(cuda):
    """a group of four captures that do not all lie inside
    [off[4q], off[4q + 4]) cannot use the group buffer descriptor and takes the
    per-capture guarded loads (search_kernel.hip, gfast false).  Captures laid
    out in reverse order: off = [a0, b0, a1, b1, ...] with a_{k+1} < b_k, so
    capture 2k = [a_k, b_k) is real and capture 2k + 1 (end below start) is
    empty, -1 (ethernet/crc.go:29-34)."""
    import torch
    import lneto_amd as L
    rng = np.random.default_rng(24)
    caps = []
    for i in range(600):
        body = rng.integers(0, 256, size=int(rng.integers(0, 1800)), dtype=np.uint8).tobytes()
        if i % 4 != 3:
            cut = int(rng.integers(0, len(body) + 1))
            body = body[:cut] + struct.pack("<I", O.crc32(body[:cut])) + body[cut:cut + int(rng.integers(0, 40))]
        caps.append(body)
    pad = 3
    blob = bytearray(b"\x5a" * pad)
    pos = {}
    for k in reversed(range(len(caps))):  # capture k sits before capture k - 1 in memory
        pos[k] = len(blob)
        blob += caps[k] + bytes(int(rng.integers(0, 5)))
    blob += b"\0" * 8
    offs, want, mins = [], [], []
    for k, c in enumerate(caps):
        offs += [pos[k], pos[k] + len(c)]
    offs = np.array(offs, dtype=np.int64)
    for i in range(len(offs) - 1):
        s, e = int(offs[i]), int(offs[i + 1])
        cap = bytes(blob[s:e]) if e > s else b""
        m = int(rng.choice([0, 1, len(cap) // 2]))
        mins.append(m)
        want.append(O.crc32_search(cap, m))
    assert sum(w >= 0 for w in want) > 300
    d = torch.from_numpy(np.frombuffer(bytes(blob), dtype=np.uint8).copy()).to(cuda)
    got = L.crc32_search_batch(d, torch.from_numpy(offs).to(cuda),
                               torch.tensor(mins, dtype=torch.int64, device=cuda)).cpu().numpy().tolist()
    bad = [i for i, (g, w) in enumerate(zip(got, want)) if g != w]
    assert not bad, [(i, got[i], want[i]) for i in bad[:10]]


@pytest.mark.parametrize("count", [1, 2, 3, 5, 6, 7, 257])
def test_four_captures_per_wave_groups(cuda, count):
    """crc32_search_u_kernel<2> folds captures 4q .. 4q + 3 in one wave (two
    per 32-lane half, side by side): every group size at the end of the batch,
    and groups whose four captures end in different 1536-byte blocks (the
    block loop runs until the last of them is done)."""
    rng = np.random.default_rng(100 + count)
    caps, mins = [], []
    for i in range(count):
        n_body = int(rng.choice([0, 3, 40, 1500, 1536, 3000, 4700]))
        body = rng.integers(0, 256, size=n_body, dtype=np.uint8).tobytes()
        if i % 3 != 2:
            cut = int(rng.integers(0, n_body + 1))
            body = body[:cut] + struct.pack("<I", O.crc32(body[:cut])) + body[cut:]
        caps.append(body)
        mins.append(int(rng.choice([0, 1, len(body) // 2])))
    got = _run(cuda, caps, mins)
    want = [O.crc32_search(c, m) for c, m in zip(caps, mins)]
    assert list(got) == want
