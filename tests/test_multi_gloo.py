"""Multi-GPU path, rehearsed on CPU: per-rank frame partition with no data-path
collective.  world_size 2 over gloo on 127.0.0.1; each rank
computes its contiguous slice with the oracle and the gathered result must equal
the single-process result.  The same shard_range() drives bench.py."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from bench import shard_range


@pytest.mark.parametrize("n", [0, 1, 7, 16, 1000, 1 << 20])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
def test_shard_ranges_partition(n, world):
    covered = []
    for r in range(world):
        lo, hi = shard_range(n, world, r)
        assert 0 <= lo <= hi <= n
        covered.extend(range(lo, hi)) if n < 5000 else covered.append((lo, hi))
    if n < 5000:
        assert covered == list(range(n))
    else:
        assert covered[0][0] == 0 and covered[-1][1] == n
        assert all(a[1] == b[0] for a, b in zip(covered, covered[1:]))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from lneto_amd import synth
    from oracle import oracle as O
    n = 3001
    off = synth.offsets_from_lengths(synth.zipf_lengths(n))
    data = synth.bytes_np(int(off[-1]))
    lo, hi = shard_range(n, world, rank)
    local = O.crc32_frames(data[int(off[lo]):int(off[hi])], off[lo:hi + 1] - off[lo])
    per = (n + world - 1) // world
    buf = torch.zeros(per, dtype=torch.int64)
    buf[: hi - lo] = torch.from_numpy(local.astype(np.int64))
    gathered = [torch.zeros(per, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(gathered, buf)  # result collection for the test only, not a data-path step
    t = torch.tensor([float(rank + 1)])
    dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the bench's max-over-ranks timing reduction
    if rank == 0:
        full = np.concatenate([g.numpy() for g in gathered])[:n].astype(np.uint32)
        q.put((full.tolist(), O.crc32_frames(data, off).tolist(), float(t.item())))
    dist.destroy_process_group()


def test_world2_partition_matches_single_process():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got, want, tmax = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got == want
    assert tmax == 2.0
