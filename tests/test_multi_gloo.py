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


def test_bench_world2_on_cpu_ranks():
    """bench.py's N>1 control flow end to end on host cores: torch.distributed.run
    with 2 ranks, the gloo barrier and max-over-ranks (no RCCL), rank 0's one
    JSON line with the whole-job value.  LNETO_BENCH_CPU_RANKS swaps the device
    step for the library's host CRC so it runs without a GPU."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, LNETO_BENCH_CPU_RANKS="1", LNETO_BENCH_CPU_FRAMES="256")
    env.pop("LNETO_AMD_LIB", None)
    port = _free_port()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                        "--gpus", "2", "--steps", "4", "--warmup", "1", "--prewarm-s", "0"],
                       capture_output=True, text=True, timeout=240, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    js = json.loads(lines[0])
    assert js["n_gpus"] == 2 and js["steps"] == 4 and js["scaling"] == "weak"
    assert js["config"]["frames_per_gpu"] == 256 and js["config"]["bytes_per_gpu"] == 256 * 1500
    # whole-job value: both ranks' bytes over the max-over-ranks time
    assert abs(js["value"] - 2 * 256 * 1500 * 4 / (js["ms_per_step"] * 4e-3) / 2**30) < 0.02 * js["value"] + 1e-3
    assert "nccl" not in r.stderr.lower()
