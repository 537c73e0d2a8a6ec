"""The library's per-stream state: the staged kernel's giant-slice
scratch and the staged launch's flag word are per stream, zeroed on that
stream when made, keyed per thread for hipStreamPerThread, and at most 32 live
per device (the least recently used one freed after a device sync).  GPU
tests through the C-ABI against the C oracle (ethernet/crc.go:19-21)."""
import ctypes
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _giant_case(cuda, seed):
    """64 frames of 1 MiB + 3 (giant by mean: every workgroup of the staged
    launch folds pieces through the stream's scratch) and their oracle CRCs."""
    import torch
    from lneto_amd import synth
    from oracle import oracle as O
    off = synth.offsets_from_lengths(np.full(64, (1 << 20) + 3)).astype(np.uint64) + np.uint64(seed % 7)
    d = synth.bytes_torch(int(off[-1]) + 8, cuda, seed=seed)
    want = O.crc32_frames(d.cpu().numpy(), off, threads=8)
    return d, torch.from_numpy(off.astype(np.int64)).to(cuda), want


def test_gpu_more_streams_than_scratch_sets(cuda):
    """40 streams (more than the 32 scratch sets a device keeps) in turn, twice
    round: each call on its own stream is exact, through evictions."""
    import torch
    import lneto_amd as L
    d, o, want = _giant_case(cuda, 101)
    streams = [torch.cuda.Stream(device=cuda) for _ in range(40)]
    for rnd in range(2):
        outs = []
        for s in streams:
            with torch.cuda.stream(s):
                outs.append(L.crc32_batch(d, o, stream=s))
        torch.cuda.synchronize()
        for k, c in enumerate(outs):
            assert (c.cpu().numpy().view(np.uint32) == want).all(), (rnd, k)


def test_gpu_per_thread_default_stream(cuda):
    """hipStreamPerThread from two host threads at once: each thread's calls
    get their own scratch (the same handle names two streams), results exact."""
    import torch
    import lneto_amd as L
    cases = [_giant_case(cuda, 200 + t) for t in range(2)]
    outs = [torch.empty(64, dtype=torch.int32, device=cuda) for _ in range(2)]
    torch.cuda.synchronize()
    rcs = [[], []]

    def run(t):
        torch.cuda.set_device(cuda)
        d, o, _ = cases[t]
        for _ in range(20):
            rcs[t].append(L.lib.lnx_crc32_batch(ctypes.c_void_p(d.data_ptr()), ctypes.c_void_p(o.data_ptr()), 64,
                                                ctypes.c_void_p(outs[t].data_ptr()), ctypes.c_void_p(2)))
        torch.cuda.synchronize()

    th = [threading.Thread(target=run, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join()
    torch.cuda.synchronize()
    assert rcs[0] == [0] * 20 and rcs[1] == [0] * 20
    for t in range(2):
        assert (outs[t].cpu().numpy().view(np.uint32) == cases[t][2]).all(), t
