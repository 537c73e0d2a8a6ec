"""Synthetic workload generators (BASELINE.md "Inputs"): host and device agree."""
import numpy as np
import torch

from lneto_amd import synth


def test_numpy_and_torch_bytes_agree():
    for n in [0, 1, 7, 8, 9, 1000, 123457]:
        a = synth.bytes_np(n)
        b = synth.bytes_torch(n, "cpu", chunk_words=1000).numpy()
        assert np.array_equal(a, b)


def test_splitmix_reference_values():
    # splitmix64 with state seed: first outputs for seed 0 (public reference values)
    w = synth.splitmix_words_np(0, 3, seed=0)
    assert [hex(int(x)) for x in w] == ["0xe220a8397b1dcdaf", "0x6e789e6aa1b965f4", "0x6c45d188009454f"]


def test_zipf_lengths_stats():
    L = synth.zipf_lengths(1 << 20)
    assert L.min() >= 64 and L.max() <= 1500
    assert abs(L.mean() - 246.1) < 1.5
    assert abs((L == 64).mean() - 0.127) < 0.003
    assert np.array_equal(L[:1000], synth.zipf_lengths(1000))  # deterministic prefix


def test_offsets():
    off = synth.offsets_from_lengths(np.array([3, 0, 5]))
    assert off.tolist() == [0, 3, 3, 8] and off.dtype == np.uint64
    assert synth.fixed_offsets(3, 1500).tolist() == [0, 1500, 3000, 4500]
