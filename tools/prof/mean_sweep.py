#!/usr/bin/env python3
"""Crossover of the two CRC-32 kernels by mean frame length (round 5,
DESIGN.md §3.10): for each length mix, about BUDGET bytes of frames are timed
through the rows kernel (short_frames=False: the round-4 lnx_crc32_batch) and
the staged kernel (LNX_BATCH_SHORT_FRAMES), median of R
round-robin launches each bracketed by HIP events.

Mixes: fixed L; uniform [64, 2 L - 64] (mean L); the Zipf mix scaled so its
mean is L (lengths clipped to [64, 9000]).  One JSON line per (mix, L).
Not part of the product.  usage: mean_sweep.py [--budget-gb 2] [--reps 7]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--budget-gb", type=float, default=2.0)
    ap.add_argument("--reps", type=int, default=7)
    ap.add_argument("--lengths", default="64,96,128,192,256,320,384,448,512,640,768,1024,1500")
    ap.add_argument("--mixes", default="fixed,uniform,zipf")
    args = ap.parse_args()
    import torch
    import lneto_amd as L
    from lneto_amd import synth

    dev = torch.device("cuda:0")
    s = torch.cuda.current_stream(dev)
    rng = np.random.default_rng(5)
    zl = synth.zipf_lengths(1 << 20).astype(np.float64)
    for mix in args.mixes.split(","):
        for ln in [int(x) for x in args.lengths.split(",")]:
            n = int(args.budget_gb * 1e9 / ln)
            if mix == "fixed":
                lens = np.full(n, ln, dtype=np.int64)
            elif mix == "uniform":
                lens = rng.integers(64, 2 * ln - 64 + 1, n) if ln > 64 else np.full(n, 64)
            else:
                z = zl[rng.integers(0, len(zl), n)]
                lens = np.clip(np.rint(z * (ln / zl.mean())), 64, 9000).astype(np.int64)
            off = synth.offsets_from_lengths(lens)
            d = synth.bytes_torch(int(off[-1]), dev)
            o = torch.from_numpy(off.astype(np.int64)).to(dev)
            c = torch.empty(n, dtype=torch.int32, device=dev)
            forms = {"rows": False, "stage": True}
            ts = {k: [] for k in forms}
            for _ in range(3):
                for k, sf in forms.items():
                    L.crc32_batch(d, o, out=c, stream=s, short_frames=sf)
            for _ in range(args.reps):
                for k, sf in forms.items():
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(s)
                    L.crc32_batch(d, o, out=c, stream=s, short_frames=sf)
                    b.record(s)
                    b.synchronize()
                    ts[k].append(a.elapsed_time(b))
            nb = int(off[-1])
            rec = {"mix": mix, "mean": round(nb / n, 1), "L": ln, "frames": n, "bytes": nb}
            for k in forms:
                ms = float(np.median(ts[k]))
                rec[k + "_ms"] = round(ms, 4)
                rec[k + "_frac"] = round(nb / (ms * 1e-3) / 8e12, 4)
            rec["stage_over_rows"] = round(rec["stage_ms"] / rec["rows_ms"], 4)
            print(json.dumps(rec), flush=True)
            del d, o, c
            torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
