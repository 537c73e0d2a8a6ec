#!/usr/bin/env python3
"""A/B of two builds of the library on one box: bench.py runs alternately
under LNETO_AMD_LIB=A and =B (separate processes, same arguments), REPS times
each; prints every line's kernel time (the host clock per step for the
host-memory ops) and the medians.

usage: lib_ab.py LIB_A LIB_B REPS [bench.py args ...]"""
import json
import os
import statistics
import subprocess
import sys

a, b, reps, rest = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:]
res = {a: [], b: []}
for r in range(reps):
    for lib in (a, b) if r % 2 == 0 else (b, a):
        env = dict(os.environ, LNETO_AMD_LIB=os.path.abspath(lib))
        out = subprocess.run([sys.executable, "-u", "bench.py", "--no-cpu-baseline", "--no-slice16m", *rest],
                             env=env, capture_output=True, text=True, timeout=300)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        if out.returncode != 0 or not line:
            print(out.stdout[-2000:], out.stderr[-2000:])
            sys.exit(1)
        d = json.loads(line[-1])
        r = d.get("roofline") or {}
        ms = r.get("kernel_ms", d["ms_per_step"])  # (host-memory ops: the host clock per step)
        res[lib].append(ms)
        print(f"{os.path.basename(lib):28s} ms {ms:.4f} frac {r.get('frac', 0):.4f} value {d['value']}", flush=True)
for lib, v in res.items():
    print(f"median {os.path.basename(lib):28s} {statistics.median(v):.4f} ms  ({' '.join(f'{x:.4f}' for x in v)})")
