#!/usr/bin/env python3
"""Flag loops with a DIVERGENT exit whose body issues vector memory loads.

The sum16 line-row kernel of round 1 looped to each row's own line count: the
structurizer turned that into a loop whose latch retires finished lanes with
`s_andn2_b64 exec, exec, sN` and branches back on `s_cbranch_execnz` (or
leaves on `s_cbranch_execz`), with exec-masked global_load_dwordx2 in the
body; on MI355X it returned wrong sums for ~1 % of the segments of workgroups
256 and up, differently each launch.  The same loop bounded
by a wave-uniform count never failed.  No product kernel may contain that
shape: this audit lists, per kernel symbol, every INNERMOST loop (the text
between a backward branch's target label and the branch, holding no other
loop) that both narrows exec with s_andn2_b64 exec and issues a multi-dword
VMEM load.  The same structure with single-dword loads (sum16's half-line
rows) and multi-dword loads in a wave-uniform loop (the shipped line rows)
never failed, so neither is flagged; outer grid-stride loops are not
innermost.

usage: audit_loops.py file.s [symbol-regex]   (exit 1 if any loop is flagged)
"""
import re
import sys

VMEM_LOAD = re.compile(r"^(global_load|buffer_load|flat_load)_dwordx[234]")


def kernels(lines):
    """(symbol, first line, last line) of every function body in the .s."""
    out = []
    for i, l in enumerate(lines):
        m = re.match(r"^(_Z\w+):", l)
        if m:
            j = next(k for k in range(i, len(lines)) if lines[k].strip().startswith("s_endpgm"))
            out.append((m.group(1), i, j))
    return out


def divergent_load_loops(body):
    """[(label, loads, latch text)] for loops with an exec-narrowing latch and loads inside."""
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    back = []  # (header line, latch line) of every backward branch
    for i, l in enumerate(body):
        m = re.match(r"^s_cbranch_\w+\s+(\.LBB\w+)", l) or re.match(r"^s_branch\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] <= i:
            back.append((labels[m.group(1)], i))
    found = []
    for start, i in back:
        if any(start < s2 and j2 <= i and (s2, j2) != (start, i) for s2, j2 in back):
            continue  # holds another loop: not innermost
        l = body[i]
        m = re.match(r"^s_c?branch\w*\s+(\.LBB\w+)", l)
        loop = body[start:i + 1]
        narrows = any(re.match(r"^s_andn2_b64 exec, exec,", t) for t in loop)
        loads = [t for t in loop if VMEM_LOAD.match(t)]
        if narrows and loads:
            found.append((m.group(1), len(loads), l))
    return found


def main():
    path = sys.argv[1]
    pat = re.compile(sys.argv[2]) if len(sys.argv) > 2 else None
    lines = [l.split(";")[0].strip() for l in open(path).read().split("\n")]
    bad = 0
    for sym, a, b in kernels(lines):
        if pat and not pat.search(sym):
            continue
        for lab, nl, latch in divergent_load_loops(lines[a:b + 1]):
            print(f"{sym}: loop at {lab} narrows exec and issues {nl} VMEM loads (latch: {latch})")
            bad += 1
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
