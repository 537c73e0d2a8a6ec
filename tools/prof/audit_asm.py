#!/usr/bin/env python3
"""Audit a gfx950 kernel's .s for reads of registers whose asm-issued load has
not been waited for (hipcc does not count asm loads: cdna_hip_programming.md
§5.7 item 1).

Model (straight-line approximation over the text, branch targets ignored):
  - every `global_load_dword* ... nt` (our streaming asm loads) and every other
    VMEM op is appended to an in-order VMEM queue; `s_waitcnt vmcnt(N)` retires
    all but the N youngest;
  - `s_load_*` destinations stay pending until `s_waitcnt lgkmcnt(0)`.
A read of a pending destination register is reported.

usage: audit_asm.py file.s [kernel-symbol-substring]
"""
import re
import sys


def regs(text):
    out = set()
    for t, a, b in re.findall(r"\b([vs])\[(\d+):(\d+)\]", text):
        out |= {f"{t}{x}" for x in range(int(a), int(b) + 1)}
    for t, a in re.findall(r"\b([vs])(\d+)\b", text):
        out.add(f"{t}{a}")
    return out


VMEM = ("global_load", "global_store", "buffer_load", "buffer_store", "global_atomic", "buffer_atomic")
NO_DST = ("s_cmp", "v_cmp", "s_bitcmp", "buffer_store", "global_store", "ds_write", "s_cbranch", "s_branch",
          "s_waitcnt", "s_nop", "s_barrier", "s_endpgm", "s_setprio", "s_sleep")


def audit(lines):
    vq = []        # list of (set(dst regs), line)
    pend_s = {}
    bad = []
    for i, l in enumerate(lines):
        t = l.split(";")[0].strip()
        if not t or t.startswith("."):
            continue
        op, _, ops = t.partition(" ")
        if op == "s_waitcnt":
            m = re.search(r"vmcnt\((\d+)\)", ops)
            if m:
                n = int(m.group(1))
                vq = vq[-n:] if n else []
            if "lgkmcnt(0)" in ops:
                pend_s = {}
            continue
        parts = [p.strip() for p in ops.split(",")] if ops else []
        dst = parts[0] if parts and not op.startswith(NO_DST) else ""
        srcs = ",".join(parts[1:]) if dst else ops
        pending_v = set().union(*[d for d, _ in vq]) if vq else set()
        for r in regs(srcs):
            if r in pending_v or r in pend_s:
                bad.append((i, t, r))
        if op.startswith(VMEM):
            d = regs(dst) if op.startswith(("global_load", "buffer_load")) else set()
            vq.append((d, i))
        elif op.startswith("s_load") or op.startswith("s_buffer_load"):
            for r in regs(dst):
                pend_s[r] = i
        else:
            # a plain write to a register ends any pending state for it
            for r in regs(dst):
                pend_s.pop(r, None)
    return bad


def main():
    path = sys.argv[1]
    sym = sys.argv[2] if len(sys.argv) > 2 else None
    text = open(path).read().split("\n")
    if sym:
        start = next(i for i, l in enumerate(text) if l.startswith(sym) or (sym in l and l.rstrip().endswith(":") and not l.startswith("\t")))
        end = next(i for i in range(start, len(text)) if "s_endpgm" in text[i])
        text = text[start:end + 1]
    bad = audit(text)
    for i, t, r in bad[:30]:
        print(f"line {i}: reads pending {r}: {t}")
    print(f"{len(bad)} pending-register reads")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
