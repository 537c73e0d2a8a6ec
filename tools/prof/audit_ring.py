#!/usr/bin/env python3
"""Audit the CRC kernel's .s for hazards on the asm-loaded ring registers.

The destination register of a streaming `global_load_dword ... nt` (issued
by inline asm, invisible to hipcc's waitcnt pass) must not be read, copied or
reused by any compiler-emitted instruction while that load may still be in
flight: that would be a silent data race.  Checked in text order (which is the
hot path's execution order): after each load its register is "outstanding"
until a hand-written `s_waitcnt vmcnt(N)` retires it (all but the N youngest
loads retire); any instruction naming an outstanding register is reported.
usage: audit_ring.py file.s kernel-symbol
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


def vmem_dest(t):
    """(is a vmcnt event, destination registers) of an instruction.  On gfx9
    loads, returning atomics (sc0) and stores all count in vmcnt."""
    if t.startswith("buffer_load_dword") or (t.startswith("global_load_dword ") and t.endswith(" nt")):
        return True, regs(t.split(",")[0].split(None, 1)[1])
    if t.startswith("buffer_atomic_") and " sc0" in t:
        return True, regs(t.split(",")[0].split(None, 1)[1])
    if t.startswith("buffer_store") or t.startswith("global_store"):
        return True, set()
    return False, set()


def main():
    path, sym = sys.argv[1], sys.argv[2]
    lines = open(path).read().split("\n")
    start = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    body = [l.split(";")[0].strip() for l in lines[start:end + 1]]
    ring, first = set(), None
    for i, t in enumerate(body):
        ev, d = vmem_dest(t)
        if ev and d:
            ring |= d
            first = i if first is None else first
    bad = []
    # linear-order pending check: vmcnt(N) retires all but the N youngest loads
    seq, pending = [], set()
    for i, t in enumerate(body):
        if t.startswith("s_waitcnt") and "vmcnt(" in t:
            n = int(re.search(r"vmcnt\((\d+)\)", t).group(1))
            seq = seq[-n:] if n else []
            live = set().union(*seq) if seq else set()
            pending = {r for r in pending if r in live}
            continue
        ev, d = vmem_dest(t)
        if ev:
            # a later load of the same asm run whose offset VGPR is an earlier
            # load's destination (outputs not early-clobber): if the earlier
            # load returns before this one issues, the offset is garbage
            srcs = regs(t.partition(" ")[2].partition(",")[2]) if d else regs(t.partition(" ")[2])
            if srcs & pending:
                bad.append((i, t, "reads a register an outstanding load will overwrite"))
            pending |= d
            seq.append(frozenset(d))
            continue
        if not t or t.startswith("."):
            continue
        if regs(t.partition(" ")[2]) & pending:
            bad.append((i, t, "touches a ring register whose load is outstanding"))
    # descriptor hazard: a VALU write of an SGPR (v_readlane, v_readfirstlane,
    # v_cmp with SGPR dst, ...) needs 5 wait states before a VMEM reads it as a
    # descriptor; hipcc pads only instructions it can see, so every asm buffer
    # load must be preceded by an s_nop >= 4 (or >= 5 other instructions).
    for i, t in enumerate(body):
        if not (t.startswith("buffer_load_dword") or t.startswith("buffer_atomic_")):
            continue
        rs = regs(t.split(",")[2]) if len(t.split(",")) > 2 else set()
        waits = 0
        for j in range(i - 1, max(i - 8, -1), -1):
            u = body[j]
            if not u or u.startswith("."):
                continue
            if u.startswith("s_nop"):
                waits += int(u.split()[1]) + 1
            elif u.startswith("v_"):
                dst = u.partition(" ")[2].split(",")[0]
                if regs(dst) & rs and waits < 5:
                    bad.append((i, t, f"descriptor written by VALU {waits} wait states before: {u}"))
                waits += 1
            else:
                waits += 1
            if waits >= 5:
                break
    print(f"ring registers: {sorted(ring, key=lambda r: int(r[1:]))}")
    for i, t, why in bad[:20]:
        print(f"  {why}: {t}")
    print(f"{len(bad)} hazards")
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
