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

Second check (round 4, the stale-register hypothesis of that failure): every
CROSS-LANE read -- a DPP operand (quad_perm / row_* / wave_* / row_bcast),
ds_swizzle_b32, ds_bpermute_b32, v_readlane_b32, v_permlane*_swap -- takes
values from OTHER lanes, so a source VGPR that some lanes never wrote (they
were masked off at every write) would hand those lanes' stale contents, left
by an earlier wave in the same registers, to their neighbours.  Per kernel,
the audit tracks the exec-mask depth through the linear code (s_and_saveexec /
s_andn2_saveexec / s_and_b64 exec / s_andn2_b64 exec narrow it, s_or_b64 exec /
s_mov_b64 exec restore it; the body of a loop whose latch retires lanes counts
as narrowed) and flags a cross-lane read whose source has no write, anywhere
before it in the kernel, at an exec depth no narrower than the read's own.

Third check (round 4, --masked, report only): a cross-lane read issued while
exec is narrowed (`masked_cross_lane_reads`): its reads of inactive lanes
return 0.  The stage kernel's first carry read lane 0 from under
`lane == 0 || bpermute(...)`, which hipcc compiles with lane 0 masked off.
The linear depth scan cannot follow every if / else join, so this list has
false positives and does not set the exit status.

usage: audit_loops.py file.s [symbol-regex] [--masked]   (exit 1 if any loop or stale read is flagged)
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
            j = next((k for k in range(i, len(lines)) if lines[k].strip().startswith("s_endpgm")), None)
            if j is not None:  # (a data symbol, e.g. a __device__ variable, has no code)
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


NARROW = re.compile(r"^(s_and_saveexec_b64|s_andn2_saveexec_b64|s_and_b64 exec,|s_andn2_b64 exec,)")
RESTORE = re.compile(r"^(s_or_b64 exec, exec,|s_mov_b64 exec, s|s_or_saveexec_b64)")
CROSS = re.compile(r"(quad_perm:|row_shl:|row_shr:|row_ror:|row_mirror|row_half_mirror|row_bcast|wave_shl|wave_rol|"
                   r"wave_shr|wave_ror|row_newbcast|row_share|row_xmask)|^(ds_swizzle_b32|ds_bpermute_b32|v_readlane_b32|"
                   r"v_permlane16_swap|v_permlane32_swap)")
VREG = re.compile(r"\bv(\d+)\b|\bv\[(\d+):(\d+)\]")


def regs_of(operand: str):
    out = set()
    for m in VREG.finditer(operand):
        if m.group(1) is not None:
            out.add(int(m.group(1)))
        else:
            out.update(range(int(m.group(2)), int(m.group(3)) + 1))
    return out


def operands(line: str):
    """(mnemonic, [operand strings]) of an instruction line."""
    parts = line.split(None, 1)
    if len(parts) < 2:
        return parts[0] if parts else "", []
    ops = [o.strip() for o in re.split(r",(?![^\[]*\])", parts[1])]
    return parts[0], ops


def exec_depths(body):
    """Exec-narrowing depth of every line (see the module docstring).  An if
    region opens with s_and_saveexec_b64 sX (or s_and_b64 / s_andn2_b64 exec
    outside a loop latch) and closes with s_or_b64 exec, exec, sX / s_mov_b64
    exec, sX: the depth is the count of open regions (a stack of the saved
    masks; a restore of a mask that is not on it, e.g. the exit of a loop whose
    latch retired lanes, closes nothing)."""
    stack, out = [], []
    for l in body:
        m = re.match(r"^(s_and_saveexec_b64|s_andn2_saveexec_b64|s_or_saveexec_b64)\s+(s\[\d+:\d+\])", l)
        r = re.match(r"^(s_or_b64 exec, exec,|s_mov_b64 exec,)\s*(s\[\d+:\d+\])", l)
        e = re.match(r"^s_or_saveexec_b64\s+(s\[\d+:\d+\]),\s*(s\[\d+:\d+\])", l)
        if e:
            # the else arm of an if / else: the then-arm's saved mask becomes
            # the else-arm's, closed later by s_or_b64 exec, exec, <new>
            if e.group(2) in stack:
                stack[stack.index(e.group(2))] = e.group(1)
        elif m and m.group(1) != "s_or_saveexec_b64":
            stack.append(m.group(2))
        elif r and r.group(2) in stack:
            while stack and stack.pop() != r.group(2):
                pass
        out.append(len(stack))
    # the body of an innermost loop that retires lanes at its latch runs narrowed after its first trip
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    for i, l in enumerate(body):
        m = re.match(r"^s_c?branch\w*\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] <= i:
            start = labels[m.group(1)]
            # the latch block (from the last label before the backward branch)
            # retires lanes: its own s_andn2_b64 exec, not a nested loop's
            k0 = next(k for k in range(i, start - 1, -1) if re.match(r"^\.LBB\w+:", body[k]))
            if any(re.match(r"^s_andn2_b64 exec, exec,", t) for t in body[k0:i + 1]):
                for k in range(start, i + 1):
                    out[k] += 1
    return out


def loop_regions(body):
    """(first, last) line of every loop (a backward branch and its target label)."""
    labels = {}
    for i, l in enumerate(body):
        m = re.match(r"^(\.LBB\w+):", l)
        if m:
            labels[m.group(1)] = i
    out = []
    for i, l in enumerate(body):
        m = re.match(r"^s_c?branch\w*\s+(\.LBB\w+)", l)
        if m and m.group(1) in labels and labels[m.group(1)] <= i:
            out.append((labels[m.group(1)], i))
    return out


def vgpr_writes(body, dep):
    """[(line, reg, exec depth)] of every instruction that writes a VGPR."""
    out = []
    for i, l in enumerate(body):
        if not l or l.startswith(".") or l.endswith(":"):
            continue
        mn, ops = operands(l)
        if not ops:
            continue
        if mn == "v_writelane_b32":
            # writes its one lane whatever exec is (hipcc's SGPR spill slots:
            # v_writelane under a narrowed exec, v_readlane later): depth 0
            for r in regs_of(ops[0]):
                out.append((i, r, 0))
            continue
        if (re.match(r"^(v_|ds_read|ds_bpermute|ds_swizzle|global_load|buffer_load|flat_load|scratch_load)", mn)
                or re.match(r"^(global_atomic|buffer_atomic|ds_)\w*_rtn", mn)) and not mn.startswith(
                    ("v_cmp", "v_readfirstlane", "v_readlane")):
            for r in regs_of(ops[0]):
                out.append((i, r, dep[i]))
        elif mn.startswith("v_cmp") and not ops[0].startswith(("s", "vcc")):
            for r in regs_of(ops[0]):
                out.append((i, r, dep[i]))
    return out


def stale_cross_lane_reads(body):
    """[(line, instruction, reg)] of cross-lane reads whose source VGPR has no
    write at an exec depth <= the read's, before it in the code or anywhere in
    a loop around it (a loop body laid out after its latch block)."""
    dep = exec_depths(body)
    loops = loop_regions(body)
    writes = {}
    for i, r, d in vgpr_writes(body, dep):
        writes.setdefault(r, []).append((i, d))
    found = []
    for i, l in enumerate(body):
        if not CROSS.search(l):
            continue
        mn, ops = operands(l)
        if not ops:
            continue
        if mn.startswith("ds_bpermute"):
            srcs = regs_of(ops[2]) if len(ops) > 2 else set()   # data operand (the address is this lane's)
        elif mn.startswith("ds_swizzle") or mn.startswith("v_readlane"):
            srcs = regs_of(ops[1]) if len(ops) > 1 else set()
        elif mn.startswith("v_permlane"):
            srcs = regs_of(ops[0]) | regs_of(ops[1])
        else:  # DPP: the first source operand is the one read from another lane
            srcs = regs_of(ops[1]) if len(ops) > 1 else set()
        around = [(a, b) for a, b in loops if a <= i <= b]
        for r in sorted(srcs):
            ok = any(d <= dep[i] and (j < i or any(a <= j <= b for a, b in around)) for j, d in writes.get(r, []))
            if not ok:
                found.append((i, l, r))
    return found


MASKED = re.compile(r"(quad_perm:|row_shl:|row_shr:|row_ror:|row_mirror|row_half_mirror|row_bcast|wave_shl|wave_rol|"
                    r"wave_shr|wave_ror|row_newbcast|row_share|row_xmask)|^(ds_swizzle_b32|ds_bpermute_b32|"
                    r"v_permlane16_swap|v_permlane32_swap)")


def masked_cross_lane_reads(body):
    """[(line, instruction)] of cross-lane reads issued under a narrowed exec
    (round 4, the stage kernel's first carry): a lane that reads an INACTIVE
    lane through ds_bpermute / ds_swizzle gets 0, through DPP 0 or its own old
    value, not the source lane's register.  hipcc narrows exec around a
    cross-lane builtin that sits in the right operand of `||` / `&&` or in a
    divergent branch; such a read is correct only if no active lane reads an
    inactive one, which the ISA alone cannot show, so every one is listed."""
    dep = exec_depths(body)
    return [(i, l) for i, l in enumerate(body) if dep[i] > 0 and MASKED.search(l)]


def main():
    masked = "--masked" in sys.argv
    args = [a for a in sys.argv[1:] if a != "--masked"]
    path = args[0]
    pat = re.compile(args[1]) if len(args) > 1 else None
    lines = [l.split(";")[0].strip() for l in open(path).read().split("\n")]
    bad = nread = 0
    for sym, a, b in kernels(lines):
        if pat and not pat.search(sym):
            continue
        body = lines[a:b + 1]
        for lab, nl, latch in divergent_load_loops(body):
            print(f"{sym}: loop at {lab} narrows exec and issues {nl} VMEM loads (latch: {latch})")
            bad += 1
        nread += sum(1 for l in body if CROSS.search(l))
        for i, l, r in stale_cross_lane_reads(body):
            print(f"{sym}: cross-lane read of v{r} with no earlier write at its exec depth: {l}")
            bad += 1
        if masked:  # report only: the linear exec-depth scan over-counts across if / else joins
            for i, l in masked_cross_lane_reads(body):
                print(f"{sym}: cross-lane read under a narrowed exec (inactive source lanes read as 0): {l}")
    print(f"audit: {nread} cross-lane reads checked, {bad} findings", file=sys.stderr)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
