"""Static audit of the compiled CRC kernels (CPU only; needs hipcc, no GPU).

The streaming loads are inline asm that hipcc neither counts for vmcnt nor pads
for hazards, so two classes of bug compile silently and surface only as wrong
CRCs or GPU memory faults on the box.  tools/prof/audit_ring.py checks every
instantiation's .s for (1) a compiler instruction touching a ring register
while its load is outstanding and (2) a VALU write of a buffer-descriptor SGPR
fewer than 5 wait states before an asm buffer load that reads it.
"""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "lneto_amd", "csrc", "crc32_kernel.hip")
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("build", ["product", "research"])
def test_every_kernel_instantiation_passes_the_ring_audit(tmp_path, build):
    """Both libraries: the product's instances and the research variants the GPU tests still run."""
    flags = ["-DLNX_RESEARCH"] if build == "research" else []
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++20", "-mllvm", "-amdgpu-atomic-optimizer-strategy=None",
                    "-c", "--save-temps", *flags,
                    "-o", str(tmp_path / "k.o"), SRC], cwd=tmp_path, check=True, capture_output=True)
    asm = next(p for p in os.listdir(tmp_path) if p.endswith("gfx950.s"))
    text = open(tmp_path / asm).read()
    syms = re.findall(r"^(_ZN3lnx17crc32_rows_kernel\w+):", text, flags=re.M)
    assert len(syms) >= 3
    for sym in syms:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "audit_ring.py"),
                            str(tmp_path / asm), sym], capture_output=True, text=True)
        assert r.returncode == 0, f"{sym}:\n{r.stdout}"


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src", ["crc32_kernel", "stage_kernel", "stage_research", "sum16_kernel", "ingress_kernel", "rx_verify_kernel",
                                 "search_kernel", "rx_ring"])
@pytest.mark.parametrize("build", ["product", "research"])
def test_no_divergent_exit_loop_around_wide_loads(tmp_path, src, build):
    """tools/prof/audit_loops.py over every product kernel: no innermost loop
    that retires lanes with s_andn2_b64 exec and issues multi-dword loads (the
    shape of round 1's wrong-sum sum16 form)."""
    path = os.path.join(ROOT, "lneto_amd", "csrc", ("research/" if src == "stage_research" else "") + src + ".hip")
    flags = ["-DLNX_RESEARCH"] if build == "research" else []
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++20", "-mllvm",
                    "-amdgpu-atomic-optimizer-strategy=None", "-c", "--save-temps", *flags, "-o", str(tmp_path / "k.o"),
                    path],
                   cwd=tmp_path, check=True, capture_output=True)
    asm = next(p for p in os.listdir(tmp_path) if p.endswith("gfx950.s"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "audit_loops.py"), str(tmp_path / asm)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stdout
    if build == "product":
        # no product kernel spills to scratch: round 5's rx_verify / tx_finish
        # spills (120-170 bytes per lane, reloaded in the row passes) doubled
        # their memory traffic and time
        meta = open(tmp_path / asm).read()
        spills = re.findall(r"\.name:\s+(\S+)\s*\n(?:.*\n)*?\s+\.private_segment_fixed_size:\s+(\d+)", meta)
        assert spills or src == "stage_research", "no kernel metadata found"  # (research-only source: empty product)
        assert all(int(b) == 0 for _, b in spills), [(k, b) for k, b in spills if int(b)]


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
@pytest.mark.parametrize("src,nsyms", [("stage_kernel", 2), ("stage_research", 30)])
def test_stage_kernel_passes_the_ring_audit(tmp_path, src, nsyms):
    """The staged lane streams (stage_kernel.hip: the product CRC / verify
    pair; stage_research.hip: the round-4 variants): each round's hand-placed
    vmcnt(10) must cover the 8 loads of the slot it drains, with the
    held-result stores (2 per round, in asm so hipcc cannot drop or move them)
    and the next slot's 8 loads younger than it."""
    path = os.path.join(ROOT, "lneto_amd", "csrc", ("research/" if src == "stage_research" else "") + src + ".hip")
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++20", "-c", "--save-temps", "-DLNX_RESEARCH",
                    "-o", str(tmp_path / "k.o"), path], cwd=tmp_path, check=True, capture_output=True)
    asm = next(p for p in os.listdir(tmp_path) if p.endswith("gfx950.s"))
    syms = re.findall(r"^(_ZN3lnx\w*crc32_stage_(?:rs_)?kernel\w+):", open(tmp_path / asm).read(), flags=re.M)
    # research: CRC / verify x (the three folds, + 766-frame blocks, + the deferred correction, + the patched
    # boundary word, + two chains per half, + 190- / 254-frame blocks, + offsets loaded a block ahead, + 510-frame
    # blocks, + 6 waves, + 6 timing-only diagnostics)
    assert len(syms) == nsyms, syms
    for sym in syms:
        r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "audit_ring.py"),
                            str(tmp_path / asm), sym], capture_output=True, text=True)
        assert r.returncode == 0, f"{sym}:\n{r.stdout}"


def _audit_fixture(tmp_path, name):
    path = os.path.join(ROOT, "tests", "audit_fixtures", name)
    subprocess.run([HIPCC, "--offload-arch=gfx950", "-O3", "-std=c++20", "-c", "--save-temps", "-o",
                    str(tmp_path / "k.o"), path], cwd=tmp_path, check=True, capture_output=True)
    asm = next(p for p in os.listdir(tmp_path) if p.endswith("gfx950.s"))
    return subprocess.run([sys.executable, os.path.join(ROOT, "tools", "prof", "audit_loops.py"), str(tmp_path / asm)],
                          capture_output=True, text=True)


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_cross_lane_audit_catches_a_stale_source(tmp_path):
    """The cross-lane check (a DPP / bpermute / readlane source that some lanes
    never wrote) flags a register written only under a narrowed exec and
    passes the same kernel with the register zeroed first."""
    r = _audit_fixture(tmp_path, "stale_dpp.hip")
    found = [l for l in r.stdout.splitlines() if "cross-lane" in l]
    assert len(found) == 1 and found[0].startswith("_Z5stale"), r.stdout


@pytest.mark.skipif(not os.path.exists(HIPCC), reason="hipcc not installed")
def test_r1g_failing_form_has_no_stale_cross_lane_source(tmp_path):
    """the round-1 sum16 form that returned wrong sums is
    caught by the loop-shape check, but none of its cross-lane reads (the
    row_add16 DPP chain) takes a register some lanes never wrote: the
    stale-register hypothesis does not explain it."""
    r = _audit_fixture(tmp_path, "sum16_r1g_divergent.hip")
    assert any("narrows exec" in l for l in r.stdout.splitlines()), r.stdout
    assert not any("cross-lane" in l for l in r.stdout.splitlines()), r.stdout
    assert "8 cross-lane reads checked" in r.stderr
