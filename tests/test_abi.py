"""The C-ABI library loads, exports every symbol include/lneto_amd.h declares,
and rejects bad arguments without touching a GPU (CPU-only checks)."""
import ctypes
import os
import re
import subprocess

import pytest

import lneto_amd as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "lneto_amd.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(lnx_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    for s in ["lnx_crc32", "lnx_crc32_update", "lnx_crc32_search", "lnx_sum16_payload",
              "lnx_crc32_batch", "lnx_fcs_verify_batch", "lnx_sum16_batch", "lnx_crc32_batch_multi"]:
        assert s in syms


def test_library_exports_every_declared_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\sT\s+(lnx_\w+)", out))
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    for s in declared_symbols():
        assert getattr(L.lib, s) is not None


def test_library_contains_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-readelf", "-S", L.LIB_PATH], capture_output=True, text=True)
    assert ".hip_fatbin" in out.stdout
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_batch_entry_points_validate_without_gpu():
    # n == 0 is a no-op; NULL buffers with n > 0 are EINVAL (checked before any HIP call)
    assert L.lib.lnx_crc32_batch(None, None, 0, None, None) == 0
    assert L.lib.lnx_crc32_batch(None, None, 5, None, None) == L.LNX_EINVAL
    assert L.lib.lnx_fcs_verify_batch(None, None, 5, None, None) == L.LNX_EINVAL
    assert L.lib.lnx_sum16_batch(None, None, None, None, 5, None, None) == L.LNX_EINVAL
    assert L.lib.lnx_crc32_batch_multi(0, None, None, None, None, None) == L.LNX_EINVAL
    assert L.lib.lnx_crc32_batch_ex(None, None, 5, None, L.BATCH_SHORT_FRAMES, None) == L.LNX_EINVAL
    assert L.lib.lnx_crc32_batch_ex(None, None, 0, None, 2, None) == L.LNX_EINVAL  # unknown flag bit
    assert L.lib.lnx_fcs_verify_batch_ex(None, None, 0, None, L.BATCH_SHORT_FRAMES, None) == 0
    # the transmit tail in one read: NULL buffers, unknown flag bits
    assert L.lib.lnx_tx_finish_batch(None, None, None, 0, 1536, 3, None, None) == 0
    assert L.lib.lnx_tx_finish_batch(None, None, None, 5, 1536, 3, None, None) == L.LNX_EINVAL
    b1 = (ctypes.c_uint8 * 64)()
    s1 = (ctypes.c_uint64 * 1)(0)
    l1 = (ctypes.c_uint32 * 1)(60)
    st1 = (ctypes.c_uint8 * 1)()
    assert L.lib.lnx_tx_finish_batch(ctypes.addressof(b1), ctypes.addressof(s1), ctypes.addressof(l1), 1, 64, 4,
                                     ctypes.addressof(st1), None) == L.LNX_EINVAL
    buf = (ctypes.c_uint8 * 8)()
    off = (ctypes.c_uint64 * 2)(0, 100)  # offset beyond nbytes
    out = (ctypes.c_uint32 * 1)()
    assert L.lib.lnx_crc32_batch_host(ctypes.addressof(buf), 8, ctypes.addressof(off), 1,
                                      ctypes.addressof(out), 0) == L.LNX_EINVAL


def test_version_string():
    assert "gfx950" in L.version()


def test_cpp_host_api_compiles_and_runs(tmp_path):
    """include/lneto_amd.hpp (C++ mirror of the Go API) against the built library."""
    src = os.path.join(ROOT, "tests", "cpp", "test_host_api.cpp")
    exe = tmp_path / "test_host_api"
    subprocess.run(["g++", "-std=c++17", "-O1", "-Wall", "-I", os.path.join(ROOT, "include"), src,
                    "-o", str(exe), "-L", os.path.dirname(L.LIB_PATH), "-llneto_amd",
                    f"-Wl,-rpath,{os.path.dirname(L.LIB_PATH)}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ok" in r.stdout


def test_rows_kernel_algebra_emulated_on_cpu(tmp_path):
    """tests/cpp/rows_emulator.cpp: the CRC kernel's per-row algebra (window
    geometry, masks, junk removal, F, row XOR, Z_{-t}) replayed lane by lane on
    the CPU from the library's real LDS images, for every row layout including
    the lean line rows."""
    src = os.path.join(ROOT, "tests", "cpp", "rows_emulator.cpp")
    exe = tmp_path / "rows_emulator"
    subprocess.run(["g++", "-std=c++17", "-O2", "-Wall", src, "-o", str(exe), "-L", os.path.dirname(L.LIB_PATH),
                    "-llneto_amd", f"-Wl,-rpath,{os.path.dirname(L.LIB_PATH)}"], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout + r.stderr


@pytest.mark.gpu
def test_cpp_host_api_on_gpu(cuda, tmp_path):
    """The same C++ program on the MI355X: the ring opens and verifies FCS."""
    test_cpp_host_api_compiles_and_runs(tmp_path)


def _kernels(path):
    """Kernel symbols (mangled) in the .so's gfx950 code objects."""
    out = subprocess.run(["objcopy", "-O", "binary", "--only-section=.hip_fatbin", path, "/dev/stdout"],
                         capture_output=True, check=True).stdout
    return sorted(set(m.decode() for m in re.findall(rb"(_ZN3lnx\w+)\.kd", out)))


def test_product_library_holds_only_product_kernels():
    """The product .so carries exactly the shipped kernel instances: every
    crc32_rows_kernel with VAR = 0 and no streaming form (STR = 0), one instance
    each of sum16 / search / ring, ingress verify + TX generate; the research
    variants live in liblneto_amd_research.so only."""
    ks = _kernels(L.LIB_PATH)
    rows = [k for k in ks if "crc32_rows_kernel" in k]
    assert len(rows) == 5, rows  # offsets crc / verify, segments crc / verify / append
    for k in rows:
        assert re.search(r"CrcModeE\dELi0E", k), k          # VAR = 0
        assert re.search(r"ELi0EEEvPKh", k), k              # STR = 0
    others = sorted(re.sub(r"^_ZN3lnx\d+(\w+?kernel).*$", r"\1", k) for k in ks if k not in rows)
    # ingress: filtered / unfiltered verdicts, TX generate; rx_verify: (FCS / none) x (filter / none) x
    # (HBM / host memory); tx_finish: (FCS / none) x (checksum / none) x (HBM / host memory)
    assert others == (["crc32_search_o_kernel"] + ["crc32_stage_kernel"] * 2 + ["ingress_verify_kernel"] * 3 + ["pcap_rows_kernel"] +
                      ["ring_segments_kernel"] + ["rx_verify_kernel"] * 8 + ["sum16_lines_kernel"] + ["tx_finish_kernel"] * 8 +
                      ["tx_gate_probe_kernel"]), others
    stage = [k for k in ks if "crc32_stage_kernel" in k]
    assert all(re.search(r"crc32_stage_kernelILNS_9StageModeE\dEEEv", k) for k in stage), stage  # CRC / verify only
    research = os.path.join(os.path.dirname(L.LIB_PATH), "liblneto_amd_research.so")
    if os.path.exists(research):
        rk = _kernels(research)
        assert set(ks) <= set(rk) and len(rk) > len(ks) + 40
        # the round-4 staged variants live in stage_research.hip's namespace lnx::rs only
        assert any("2rs21crc32_stage_rs_kernel" in k for k in rk)
        assert not any("crc32_stage_rs_kernel" in k for k in ks)


def test_product_library_reads_no_environment():
    """No getenv in the product library's code (the LNX_PROF_* knobs are research-only)."""
    out = subprocess.run(["nm", "-D", "--undefined-only", L.LIB_PATH], capture_output=True, text=True,
                         check=True).stdout
    assert not re.search(r"\bgetenv\b", out), "product library imports getenv"
    assert not hasattr_sym(L.lib, "lnx__crc32_variant")


def hasattr_sym(lib, name):
    try:
        getattr(lib, name)
        return True
    except AttributeError:
        return False
