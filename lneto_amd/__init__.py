"""lneto_amd — MI355X-native batched checksum path of lneto.

Python binding (ctypes) of the C-ABI in include/lneto_amd.h, implemented by
lneto_amd/liblneto_amd.so (hand-written HIP kernels for gfx950 + host C++).
PyTorch is used only as device-memory / stream plumbing for the batch calls.

Mirrors the reference's API for this path:
    ethernet.CRC32 / CRC32Search / crc32.Update   -> crc32, crc32_search, crc32_update
    lneto.CRC791 / NeverZeroSum                   -> CRC791, never_zero_sum
    batch (device-resident) extensions            -> crc32_batch, fcs_verify_batch, sum16_batch

There is no CPU fallback for the batch calls: if the library is missing this
module raises at import; if no HIP device is usable the batch calls raise
LnetoError.
"""
from __future__ import annotations

import ctypes
import os

__all__ = [
    "LnetoError", "lib", "crc32", "crc32_update", "crc32_search", "sum_write_even", "sum16",
    "payload_sum16", "never_zero_sum", "CRC791", "crc32_batch", "fcs_verify_batch", "sum16_batch",
    "crc32_batch_host", "crc32_batch_multi", "tx_checksum_batch", "rx_verify_batch", "device_count", "version", "build_id", "LIB_PATH",
    "CRC32_RESIDUE", "RxRing", "RxFilter", "RX_NO_FCS", "research_lib",
]

HERE = os.path.dirname(os.path.abspath(__file__))
# LNETO_AMD_LIB selects an alternative in-tree build (profiling experiments only).
LIB_PATH = os.environ.get("LNETO_AMD_LIB") or os.path.join(HERE, "liblneto_amd.so")
CRC32_RESIDUE = 0x2144DF1C

LNX_OK, LNX_EINVAL, LNX_ENODEV, LNX_EHIP, LNX_ENOMEM = 0, -1, -2, -3, -5
_ERRNAMES = {LNX_EINVAL: "EINVAL", LNX_ENODEV: "ENODEV", LNX_EHIP: "EHIP", LNX_ENOMEM: "ENOMEM"}


class LnetoError(RuntimeError):
    pass


if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} is not built; run `python -c 'import __graft_entry__ as g; g.build()'` "
                      "or `make -C lneto_amd/csrc`")

# PyTorch-ROCm bundles its own libamdhip64.so.7 / libhsa-runtime64.so.1.  If this
# library were loaded first it would pull /opt/rocm's copies in, and torch would
# then load its bundled ones as well: two HSA runtimes in one process, and HIP
# calls from one of them see no device.  Importing torch first makes the dynamic
# linker resolve our libamdhip64.so.7 dependency to torch's already-loaded one,
# so the process has exactly one HIP runtime.  (C / C++ / cgo users get /opt/rocm's.)
try:
    import torch as _torch  # noqa: F401
except ImportError:  # pragma: no cover - torch is plumbing, not a dependency of the C-ABI
    _torch = None

lib = ctypes.CDLL(LIB_PATH)

_u8p = ctypes.POINTER(ctypes.c_uint8)
_vp = ctypes.c_void_p


class RxFilter(ctypes.Structure):
    """lnx_rx_filter (include/lneto_amd.h): the stack configuration behind the
    receive verdicts' ErrPacketDrop checks (internet/stack-ethernet.go:146-161,
    internet/stack-ip4.go:108-141, internet/stack-ip6.go:93-111).  Build it with
    RxFilter.make(mac=..., ip4=..., ...)."""
    _fields_ = [
        ("mac", ctypes.c_uint8 * 6), ("eth_accept_multicast", ctypes.c_uint8),
        ("ip4_accept_multicast", ctypes.c_uint8), ("ip4_accept_broadcast", ctypes.c_uint8),
        ("ip6_accept_multicast", ctypes.c_uint8), ("ip4", ctypes.c_uint8 * 4), ("ip6", ctypes.c_uint8 * 16),
        ("ethertypes", ctypes.c_uint16 * 8), ("n_ethertypes", ctypes.c_uint32),
        ("ip4_protocols", ctypes.c_uint8 * 32), ("ip6_protocols", ctypes.c_uint8 * 32),
    ]

    @classmethod
    def make(cls, mac: bytes, ethertypes=(0x0800, 0x86DD, 0x0806), ip4: bytes = bytes(4), ip6: bytes = bytes(16),
             ip4_protocols=(1, 6, 17), ip6_protocols=(6, 17, 58), eth_accept_multicast: bool = False,
             ip4_accept_multicast: bool = False, ip4_accept_broadcast: bool = False,
             ip6_accept_multicast: bool = False) -> "RxFilter":
        if len(mac) != 6 or len(ip4) != 4 or len(ip6) != 16 or len(ethertypes) > 8:
            raise LnetoError("RxFilter: mac 6 bytes, ip4 4, ip6 16, at most 8 EtherTypes")
        if any(et <= 1500 or et > 0xFFFF for et in ethertypes):
            # RegisterEthernet: proto > MaxUint16 || proto <= 1500 -> ErrInvalidConfig (internet/stack-ethernet.go:131-135)
            raise LnetoError("RxFilter: EtherTypes must be in (1500, 0xFFFF] (RegisterEthernet)")
        f = cls()
        f.mac[:] = list(mac)
        f.ip4[:] = list(ip4)
        f.ip6[:] = list(ip6)
        f.eth_accept_multicast, f.ip4_accept_multicast = int(eth_accept_multicast), int(ip4_accept_multicast)
        f.ip4_accept_broadcast, f.ip6_accept_multicast = int(ip4_accept_broadcast), int(ip6_accept_multicast)
        f.n_ethertypes = len(ethertypes)
        for i, et in enumerate(ethertypes):
            f.ethertypes[i] = et
        for arr, protos in ((f.ip4_protocols, ip4_protocols), (f.ip6_protocols, ip6_protocols)):
            for p in protos:
                arr[p >> 3] |= 1 << (p & 7)
        return f
_sig = {
    "lnx_crc32_update": (ctypes.c_uint32, [ctypes.c_uint32, _u8p, ctypes.c_size_t]),
    "lnx_crc32": (ctypes.c_uint32, [_u8p, ctypes.c_size_t]),
    "lnx_crc32_search": (ctypes.c_int64, [_u8p, ctypes.c_size_t, ctypes.c_int64]),
    "lnx_sum_write_even": (ctypes.c_uint32, [ctypes.c_uint32, _u8p, ctypes.c_size_t]),
    "lnx_sum16": (ctypes.c_uint16, [ctypes.c_uint32]),
    "lnx_sum16_payload": (ctypes.c_uint16, [ctypes.c_uint32, _u8p, ctypes.c_size_t]),
    "lnx_never_zero_sum": (ctypes.c_uint16, [ctypes.c_uint16]),
    "lnx_crc32_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "lnx_fcs_verify_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "lnx_sum16_batch": (ctypes.c_int, [_vp, _vp, _vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "lnx_ingress_verify_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp, _vp]),
    "lnx_ingress_verify_batch_filtered": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32,
                                                         ctypes.POINTER(RxFilter), _vp, _vp]),
    "lnx_rx_ring_set_filter": (ctypes.c_int, [_vp, ctypes.POINTER(RxFilter)]),
    "lnx_crc32_search_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "lnx_crc32_segments": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "lnx_fcs_append_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, _vp, _vp]),
    "lnx_tx_checksum_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "lnx_crc32_batch_host": (ctypes.c_int, [_vp, ctypes.c_uint64, _vp, ctypes.c_uint64, _vp, ctypes.c_int]),
    "lnx_crc32_batch_multi": (ctypes.c_int, [ctypes.c_int, _vp, _vp, _vp, _vp, _vp]),
    "lnx_rx_ring_create": (ctypes.c_int, [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.POINTER(_vp)]),
    "lnx_rx_ring_destroy": (None, [_vp]),
    "lnx_rx_ring_slots": (_vp, [_vp]),
    "lnx_rx_ring_lengths": (_vp, [_vp]),
    "lnx_rx_ring_ingress": (ctypes.c_int, [_vp, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           _vp, _vp]),
    "lnx_ingress_packets": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                           _vp, _vp]),
    "lnx_crc32_batch_ex": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp]),
    "lnx_fcs_verify_batch_ex": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, ctypes.c_uint32, _vp]),
    "lnx_egress_packets": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, _vp]),
    "lnx_rx_verify_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.POINTER(RxFilter),
                                            _vp, _vp, _vp]),
    "lnx_ingress_verdict": (ctypes.c_int, [_vp, ctypes.c_size_t, ctypes.c_uint32, ctypes.POINTER(RxFilter)]),
    "lnx_pcap_checksums": (ctypes.c_int, [_vp, ctypes.c_size_t]),
    "lnx_pcap_verify_batch": (ctypes.c_int, [_vp, _vp, ctypes.c_uint64, _vp, _vp]),
    "lnx_tx_checksum": (ctypes.c_int, [_vp, ctypes.c_size_t]),
    "lnx_fcs_append": (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_uint32), ctypes.c_uint32]),
    "lnx_rx_ring_set_host_threshold": (ctypes.c_int, [_vp, ctypes.c_uint32]),
    "lnx_rx_ring_stats": (ctypes.c_int, [_vp, _vp]),
    "lnx_rx_ring_set_zero_copy": (ctypes.c_int, [_vp, ctypes.c_int]),
    "lnx_tx_finish_batch": (ctypes.c_int, [_vp, _vp, _vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, _vp, _vp]),
    "lnx_device_count": (ctypes.c_int, []),
    "lnx_last_error": (ctypes.c_char_p, []),
    "lnx_version": (ctypes.c_char_p, []),
}
for _name, (_res, _args) in _sig.items():
    _f = getattr(lib, _name)
    _f.restype = _res
    _f.argtypes = _args


def _check(rc: int, what: str) -> None:
    if rc != LNX_OK:
        detail = lib.lnx_last_error().decode() if rc == LNX_EHIP else ""
        raise LnetoError(f"{what} failed: {_ERRNAMES.get(rc, rc)} {detail}".strip())


def _buf(data: bytes):
    data = bytes(data)
    return (ctypes.c_uint8 * max(len(data), 1)).from_buffer_copy(data or b"\0"), len(data)


# ----------------------------------------------------------- per-frame (host)
def crc32_update(crc: int, p: bytes) -> int:
    """Go crc32.Update(crc, IEEETable, p) — the CRC32Update hook (internet/stack-ethernet.go:31-32)."""
    b, n = _buf(p)
    return lib.lnx_crc32_update(crc & 0xFFFFFFFF, b, n)


def crc32(p: bytes) -> int:
    """ethernet.CRC32 (ethernet/crc.go:19-21)."""
    b, n = _buf(p)
    return lib.lnx_crc32(b, n)


def crc32_search(p: bytes, min_off: int) -> int:
    """ethernet.CRC32Search (ethernet/crc.go:28-47)."""
    b, n = _buf(p)
    return lib.lnx_crc32_search(b, n, min_off)


def sum_write_even(s: int, p: bytes) -> int:
    if len(p) & 1:
        raise IndexError("WriteEven requires an even-length buffer (crc.go:30)")
    b, n = _buf(p)
    return lib.lnx_sum_write_even(s & 0xFFFFFFFF, b, n)


def sum16(s: int) -> int:
    return lib.lnx_sum16(s & 0xFFFFFFFF)


def payload_sum16(s: int, p: bytes) -> int:
    b, n = _buf(p)
    return lib.lnx_sum16_payload(s & 0xFFFFFFFF, b, n)


def never_zero_sum(x: int) -> int:
    return lib.lnx_never_zero_sum(x & 0xFFFF)


class CRC791:
    """lneto.CRC791 (crc.go:13-62): running RFC 791 one's-complement sum."""

    __slots__ = ("sum",)

    def __init__(self) -> None:
        self.sum = 0

    def WriteEven(self, buff: bytes) -> None:
        self.sum = sum_write_even(self.sum, buff)

    def AddUint16(self, v: int) -> None:
        self.sum = (self.sum + (v & 0xFFFF)) & 0xFFFFFFFF

    def AddUint32(self, v: int) -> None:
        self.AddUint16((v >> 16) & 0xFFFF)
        self.AddUint16(v & 0xFFFF)

    def Sum16(self) -> int:
        return sum16(self.sum)

    def PayloadSum16(self, buff: bytes) -> int:
        return payload_sum16(self.sum, buff)

    def Reset(self) -> None:
        self.sum = 0


# ------------------------------------------------------- batched (device)
def _dtypes(*names):
    import torch
    table = {
        "u8": (torch.uint8, torch.int8),
        "i16": (torch.int16, getattr(torch, "uint16", torch.int16)),
        "i32": (torch.int32, getattr(torch, "uint32", torch.int32)),
        "i64": (torch.int64, getattr(torch, "uint64", torch.int64)),
    }
    return [table[n] for n in names]


class _Batch:
    """Argument check and device scope of one batch call.

    Every tensor must be a contiguous device tensor of the 8-, 16-, 32- or 64-bit
    width the C-ABI reads through it (signedness is free: the kernels see the
    bits), and all of them must live on ONE device.  The call then runs with that
    device current and on its stream (the caller's ``stream`` must be on the same
    device), so the library's per-device context and the kernel's memory agree.
    """

    def __init__(self, what, args, stream):
        import torch
        self.what = what
        dev = None
        # a kind ending in "?" marks an optional argument (NULL in the C-ABI)
        for name, t, kind in args:
            if t is None and not kind.endswith("?"):
                raise LnetoError(f"{what}: {name} is required")
        for name, t, kind in args:
            kind = kind.rstrip("?")
            if t is None:
                continue
            if not isinstance(t, torch.Tensor) or not t.is_cuda or not t.is_contiguous():
                raise LnetoError(f"{what}: {name} must be a contiguous device tensor")
            if t.dtype not in _dtypes(kind)[0]:
                raise LnetoError(f"{what}: {name} must be {kind} (got {t.dtype})")
            if dev is None:
                dev = t.device
            elif t.device != dev:
                raise LnetoError(f"{what}: {name} is on {t.device}, other arguments on {dev}")
        self.device = dev
        if stream is not None and stream.device != dev:
            raise LnetoError(f"{what}: stream is on {stream.device}, tensors on {dev}")
        self._stream = stream
        self._ctx = torch.cuda.device(dev)

    def __enter__(self):
        import torch
        self._ctx.__enter__()
        s = self._stream if self._stream is not None else torch.cuda.current_stream(self.device)
        return s.cuda_stream

    def __exit__(self, *exc):
        return self._ctx.__exit__(*exc)


def _out(what, out, n, dtype, kind, device):
    """Caller-supplied output: checked like an input and at least n elements; else allocated."""
    import torch
    if out is None:
        return torch.empty(max(n, 0), dtype=dtype, device=device)
    if not isinstance(out, torch.Tensor) or not out.is_cuda or not out.is_contiguous():
        raise LnetoError(f"{what}: out must be a contiguous device tensor")
    if out.dtype not in _dtypes(kind)[0]:
        raise LnetoError(f"{what}: out must be {kind} (got {out.dtype})")
    if out.device != device:
        raise LnetoError(f"{what}: out is on {out.device}, inputs on {device}")
    if out.numel() < n:
        raise LnetoError(f"{what}: out holds {out.numel()} elements, {n} needed")
    return out


def _need_len(what, name, t, n):
    if t is not None and t.numel() < n:
        raise LnetoError(f"{what}: {name} holds {t.numel()} elements, {n} needed")


BATCH_SHORT_FRAMES = 1  # LNX_BATCH_SHORT_FRAMES


def crc32_batch(d_bytes, d_off, out=None, stream=None, short_frames=False):
    """CRC32 of every frame d_bytes[d_off[i]:d_off[i+1]] on the GPU.

    d_bytes: uint8 device tensor; d_off: int64 device tensor of N+1 offsets.
    Returns an int32 device tensor holding the uint32 CRCs bit-for-bit.
    short_frames=True (lnx_crc32_batch_ex with LNX_BATCH_SHORT_FRAMES): the
    staged lane-stream kernel reads every slice that is not giant, where the
    plain entry picks the kernel per slice on the device (same results).
    """
    import torch
    what = "lnx_crc32_batch_ex" if short_frames else "lnx_crc32_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_off", d_off, "i64")], stream)
    n = d_off.numel() - 1
    out = _out(what, out, n, torch.int32, "i32", b.device)
    if n > 0:
        with b as s:
            if short_frames:
                _check(lib.lnx_crc32_batch_ex(d_bytes.data_ptr(), d_off.data_ptr(), n, out.data_ptr(),
                                              BATCH_SHORT_FRAMES, s), what)
            else:
                _check(lib.lnx_crc32_batch(d_bytes.data_ptr(), d_off.data_ptr(), n, out.data_ptr(), s), what)
    return out


def fcs_verify_batch(d_bytes, d_off, out=None, stream=None, short_frames=False):
    """1 where frame i (payload + trailing LE FCS) passes the FCS check, else 0
    (short_frames as crc32_batch)."""
    import torch
    what = "lnx_fcs_verify_batch_ex" if short_frames else "lnx_fcs_verify_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_off", d_off, "i64")], stream)
    n = d_off.numel() - 1
    out = _out(what, out, n, torch.uint8, "u8", b.device)
    if n > 0:
        with b as s:
            if short_frames:
                _check(lib.lnx_fcs_verify_batch_ex(d_bytes.data_ptr(), d_off.data_ptr(), n, out.data_ptr(),
                                                   BATCH_SHORT_FRAMES, s), what)
            else:
                _check(lib.lnx_fcs_verify_batch(d_bytes.data_ptr(), d_off.data_ptr(), n, out.data_ptr(), s), what)
    return out


def crc32_segments(d_bytes, d_start, d_len, out=None, stream=None):
    """CRC32 of every frame d_bytes[d_start[i] : d_start[i] + d_len[i]] (lnx_crc32_segments);
    d_start int64, d_len int32; frames in address order, not overlapping."""
    import torch
    what = "lnx_crc32_segments"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_start", d_start, "i64"), ("d_len", d_len, "i32")], stream)
    n = d_start.numel()
    _need_len(what, "d_len", d_len, n)
    out = _out(what, out, n, torch.int32, "i32", b.device)
    if n > 0:
        with b as s:
            _check(lib.lnx_crc32_segments(d_bytes.data_ptr(), d_start.data_ptr(), d_len.data_ptr(), n,
                                          out.data_ptr(), s), what)
    return out


def fcs_append_batch(d_bytes, d_start, d_len, capacity: int, status=None, stream=None):
    """TX FCS append in place (lnx_fcs_append_batch): pad to 60, append LE FCS,
    d_len (int32, updated) += padding + 4.  Returns the uint8 status (0 or 6)."""
    import torch
    what = "lnx_fcs_append_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_start", d_start, "i64"), ("d_len", d_len, "i32")], stream)
    n = d_start.numel()
    _need_len(what, "d_len", d_len, n)
    status = _out(what, status, n, torch.uint8, "u8", b.device)
    if n > 0:
        with b as s:
            _check(lib.lnx_fcs_append_batch(d_bytes.data_ptr(), d_start.data_ptr(), d_len.data_ptr(), n, capacity,
                                            status.data_ptr(), s), what)
    return status


def tx_checksum_batch(d_bytes, d_start, d_len, status=None, stream=None):
    """Transmit checksum generate in place (lnx_tx_checksum_batch): IPv4 / IPv6
    length fields, IPv4 header CRC, TCP / UDP / ICMP CRCs of every frame
    d_bytes[d_start[i] : d_start[i] + d_len[i]] (int64 starts, int32 lengths).
    Returns the uint8 status (0, 18 ErrTruncatedFrame, 15 ErrInvalidLengthField)."""
    import torch
    what = "lnx_tx_checksum_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_start", d_start, "i64"), ("d_len", d_len, "i32")], stream)
    n = d_start.numel()
    _need_len(what, "d_len", d_len, n)
    status = _out(what, status, n, torch.uint8, "u8", b.device)
    if n > 0:
        with b as s:
            _check(lib.lnx_tx_checksum_batch(d_bytes.data_ptr(), d_start.data_ptr(), d_len.data_ptr(), n,
                                             status.data_ptr(), s), what)
    return status


def tx_finish_batch(d_bytes, d_start, d_len, capacity: int, flags: int = 3, status=None, stream=None):
    """The transmit tail in one read (lnx_tx_finish_batch): the checksum step
    (flags & TX_CHECKSUM) then padding + FCS (flags & TX_FCS) of every frame
    d_bytes[d_start[i] : d_start[i] + d_len[i]], in place; d_len (int32) is
    updated.  Returns the uint8 status (the checksum step's if non-zero, else
    the append's)."""
    import torch
    what = "lnx_tx_finish_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_start", d_start, "i64"), ("d_len", d_len, "i32")], stream)
    n = d_start.numel()
    _need_len(what, "d_len", d_len, n)
    status = _out(what, status, n, torch.uint8, "u8", b.device)
    if n > 0:
        with b as s:
            _check(lib.lnx_tx_finish_batch(d_bytes.data_ptr(), d_start.data_ptr(), d_len.data_ptr(), n, capacity,
                                           flags, status.data_ptr(), s), what)
    return status


def crc32_search_batch(d_bytes, d_off, d_min_off=None, out=None, stream=None):
    """ethernet.CRC32Search of every capture d_bytes[d_off[i]:d_off[i+1]] on the GPU
    (lnx_crc32_search_batch).  d_min_off: int64 (N) or None.  Returns int64 (N), -1 = none."""
    import torch
    what = "lnx_crc32_search_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_off", d_off, "i64"), ("d_min_off", d_min_off, "i64?")],
               stream)
    n = d_off.numel() - 1
    _need_len(what, "d_min_off", d_min_off, n)
    out = _out(what, out, n, torch.int64, "i64", b.device)
    if n > 0:
        with b as s:
            _check(lib.lnx_crc32_search_batch(d_bytes.data_ptr(), d_off.data_ptr(),
                                              d_min_off.data_ptr() if d_min_off is not None else None, n,
                                              out.data_ptr(), s), what)
    return out


VERIFY_EVIL_BIT = 1  # LNX_VERIFY_EVIL_BIT
VERIFY_ICMP = 2      # LNX_VERIFY_ICMP
RX_NO_FCS = 4        # LNX_RX_NO_FCS: the device strips the FCS (x/netdev/interface.go:34-40)
TX_CHECKSUM, TX_FCS = 1, 2  # LNX_TX_CHECKSUM, LNX_TX_FCS
HOST_BATCH_DEFAULT = 64  # LNX_HOST_BATCH_DEFAULT: packet batches below it run on the host


def ingress_verify_batch(d_bytes, d_off, flags: int = 0, out=None, stream=None, filter: RxFilter | None = None):
    """Receive-path checksum verdict per Ethernet frame (lnx_ingress_verify_batch,
    or lnx_ingress_verify_batch_filtered with a stack ``filter``): 0 = checks
    passed / none apply, else lneto's errGeneric code (3 = ErrBadCRC, 2 = ErrPacketDrop, ...)."""
    import torch
    what = "lnx_ingress_verify_batch" if filter is None else "lnx_ingress_verify_batch_filtered"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_off", d_off, "i64")], stream)
    n = d_off.numel() - 1
    out = _out(what, out, n, torch.uint8, "u8", b.device)
    if n > 0:
        with b as s:
            if filter is None:
                rc = lib.lnx_ingress_verify_batch(d_bytes.data_ptr(), d_off.data_ptr(), n, flags, out.data_ptr(), s)
            else:
                rc = lib.lnx_ingress_verify_batch_filtered(d_bytes.data_ptr(), d_off.data_ptr(), n, flags,
                                                           ctypes.byref(filter), out.data_ptr(), s)
            _check(rc, what)
    return out


def rx_verify_batch(d_bytes, d_off, flags: int = 0, filter: RxFilter | None = None, out=None, stream=None):
    """lneto's whole receive check in one pass over each frame (lnx_rx_verify_batch):
    returns (fcs_ok, verdict) uint8 tensors — the FCS residue test of every frame
    d_bytes[d_off[i]:d_off[i+1]] (FCS included) and the verdict of the frame
    without its FCS.  flags: VERIFY_EVIL_BIT | VERIFY_ICMP | RX_NO_FCS."""
    import torch
    what = "lnx_rx_verify_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_off", d_off, "i64")], stream)
    n = d_off.numel() - 1
    ok, verdict = out if out is not None else (None, None)
    ok = _out(what, ok, n, torch.uint8, "u8", b.device)
    verdict = _out(what, verdict, n, torch.uint8, "u8", b.device)
    if n > 0:
        with b as s:
            _check(lib.lnx_rx_verify_batch(d_bytes.data_ptr(), d_off.data_ptr(), n, flags,
                                           ctypes.byref(filter) if filter is not None else None, ok.data_ptr(),
                                           verdict.data_ptr(), s), what)
    return ok, verdict


PCAP_IP_HDR_BAD, PCAP_PROTO_BAD = 1, 2  # LNX_PCAP_IP_HDR_BAD, LNX_PCAP_PROTO_BAD


def pcap_checksums(frame: bytes) -> int:
    """pcap's checksum findings for ONE Ethernet frame on the host
    (lnx_pcap_checksums, internet/pcap/capture.go:67-277): PCAP_IP_HDR_BAD |
    PCAP_PROTO_BAD | code << 2."""
    buf = bytes(frame)
    rc = lib.lnx_pcap_checksums(buf, len(buf))
    if rc < 0:
        _check(rc, "lnx_pcap_checksums")
    return rc


def pcap_verify_batch(d_bytes, d_off, out=None, stream=None):
    """pcap's checksum findings per Ethernet frame d_bytes[d_off[i]:d_off[i+1]]
    (lnx_pcap_verify_batch): a uint8 status tensor, as pcap_checksums."""
    import torch
    what = "lnx_pcap_verify_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_off", d_off, "i64")], stream)
    n = d_off.numel() - 1
    out = _out(what, out, n, torch.uint8, "u8", b.device)
    if n > 0:
        with b as s:
            _check(lib.lnx_pcap_verify_batch(d_bytes.data_ptr(), d_off.data_ptr(), n, out.data_ptr(), s), what)
    return out


def sum16_batch(d_bytes, d_off, d_len, d_seed=None, out=None, stream=None):
    """CRC791{seed[i]}.PayloadSum16(d_bytes[off[i]:off[i]+len[i]]) on the GPU.

    d_off: int64 (N), d_len: int32 (N), d_seed: int32 (N) or None.  Returns int16 (uint16 bits).
    """
    import torch
    what = "lnx_sum16_batch"
    b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_off", d_off, "i64"), ("d_len", d_len, "i32"),
                      ("d_seed", d_seed, "i32?")], stream)
    n = d_off.numel()
    _need_len(what, "d_len", d_len, n)
    _need_len(what, "d_seed", d_seed, n)
    out = _out(what, out, n, torch.int16, "i16", b.device)
    if n > 0:
        with b as s:
            _check(lib.lnx_sum16_batch(d_bytes.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                       d_seed.data_ptr() if d_seed is not None else None, n,
                                       out.data_ptr(), s), what)
    return out


def crc32_batch_multi(parts, devices):
    """lnx_crc32_batch_multi: one host thread per entry of ``devices``; part g is
    a (d_bytes, d_off) pair on device ``devices[g]`` (offsets local to its own
    buffer).  Synchronous; returns one int32 CRC tensor per part.  The same
    device may appear more than once (a one-GPU rehearsal of the partition)."""
    import torch
    what = "lnx_crc32_batch_multi"
    if len(parts) != len(devices) or not parts:
        raise LnetoError(f"{what}: one (d_bytes, d_off) part per device")
    outs = []
    for g, (d_bytes, d_off) in enumerate(parts):
        b = _Batch(what, [("d_bytes", d_bytes, "u8"), ("d_off", d_off, "i64")], None)
        if b.device.index != devices[g]:
            raise LnetoError(f"{what}: part {g} is on {b.device}, devices[{g}] = {devices[g]}")
        outs.append(torch.empty(max(d_off.numel() - 1, 0), dtype=torch.int32, device=b.device))
    ng = len(parts)
    devs = (ctypes.c_int * ng)(*devices)
    bp = (ctypes.c_void_p * ng)(*[p[0].data_ptr() for p in parts])
    op = (ctypes.c_void_p * ng)(*[p[1].data_ptr() for p in parts])
    ns = (ctypes.c_uint64 * ng)(*[max(p[1].numel() - 1, 0) for p in parts])
    cp = (ctypes.c_void_p * ng)(*[o.data_ptr() for o in outs])
    for d in set(devices):  # the library's threads use the null stream: order after torch's work
        torch.cuda.synchronize(d)
    _check(lib.lnx_crc32_batch_multi(ng, devs, bp, op, ns, cp), what)
    return outs


def crc32_batch_host(h_bytes, h_off, device: int = 0):
    """Host-memory convenience (H2D + kernel + D2H); numpy uint8 / uint64 in, uint32 out."""
    import numpy as np
    h_bytes = np.ascontiguousarray(h_bytes, dtype=np.uint8)
    h_off = np.ascontiguousarray(h_off, dtype=np.uint64)
    n = len(h_off) - 1
    out = np.zeros(max(n, 1), dtype=np.uint32)
    if n > 0:
        _check(lib.lnx_crc32_batch_host(h_bytes.ctypes.data, h_bytes.nbytes, h_off.ctypes.data, n,
                                        out.ctypes.data, device), "lnx_crc32_batch_host")
    return out[:max(n, 0)]


class RxRing:
    """Pinned receive ring + batched FCS verify / ingress verdicts (lnx_rx_ring_*,
    SURVEY.md §8(f).1), the batch form of netdev.Stack.IngressPackets
    (x/netdev/interface.go:82-89) over bufferSelect-style slots (x/netdev/buffer.go).

    ``slots`` is a (nslots, slot_cap) uint8 numpy view of the pinned slot memory
    and ``lengths`` a uint32 view of the per-slot buffer lengths: a producer
    writes frames (with their FCS) there, then ``ingress(first, count, offset)``
    returns (fcs_ok, verdict) uint8 arrays.  ``ingress_packets(bufs, offset)``
    takes caller-owned buffers instead (IngressPackets(bufs, offset) exactly).
    """

    def __init__(self, nslots: int, slot_cap: int = 2048, batch_slots: int = 0, depth: int = 3, device: int = 0,
                 host_threshold: int | None = None):
        import numpy as np
        h = _vp()
        _check(lib.lnx_rx_ring_create(device, nslots, slot_cap, batch_slots, depth, ctypes.byref(h)),
               "lnx_rx_ring_create")
        self._h = h
        if host_threshold is not None:
            self.set_host_threshold(host_threshold)
        self.nslots, self.slot_cap = nslots, slot_cap
        sp = lib.lnx_rx_ring_slots(h)
        lp = lib.lnx_rx_ring_lengths(h)
        self.slots = np.ctypeslib.as_array((ctypes.c_uint8 * (nslots * slot_cap)).from_address(sp)).reshape(
            nslots, slot_cap)
        self.lengths = np.ctypeslib.as_array((ctypes.c_uint32 * nslots).from_address(lp))

    def set_host_threshold(self, frames: int) -> None:
        """Batches of fewer frames run on the host, no launch (lnx_rx_ring_set_host_threshold;
        HOST_BATCH_DEFAULT unless set; 0 = every batch on the GPU)."""
        _check(lib.lnx_rx_ring_set_host_threshold(self._h, frames), "lnx_rx_ring_set_host_threshold")

    def stats(self) -> dict:
        """{host_frames, device_frames, device_batches, zero_copy_frames} since creation (lnx_rx_ring_stats)."""
        c = (ctypes.c_uint64 * 4)()
        _check(lib.lnx_rx_ring_stats(self._h, c), "lnx_rx_ring_stats")
        return {"host_frames": c[0], "device_frames": c[1], "device_batches": c[2], "zero_copy_frames": c[3]}

    def set_zero_copy(self, on: bool) -> None:
        """Kernels read (egress: patch) frames in place in the pinned slots (the default), or
        copy them through staging (lnx_rx_ring_set_zero_copy)."""
        _check(lib.lnx_rx_ring_set_zero_copy(self._h, int(bool(on))), "lnx_rx_ring_set_zero_copy")

    def set_filter(self, filt: RxFilter | None) -> None:
        """The ring's stack configuration (lnx_rx_ring_set_filter); None = accept-all."""
        _check(lib.lnx_rx_ring_set_filter(self._h, ctypes.byref(filt) if filt is not None else None),
               "lnx_rx_ring_set_filter")

    def ingress(self, first: int = 0, count: int | None = None, offset: int = 0, flags: int = 0):
        import numpy as np
        if count is None:
            count = self.nslots - first
        ok = np.zeros(max(count, 1), dtype=np.uint8)
        verdict = np.zeros(max(count, 1), dtype=np.uint8)
        _check(lib.lnx_rx_ring_ingress(self._h, first, count, offset, flags, ok.ctypes.data, verdict.ctypes.data),
               "lnx_rx_ring_ingress")
        return ok[:count], verdict[:count]

    def ingress_packets(self, bufs, offset: int = 0, flags: int = 0):
        import numpy as np
        if not isinstance(offset, int) or not 0 <= offset < 2**32:
            raise LnetoError("ingress_packets: offset must be an int in [0, 2**32)")
        arrs = [np.frombuffer(bytes(b), dtype=np.uint8) if not isinstance(b, np.ndarray)
                else np.ascontiguousarray(b, dtype=np.uint8) for b in bufs]
        n = len(arrs)
        ptrs = (ctypes.c_void_p * max(n, 1))(*[a.ctypes.data if a.size else None for a in arrs])
        lens = np.array([a.size for a in arrs] or [0], dtype=np.uint32)
        ok = np.zeros(max(n, 1), dtype=np.uint8)
        verdict = np.zeros(max(n, 1), dtype=np.uint8)
        _check(lib.lnx_ingress_packets(self._h, ptrs, lens.ctypes.data, n, offset, flags, ok.ctypes.data,
                                       verdict.ctypes.data), "lnx_ingress_packets")
        return ok[:n], verdict[:n]

    def egress_packets(self, bufs, sizes, offset: int = 0, capacity: int | None = None,
                       flags: int = 3):
        """EgressPackets(bufs, sizes, offset) for the device's part of the transmit
        path (lnx_egress_packets): bufs are writable uint8 numpy arrays, frame k =
        bufs[k][offset : offset + sizes[k]]; flags TX_CHECKSUM | TX_FCS.  The frames
        are finished in place; returns (new sizes, status) as uint32 / uint8 arrays."""
        import numpy as np
        n = len(bufs)
        if not isinstance(offset, int) or not 0 <= offset < 2**32:
            raise LnetoError("egress_packets: offset must be an int in [0, 2**32)")
        if not isinstance(capacity, (int, type(None))) or (capacity is not None and not 0 <= capacity < 2**32):
            raise LnetoError("egress_packets: capacity must be an int in [0, 2**32)")
        for b in bufs:
            if not isinstance(b, np.ndarray) or b.dtype != np.uint8 or not b.flags.c_contiguous \
                    or not b.flags.writeable:
                raise LnetoError("egress_packets: bufs must be writable contiguous uint8 numpy arrays")
        if capacity is None:
            capacity = self.slot_cap
        sz = np.asarray(sizes)
        if sz.size and (sz.dtype.kind not in "iu" or sz.min() < 0 or sz.max() >= 2**32):
            raise LnetoError("egress_packets: sizes must be non-negative integers below 2**32")
        lens = np.ascontiguousarray(sz.astype(np.uint32)).copy()
        if len(lens) != n:
            raise LnetoError("egress_packets: one size per buffer")
        for b, l in zip(bufs, lens):  # the finished frame is written back at bufs[k][offset:]
            if b.size - offset < min(capacity, max(int(l), 60) + 4):
                raise LnetoError("egress_packets: each buffer needs room for its padded frame and FCS "
                                 "(min(capacity, max(size, 60) + 4) bytes from offset)")
        ptrs = (ctypes.c_void_p * max(n, 1))(*[b.ctypes.data for b in bufs])
        status = np.zeros(max(n, 1), dtype=np.uint8)
        _check(lib.lnx_egress_packets(self._h, ptrs, lens.ctypes.data, n, offset, capacity, flags,
                                      status.ctypes.data), "lnx_egress_packets")
        return lens[:n], status[:n]

    def close(self) -> None:
        if getattr(self, "_h", None):
            self.slots = self.lengths = None
            lib.lnx_rx_ring_destroy(self._h)
            self._h = None

    def __del__(self):
        self.close()


RESEARCH_LIB_PATH = os.path.join(HERE, "liblneto_amd_research.so")
_research = None


def research_lib():
    """The research library (liblneto_amd_research.so): the same C-ABI plus the
    losing kernel variants and the lnx__* profiling hooks of DESIGN.md §3-4.
    Only tools/ and the variant tests use it; the product path never does."""
    global _research
    if _research is None:
        if not os.path.exists(RESEARCH_LIB_PATH):
            raise ImportError(f"{RESEARCH_LIB_PATH} is not built (make -C lneto_amd/csrc)")
        _research = ctypes.CDLL(RESEARCH_LIB_PATH)
    return _research


def device_count() -> int:
    return lib.lnx_device_count()


def version() -> str:
    return lib.lnx_version().decode()


def _elf_section(path: str, name: str) -> bytes:
    """Bytes of section `name` of the ELF64 little-endian file at `path`."""
    import struct
    with open(path, "rb") as fh:
        blob = fh.read()
    if blob[:4] != b"\x7fELF" or blob[4] != 2 or blob[5] != 1:
        raise ValueError(f"{path}: not an ELF64 little-endian file")
    shoff, = struct.unpack_from("<Q", blob, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", blob, 0x3A)
    def sh(i):
        return struct.unpack_from("<IIQQQQIIQQ", blob, shoff + i * shentsize)
    stroff = sh(shstrndx)[4]
    for i in range(shnum):
        nm, _, _, _, off, size = sh(i)[:6]
        end = blob.index(b"\0", stroff + nm)
        if blob[stroff + nm:end].decode() == name:
            return blob[off:off + size]
    raise KeyError(f"{path}: no section {name}")


def build_id(path: str | None = None) -> str:
    """sha256 (16 hex digits) of the gfx950 code objects (.hip_fatbin) of the
    loaded library: the kernels' identity, unlike version(), a hand-written
    string.  bench.py records it beside every line and compares it with the
    one a committed PMC pass (profiles/counters_*.json) was taken on."""
    import hashlib
    return hashlib.sha256(_elf_section(path or LIB_PATH, ".hip_fatbin")).hexdigest()[:16]
