"""The library's host path (lneto_amd/csrc/host_path.cpp):
the per-frame receive verdict, transmit checksum and FCS append that the
packet entries run below their host threshold (so netdev's one-buffer-per-call
Runner, x/netdev/runner.go:432-433, never launches a kernel).  CPU only,
through the C-ABI, against the oracle (oracle.ingress_verdict /
StackFilter, tx_checksum, fcs_append) on the same frame generators as the GPU
verdict tests."""
import ctypes

import numpy as np
import pytest

from oracle import oracle as O
from tests import framegen as G
from tests.test_rx_filter import FILTERS, _pair

import lneto_amd as L


def _verdict(frame: bytes, flags: int = 0, filt=None) -> int:
    return L.lib.lnx_ingress_verdict(frame, len(frame), flags, ctypes.byref(filt) if filt is not None else None)


@pytest.mark.parametrize("flags", [0, O.VERIFY_EVIL_BIT, O.VERIFY_ICMP, O.VERIFY_EVIL_BIT | O.VERIFY_ICMP])
def test_host_verdicts_match_oracle(flags):
    frames = G.frames(seed=3, count=3000) + G.icmp_frames(seed=4, count=600) + G.trailing_frames(seed=5, count=300)
    got = [_verdict(f, flags) for f in frames]
    want = [O.ingress_verdict(f, flags) for f in frames]
    bad = [i for i in range(len(frames)) if got[i] != want[i]]
    assert not bad, [(i, got[i], want[i]) for i in bad[:10]]


@pytest.mark.parametrize("name", sorted(FILTERS))
def test_host_filtered_verdicts_match_oracle(name):
    ofilt, cfilt = _pair(name)
    frames = G.filter_frames(seed=31, count=2400)
    for flags in (0, O.VERIFY_ICMP):
        got = [_verdict(f, flags, cfilt) for f in frames]
        want = [O.ingress_verdict(f, flags, ofilt) for f in frames]
        bad = [i for i in range(len(frames)) if got[i] != want[i]]
        assert not bad, [(i, got[i], want[i]) for i in bad[:10]]


def test_host_verdict_reference_frames():
    """lneto_test.go:119-160's two TCP SYN frames pass; each flipped byte of
    the IPv4 header or the TCP segment makes ErrBadCRC (3) or an earlier error."""
    from tests.test_ingress import _kat_frames
    for f in _kat_frames():
        assert _verdict(f) == 0
        for i in range(14, len(f)):
            b = bytearray(f)
            b[i] ^= 0x10
            assert _verdict(bytes(b)) == O.ingress_verdict(bytes(b)) != 0


def test_filter_rejects_ethertypes_register_ethernet_rejects():
    """RegisterEthernet rejects proto <= 1500 (internet/stack-ethernet.go:131-135):
    the C-ABI returns LNX_EINVAL for such a filter, the Python builder raises."""
    f = L.RxFilter.make(mac=G.MAC_US)
    f.ethertypes[1] = 1500
    assert L.lib.lnx_ingress_verdict(b"\0" * 60, 60, 0, ctypes.byref(f)) == L.LNX_EINVAL
    f.ethertypes[1] = 1501
    assert L.lib.lnx_ingress_verdict(b"\0" * 60, 60, 0, ctypes.byref(f)) >= 0
    with pytest.raises(L.LnetoError):
        L.RxFilter.make(mac=G.MAC_US, ethertypes=(0x0800, 46))


def _tx_cases():
    rng = np.random.default_rng(61)
    out = []
    for i in range(1500):
        kind = i % 9
        n = int(rng.integers(0, 1480))
        pay = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        if kind == 0:
            f = G.ether(0x0800, G.ipv4(17, G.udp(pay)))
        elif kind == 1:
            f = G.ether(0x0800, G.ipv4(6, G.tcp(pay)))
        elif kind == 2:
            f = G.ether(0x86DD, G.ipv6(17, G.udp(pay)))
        elif kind == 3:
            f = G.ether(0x86DD, G.ipv6(6, G.tcp(pay)))
        elif kind == 4:
            f = G.ether(0x0800, G.ipv4(1, G.icmp(8, pay)))
        elif kind == 5:
            f = G.ether(0x86DD, G.ipv6(58, G.icmp(128, pay)))
        elif kind == 6:
            f = G.ether(0x0806, pay)
        elif kind == 7:  # truncated
            f = G.ether(0x0800, G.ipv4(6, G.tcp(pay)))[: int(rng.integers(0, 60))]
        else:  # IHL below 5 / options
            b = bytearray(G.ether(0x0800, G.ipv4(17, G.udp(pay), opts=b"\x01\x01\x01\x01")))
            if i % 2:
                b[14] = 0x44
            f = bytes(b)
        # garble the fields the step writes: it must not depend on them
        b = bytearray(f)
        for j in rng.integers(0, max(1, len(b)), 3):
            if len(b):
                b[int(j)] ^= 0x5A
        out.append(bytes(b) if kind >= 7 else f)
    return out


def test_host_tx_checksum_matches_oracle():
    for f in _tx_cases():
        buf = (ctypes.c_uint8 * max(1, len(f))).from_buffer_copy(f + b"\0" * (len(f) == 0))
        st = L.lib.lnx_tx_checksum(buf, len(f))
        want, wst = O.tx_checksum(f)
        assert st == wst and bytes(buf)[: len(f)] == want, (f[:16].hex(), st, wst)
        if wst == 0 and f[12:14] in (b"\x08\x00", b"\x86\xdd"):
            assert O.ingress_verdict(want) in (0, O.ERR_INVALID_LENGTH_FIELD, O.ERR_TRUNCATED_FRAME)


@pytest.mark.parametrize("cap", [64, 100, 1518, 1536])
def test_host_fcs_append_matches_oracle(cap):
    rng = np.random.default_rng(cap)
    for n in list(range(0, 70)) + [int(x) for x in rng.integers(0, 1530, 200)]:
        f = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        buf = (ctypes.c_uint8 * max(cap, n, 1))()
        ctypes.memmove(buf, f, n)
        ln = ctypes.c_uint32(n)
        st = L.lib.lnx_fcs_append(buf, ctypes.byref(ln), cap)
        want, wst = O.fcs_append(f, cap)
        assert st == wst and ln.value == len(want) and bytes(buf)[: ln.value] == want, (n, cap, st, wst)
        if st == 0:
            assert O.crc32(want) == O.CRC32_RESIDUE
