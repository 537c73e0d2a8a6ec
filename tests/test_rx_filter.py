"""Destination and handler precedence of the receive verdicts (lnx_rx_filter,
oracle.StackFilter): ErrPacketDrop where lneto drops a frame the stack would
not accept, before or after the other checks exactly where the reference does
it — StackEthernet.Demux (internet/stack-ethernet.go:146-161), demux4
(internet/stack-ip4.go:108-141), demux6 (internet/stack-ip6.go:93-111).  The
CPU tests pin the oracle on hand-built cases; the GPU tests compare the kernel
(lnx_ingress_verify_batch_filtered) and the ring (lnx_rx_ring_set_filter) with it."""
import struct

import numpy as np
import pytest

from oracle import oracle as O
from tests import framegen as G

DROP, BAD, TRUNC, LEN = O.ERR_PACKET_DROP, O.ERR_BAD_CRC, O.ERR_TRUNCATED_FRAME, O.ERR_INVALID_LENGTH_FIELD
OTHER_MAC = bytes.fromhex("02aabbccddee")
MCAST_MAC = bytes.fromhex("01005e000001")


def _f(**kw):
    return O.StackFilter(mac=G.MAC_US, ip4=G.IP4_DST, ip6=G.IP6_DST, **kw)


def _dst(frame: bytes, mac: bytes) -> bytes:
    return mac + frame[6:]


def _flip(frame: bytes, i: int) -> bytes:
    b = bytearray(frame)
    b[i] ^= 0x01
    return bytes(b)


def test_ethernet_destination_precedes_size_checks():
    ok = G.ether(0x0800, G.ipv4(6, G.tcp(b"hello")))
    f = _f()
    assert O.ingress_verdict(ok, 0, f) == 0
    assert O.ingress_verdict(_dst(ok, b"\xff" * 6), 0, f) == 0              # broadcast: always accepted
    assert O.ingress_verdict(_dst(_flip(ok, 24), OTHER_MAC), 0, f) == DROP  # not for us: before the header sum
    assert O.ingress_verdict(_flip(ok, 24), 0, f) == BAD
    short = G.ether(1000, b"x" * 10)                                       # size field > frame: ValidateSize
    assert O.ingress_verdict(_dst(short, OTHER_MAC), 0, f) == DROP           # ... comes after the MAC check
    assert O.ingress_verdict(short, 0, f) == LEN
    assert O.ingress_verdict(_dst(ok, MCAST_MAC), 0, f) == DROP
    assert O.ingress_verdict(_dst(ok, MCAST_MAC), 0, _f(eth_accept_multicast=True)) == 0
    assert O.ingress_verdict(_dst(ok, OTHER_MAC), 0, _f(eth_accept_multicast=True)) == DROP  # unicast: no group bit
    assert O.ingress_verdict(ok[:13], 0, f) == TRUNC                       # ethernet.NewFrame first of all


def test_ethertype_handler_after_size_checks():
    f = _f()
    lldp = G.ether(0x88CC, bytes(46))
    assert O.ingress_verdict(lldp, 0, f) == DROP
    assert O.ingress_verdict(lldp, 0, None) == 0
    assert O.ingress_verdict(G.ether(0x0806, bytes(28)), 0, f) == 0          # ARP has a handler: nothing to check
    assert O.ingress_verdict(G.ether(0x8100, b"ab"), 0, f) == TRUNC          # VLAN size check before the handler
    assert O.ingress_verdict(G.ether(0x8100, bytes(40)), 0, f) == DROP
    assert O.ingress_verdict(G.ether(46, bytes(46)), 0, f) == DROP           # a size field: no handler
    assert O.ingress_verdict(G.ether(0x0800, G.ipv4(6, G.tcp(b""))), 0,
                             O.StackFilter(mac=G.MAC_US, ethertypes=(0x86DD,))) == DROP


def test_ipv4_destination_and_protocol():
    f = _f()
    other = bytes([192, 168, 10, 77])
    mk = lambda proto, l4, dst=G.IP4_DST: G.ether(0x0800, G.ipv4(proto, l4, dst=dst))
    tcp_other = mk(6, G.tcp(b"abc"), other)
    assert O.ingress_verdict(tcp_other, 0, f) == DROP
    assert O.ingress_verdict(_flip(tcp_other, 24), 0, f) == DROP             # before the header sum
    b = bytearray(tcp_other); b[16:18] = struct.pack(">H", 19)
    assert O.ingress_verdict(bytes(b), 0, f) == DROP                         # before ValidateExceptCRC
    assert O.ingress_verdict(tcp_other[:14 + 19], 0, f) == TRUNC             # ipv4.NewFrame still first
    assert O.ingress_verdict(tcp_other, 0, O.StackFilter(mac=G.MAC_US)) == 0  # 0.0.0.0: accept every destination
    mc = mk(17, G.udp(b"mdns"), bytes([224, 0, 0, 251]))
    bc = mk(17, G.udp(b"dhcp"), b"\xff" * 4)
    assert O.ingress_verdict(mc, 0, f) == DROP and O.ingress_verdict(bc, 0, f) == DROP
    assert O.ingress_verdict(mc, 0, _f(ip4_accept_multicast=True)) == 0
    assert O.ingress_verdict(bc, 0, _f(ip4_accept_multicast=True)) == DROP
    assert O.ingress_verdict(bc, 0, _f(ip4_accept_broadcast=True)) == 0
    gre = mk(47, b"payload-of-gre")
    assert O.ingress_verdict(gre, 0, f) == DROP                              # no handler
    assert O.ingress_verdict(_flip(gre, 24), 0, f) == BAD                    # ... but the header sum comes first
    tcp_ok = mk(6, G.tcp(b"abc"))
    no_tcp = O.StackFilter(mac=G.MAC_US, ip4=G.IP4_DST, ip4_protocols=(17,))
    assert O.ingress_verdict(_flip(tcp_ok, 55), 0, no_tcp) == DROP           # before the TCP sum
    assert O.ingress_verdict(_flip(tcp_ok, 55), 0, f) == BAD


def test_ipv6_destination_and_protocol():
    f = _f()
    mk = lambda proto, l4, dst=G.IP6_DST: G.ether(0x86DD, G.ipv6(proto, l4, dst=dst))
    other = mk(17, G.udp(b"x"), bytes(range(0x50, 0x60)))
    assert O.ingress_verdict(other, 0, f) == DROP
    assert O.ingress_verdict(other[:-1], 0, f) == DROP                       # before ValidateSize
    assert O.ingress_verdict(other[:-1], 0, None) == LEN
    mc = mk(17, G.udp(b"x"), bytes.fromhex("ff020000000000000000000000000001"))
    assert O.ingress_verdict(mc, 0, f) == DROP
    assert O.ingress_verdict(mc, 0, _f(ip6_accept_multicast=True)) == 0
    gre = mk(47, b"gre!")
    assert O.ingress_verdict(gre, 0, f) == DROP
    assert O.ingress_verdict(gre[:-1], 0, f) == LEN                          # ValidateSize before the handler
    udp_bad = _flip(mk(17, G.udp(b"abcdef")), 62)
    assert O.ingress_verdict(udp_bad, 0, f) == BAD
    assert O.ingress_verdict(udp_bad, 0, O.StackFilter(mac=G.MAC_US, ip6=G.IP6_DST, ip6_protocols=(6,))) == DROP


FILTERS = {
    "plain": dict(ip4=G.IP4_DST, ip6=G.IP6_DST),
    "accept_all_ips": dict(),
    "multicast": dict(ip4=G.IP4_DST, ip6=G.IP6_DST, eth_accept_multicast=True, ip4_accept_multicast=True,
                      ip4_accept_broadcast=True, ip6_accept_multicast=True),
    "few_handlers": dict(ip4=G.IP4_DST, ip6=G.IP6_DST, ethertypes=(0x0800, 0x88CC), ip4_protocols=(17, 47),
                         ip6_protocols=(58,)),
}


def _pair(name):
    import lneto_amd as L
    kw = FILTERS[name]
    return O.StackFilter(mac=G.MAC_US, **kw), L.RxFilter.make(mac=G.MAC_US, **kw)


def test_filter_generator_covers_every_precedence():
    import collections
    fr = G.filter_frames(count=1200)
    hist = collections.Counter(O.ingress_verdict(x, O.VERIFY_ICMP, _pair("plain")[0]) for x in fr)
    for code in (0, DROP, BAD, TRUNC, LEN):
        assert hist[code] > 0, hist


def _pack(frames, base_pad):
    parts, offs, pos = [b"\xAA" * base_pad], [base_pad], base_pad
    for f in frames:
        parts.append(f)
        pos += len(f)
        offs.append(pos)
    return np.frombuffer(b"".join(parts) + b"\0" * 8, dtype=np.uint8).copy(), np.array(offs, dtype=np.uint64)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(FILTERS))
@pytest.mark.parametrize("base_pad", [0, 3, 6])
def test_gpu_filtered_verdicts_match_oracle(cuda, name, base_pad):
    import torch
    import lneto_amd as L
    ofilt, cfilt = _pair(name)
    frames = G.filter_frames(seed=31 + base_pad, count=2400)
    data, off = _pack(frames, base_pad)
    d = torch.from_numpy(data).to(cuda)
    o = torch.from_numpy(off.astype(np.int64)).to(cuda)
    for flags in (0, L.VERIFY_ICMP):
        got = L.ingress_verify_batch(d, o, flags=flags, filter=cfilt).cpu().numpy()
        want = np.array([O.ingress_verdict(f, flags, ofilt) for f in frames], dtype=np.uint8)
        bad = np.nonzero(got != want)[0]
        assert bad.size == 0, [(int(i), int(got[i]), int(want[i]), frames[i][:14].hex()) for i in bad[:10]]


@pytest.mark.gpu
def test_gpu_unfiltered_entry_is_accept_all(cuda):
    """lnx_ingress_verify_batch == the filtered entry with a NULL filter."""
    import torch
    import lneto_amd as L
    frames = G.filter_frames(seed=5, count=600)
    data, off = _pack(frames, 1)
    d, o = torch.from_numpy(data).to(cuda), torch.from_numpy(off.astype(np.int64)).to(cuda)
    got = L.ingress_verify_batch(d, o).cpu().numpy()
    assert got.tolist() == [O.ingress_verdict(f) for f in frames]


def test_filter_struct_rejects_too_many_ethertypes():
    import lneto_amd as L
    with pytest.raises(L.LnetoError):
        L.RxFilter.make(mac=G.MAC_US, ethertypes=tuple(range(0x800, 0x809)))
    f = L.RxFilter.make(mac=G.MAC_US)
    f.n_ethertypes = 9
    assert L.lib.lnx_ingress_verify_batch_filtered(None, None, 0, 0, L.ctypes.byref(f), None, None) == L.LNX_EINVAL
