"""CPU oracle for lneto's checksum path — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module, and only as the checker / the timed CPU baseline.  The product
(lneto_amd/) never imports it.

Two independent restatements live here:

* pure-Python / zlib (this file):
    - crc32 / crc32_update  == Go crc32.Checksum / crc32.Update(IEEETable)
      (lneto ethernet/crc.go:13,19-21,36,44).  zlib.crc32 implements the same
      CRC-32/ISO-HDLC algorithm as Go's hash/crc32 (stdlib dependency, not in
      the reference tree; go.mod:3 floor go1.24, CI go1.26 ci.yaml:109).
    - crc32_search          == ethernet/crc.go:28-47
    - sum_write_even / sum16 / payload_sum16 / never_zero_sum == crc.go:17-71
    - ipv4_* / ipv6_* pseudo-header seeds == ipv4/frame.go:138-170,
      ipv6/frame.go:104-108
* C (oracle/crc_oracle.c, built to oracle/liboracle.so), used for speed and as
  the bench's CPU baseline ("port").

Pinning: tests/test_oracle.py checks both against the reference's own
known-answer vectors (lneto_test.go:119-160 IPv4/TCP sums; ethernet/crc_test.go
self-consistency cases) and against the CRC-32/ISO-HDLC check value.
"""
from __future__ import annotations

import ctypes
import os
import struct
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")

CRC32_CHECK = 0xCBF43926   # CRC-32/ISO-HDLC of b"123456789"
CRC32_RESIDUE = 0x2144DF1C  # CRC32(m || LE32(CRC32(m))) for every m


# --------------------------------------------------------------------------- CRC-32
def crc32_update(crc: int, p: bytes) -> int:
    """Go crc32.Update(crc, crc32.IEEETable, p)."""
    return zlib.crc32(bytes(p), crc) & 0xFFFFFFFF


def crc32(p: bytes) -> int:
    """ethernet.CRC32 (ethernet/crc.go:19-21)."""
    return zlib.crc32(bytes(p)) & 0xFFFFFFFF


def crc32_bitwise(p: bytes, crc: int = 0) -> int:
    """Bit-serial CRC-32/ISO-HDLC (third restatement, small inputs only)."""
    c = (~crc) & 0xFFFFFFFF
    for b in bytes(p):
        c ^= b
        for _ in range(8):
            c = (c >> 1) ^ (0xEDB88320 if c & 1 else 0)
    return (~c) & 0xFFFFFFFF


def crc32_search(data: bytes, min_off: int) -> int:
    """ethernet.CRC32Search (ethernet/crc.go:28-47)."""
    if min_off < 0:
        min_off = 0
    if len(data) < min_off + 4:
        return -1
    c = crc32(data[:min_off])
    for off in range(min_off, len(data) - 3):
        got = struct.unpack_from("<I", data, off)[0]
        if c == got:
            return off
        c = crc32_update(c, data[off:off + 1])
    return -1


# ------------------------------------------------------------------ RFC 791 sum
def sum_write_even(s: int, buff: bytes) -> int:
    """sumWriteEven (crc.go:23-28): uint32 wrap-around add of BE16 words."""
    for i in range(0, len(buff) - 1, 2):
        s = (s + ((buff[i] << 8) | buff[i + 1])) & 0xFFFFFFFF
    return s


def sum16(s: int) -> int:
    """sum16 (crc.go:17-21)."""
    s = (s & 0xFFFF) + (s >> 16)
    return (~(s + (s >> 16))) & 0xFFFF


def payload_sum16(s: int, buff: bytes) -> int:
    """(*CRC791).PayloadSum16 (crc.go:52-59), receiver sum = s."""
    odd = len(buff) & 1
    s = sum_write_even(s, buff[:len(buff) - odd])
    if odd:
        s = (s + (buff[-1] << 8)) & 0xFFFFFFFF
    return sum16(s)


def never_zero_sum(x: int) -> int:
    """NeverZeroSum (crc.go:65-71)."""
    return 0xFFFF if x == 0 else x


class CRC791:
    """Restatement of lneto.CRC791 (crc.go:13-62)."""

    def __init__(self) -> None:
        self.sum = 0

    def write_even(self, buff: bytes) -> None:
        if len(buff) & 1:
            raise IndexError("WriteEven: odd length (crc.go:30 panics)")
        self.sum = sum_write_even(self.sum, buff)

    def add_uint16(self, v: int) -> None:
        self.sum = (self.sum + (v & 0xFFFF)) & 0xFFFFFFFF

    def add_uint32(self, v: int) -> None:
        self.add_uint16(v >> 16)
        self.add_uint16(v)

    def sum16(self) -> int:
        return sum16(self.sum)

    def payload_sum16(self, buff: bytes) -> int:
        return payload_sum16(self.sum, buff)

    def reset(self) -> None:
        self.sum = 0


# ----------------------------------------------------- IPv4 / IPv6 pseudo-headers
def ipv4_header_sum16(ip: bytes) -> int:
    """ipv4.Frame.CalculateHeaderCRC (ipv4/frame.go:138-146): first 20 bytes only."""
    c = CRC791()
    c.write_even(ip[:20])
    return c.sum16()


def ipv4_tcp_pseudo(ip: bytes) -> CRC791:
    """ipv4.Frame.CRCWriteTCPPseudo (ipv4/frame.go:154-158)."""
    c = CRC791()
    c.write_even(ip[12:20])
    total_len = (ip[2] << 8) | ip[3]
    ihl = (ip[0] & 0xF) * 4
    c.add_uint16((total_len - ihl) & 0xFFFF)
    c.add_uint16(ip[9])
    return c


def ipv4_udp_pseudo(ip: bytes, udp_length: int) -> CRC791:
    """ipv4.Frame.CRCWriteUDPPseudo (ipv4/frame.go:166-170)."""
    c = CRC791()
    c.write_even(ip[12:20])
    c.add_uint16(udp_length)
    c.add_uint16(ip[9])
    return c


def ipv6_pseudo(ip6: bytes) -> CRC791:
    """ipv6.Frame.CRCWritePseudo (ipv6/frame.go:104-108)."""
    c = CRC791()
    c.write_even(ip6[8:40])
    c.add_uint32((ip6[4] << 8) | ip6[5])
    c.add_uint32(ip6[6])
    return c


# ------------------------------------------- receive-path checksum verdicts
# lneto.errGeneric codes (errors.go:6-28) the receive path returns.
ERR_PACKET_DROP = 2
ERR_BAD_CRC = 3
ERR_INVALID_FIELD = 14
ERR_INVALID_LENGTH_FIELD = 15
ERR_TRUNCATED_FRAME = 18
VERIFY_EVIL_BIT = 1  # mirrors lneto.ValidateEvilBit on the stack's Validator
# ICMP clients attached: their Demux checks up to and including the checksum
# (ipv4/icmpv4/client.go:89-102, ipv6/icmpv6/client.go:100-115)
VERIFY_ICMP = 2
ICMPV4_ECHO_REPLY, ICMPV4_ECHO = 0, 8  # ipv4/icmpv4/icmpv4.go:18-19

ETHERTYPE_IPV4 = 0x0800
ETHERTYPE_IPV6 = 0x86DD
ETHERTYPE_VLAN = 0x8100
IPPROTO_TCP = 6
IPPROTO_UDP = 17
IPPROTO_ICMP = 1     # definitions.go:48
IPPROTO_ICMPV6 = 58  # definitions.go:105


def _be16(b: bytes, i: int) -> int:
    return (b[i] << 8) | b[i + 1]


class StackFilter:
    """The stack configuration the receive path consults before and between its
    checksum checks (mirrors lnx_rx_filter, include/lneto_amd.h):
    StackEthernet's MAC and SetAcceptMulticast (internet/stack-ethernet.go:56-58,
    146-152) and its handlers by EtherType (RegisterEthernet, :158-161); stackip4's
    address, SetAcceptMulticast / SetAcceptBroadcast and handlers by protocol
    (internet/stack-ip4.go:88-93,108-119,135-141); stackip6's address,
    SetAcceptMulticast6 and handlers (internet/stack-ip6.go:74,93-111)."""

    def __init__(self, mac: bytes, ethertypes=(0x0800, 0x86DD, 0x0806), ip4: bytes = bytes(4),
                 ip6: bytes = bytes(16), ip4_protocols=(1, 6, 17), ip6_protocols=(6, 17, 58),
                 eth_accept_multicast=False, ip4_accept_multicast=False, ip4_accept_broadcast=False,
                 ip6_accept_multicast=False):
        self.mac, self.ethertypes, self.ip4, self.ip6 = bytes(mac), set(ethertypes), bytes(ip4), bytes(ip6)
        self.ip4_protocols, self.ip6_protocols = set(ip4_protocols), set(ip6_protocols)
        self.eth_accept_multicast, self.ip4_accept_multicast = eth_accept_multicast, ip4_accept_multicast
        self.ip4_accept_broadcast, self.ip6_accept_multicast = ip4_accept_broadcast, ip6_accept_multicast


def _ipv4_verdict(ip: bytes, flags: int, filt: StackFilter | None = None) -> int:
    """demux4 up to its checksum checks (internet/stack-ip4.go:100-164).  With
    no filter every destination is accepted and every protocol has a handler."""
    if len(ip) < 20:                                   # ipv4.NewFrame (ipv4/frame.go:15-20)
        return ERR_TRUNCATED_FRAME
    if filt is not None and filt.ip4 != bytes(4) and ip[16:20] != filt.ip4:   # stack-ip4.go:108-119
        dst = ip[16:20]
        mc = dst[0] & 0xF0 == 0xE0                     # ipv4.IsMulticast (ipv4/definitions.go:17-19)
        bc = dst == b"\xff\xff\xff\xff"                # ipv4.IsBroadcast (:34-36)
        if not (filt.ip4_accept_multicast and mc) and not (filt.ip4_accept_broadcast and bc):
            return ERR_PACKET_DROP
    # ValidateExceptCRC (ipv4/frame.go:229-238) on a Validator without
    # validateAllowMultiErrors: the first error added wins (validation.go AddError).
    tl, ihl, version = _be16(ip, 2), ip[0] & 0xF, ip[0] >> 4
    errs = []
    if tl < 20:                                        # ValidateSize (ipv4/frame.go:214-227)
        errs.append(ERR_INVALID_LENGTH_FIELD)
    if tl > len(ip):
        errs.append(ERR_TRUNCATED_FRAME)
    if ihl < 5 or ihl * 4 > tl:
        errs.append(ERR_INVALID_LENGTH_FIELD)
    if version != 4:
        errs.append(ERR_INVALID_FIELD)
    if flags & VERIFY_EVIL_BIT and _be16(ip, 6) & (1 << 13):  # Flags.IsEvil (ipv4/definitions.go:68-87)
        errs.append(ERR_PACKET_DROP)
    if errs:
        return errs[0]
    if ipv4_header_sum16(ip) != 0:                     # CalculateHeaderCRC: first 20 bytes only
        return ERR_BAD_CRC
    hl, proto = ihl * 4, ip[9]
    payload = ip[hl:tl]                                # Frame.Payload (ipv4/frame.go:188-192)
    if filt is not None and proto not in filt.ip4_protocols:
        return ERR_PACKET_DROP                         # nodeByProto nil (stack-ip4.go:135-141)
    if proto == IPPROTO_TCP:
        if ipv4_tcp_pseudo(ip).payload_sum16(payload) != 0:
            return ERR_BAD_CRC
    elif proto == IPPROTO_UDP:
        if len(payload) < 8:                           # udp.NewFrame (udp/frame.go:15-20)
            return ERR_TRUNCATED_FRAME
        ul = _be16(payload, 4)
        if ul < 8:                                     # udp ValidateSize (udp/frame.go:96-104)
            return ERR_INVALID_LENGTH_FIELD
        if ul > len(payload):
            return ERR_TRUNCATED_FRAME
        if ipv4_udp_pseudo(ip, ul).payload_sum16(payload[:ul]) != 0:
            return ERR_BAD_CRC
    elif proto == IPPROTO_ICMP and flags & VERIFY_ICMP:
        # demux4 hands frame[:tl] at offset hl to the ICMP client
        # (stack-ip4.go:168-170); its Demux (ipv4/icmpv4/client.go:89-102):
        if len(payload) < 8:                           # icmpv4.NewFrame (icmpv4.go:62-67)
            return ERR_TRUNCATED_FRAME
        if payload[0] not in (ICMPV4_ECHO, ICMPV4_ECHO_REPLY):
            return ERR_PACKET_DROP
        if CRC791().payload_sum16(payload) != 0:       # no pseudo-header
            return ERR_BAD_CRC
    return 0


def _ipv6_verdict(ip6: bytes, flags: int = 0, filt: StackFilter | None = None) -> int:
    """demux6 up to its checksum checks (internet/stack-ip6.go:86-138)."""
    if len(ip6) < 40:                                  # ipv6.NewFrame (ipv6/frame.go:13-18)
        return ERR_TRUNCATED_FRAME
    if filt is not None and filt.ip6 != bytes(16) and ip6[24:40] != filt.ip6:   # stack-ip6.go:93-98
        if not filt.ip6_accept_multicast or ip6[24] != 0xFF:                    # internal/ip.go:30-35
            return ERR_PACKET_DROP
    pl = _be16(ip6, 4)
    if pl + 40 > len(ip6):                             # ValidateSize (ipv6/frame.go:123-128)
        return ERR_INVALID_LENGTH_FIELD
    proto = ip6[6]
    if filt is not None and proto not in filt.ip6_protocols:
        return ERR_PACKET_DROP                         # nodeByProto nil (stack-ip6.go:107-111)
    payload = ip6[40:40 + pl]                          # Frame.Payload (ipv6/frame.go:34-37)
    if proto == IPPROTO_TCP:
        if ipv6_pseudo(ip6).payload_sum16(payload) != 0:
            return ERR_BAD_CRC
    elif proto == IPPROTO_UDP:
        if len(payload) < 8:
            return ERR_TRUNCATED_FRAME
        ul = _be16(payload, 4)
        if ul < 8:
            return ERR_INVALID_LENGTH_FIELD
        if ul > len(payload):
            return ERR_TRUNCATED_FRAME
        # quirk kept: the IPv6 UDP sum covers the whole IPv6 payload, not the UDP length
        if ipv6_pseudo(ip6).payload_sum16(payload) != 0:
            return ERR_BAD_CRC
    elif proto == IPPROTO_ICMPV6 and flags & VERIFY_ICMP:
        # the ICMPv6 client gets ip6[:40 + pl] at offset 40 (stack-ip6.go:140-141);
        # its Demux (ipv6/icmpv6/client.go:100-115) checks the size, then the sum
        # with the pseudo-header src, dst, AddUint32(len), AddUint32(58) — the
        # same words as CRCWritePseudo here, pl being the message length.  The
        # type dispatch (echo / NDP, else ErrPacketDrop) comes after the sum.
        if len(payload) < 8:                           # icmpv6.NewFrame (icmpv6.go:63-68)
            return ERR_TRUNCATED_FRAME
        if ipv6_pseudo(ip6).payload_sum16(payload) != 0:
            return ERR_BAD_CRC
    return 0


def ingress_verdict(frame: bytes, flags: int = 0, filt: StackFilter | None = None) -> int:
    """Checksum-stage verdict of lneto's receive path for one Ethernet frame
    (FCS stripped): StackEthernet.Demux (internet/stack-ethernet.go:139-165)
    size checks, then demux4 / demux6 by EtherType.  0 = every check passed or
    none applies (other EtherTypes); else the errGeneric code returned.
    filt: the stack's destination and handler configuration (StackFilter), whose
    ErrPacketDrop checks take the reference's places among the others; None =
    accept-all.  flags: VERIFY_EVIL_BIT, VERIFY_ICMP (ICMP messages also take
    the ICMP clients' checks)."""
    if len(frame) < 14:                                # ethernet.NewFrame (ethernet/frame.go:13-18)
        return ERR_TRUNCATED_FRAME
    et = _be16(frame, 12)
    if filt is not None:                               # stack-ethernet.go:146-152, before ValidateSize
        dst = frame[0:6]
        if dst != b"\xff" * 6 and dst != filt.mac:    # ethernet Frame.IsBroadcast (ethernet/frame.go:57-60)
            if not filt.eth_accept_multicast or dst[0] & 1 == 0:
                return ERR_PACKET_DROP
    if et <= 1500 and len(frame) < et:                 # ValidateSize (ethernet/frame.go:119-127)
        return ERR_INVALID_LENGTH_FIELD
    if et == ETHERTYPE_VLAN and len(frame) < 18:
        return ERR_TRUNCATED_FRAME
    if filt is not None and et not in filt.ethertypes:
        return ERR_PACKET_DROP                         # demuxByProto: no handler (stack-ethernet.go:158-161)
    if et == ETHERTYPE_IPV4:
        return _ipv4_verdict(frame[14:], flags, filt)
    if et == ETHERTYPE_IPV6:
        return _ipv6_verdict(frame[14:], flags, filt)
    return 0


# ------------------------------------- pcap's checksum re-verification (a17)
# PacketBreakdown.CaptureEthernet / CaptureIPv4 / CaptureIPv6
# (internet/pcap/capture.go:67-277) check the sums with semantics of their own:
# a bad IPv4 header sum is recorded and the protocol check still runs (:229-231),
# the TCP / UDP checks on IPv4 run only when tcp / udp.NewFrame accept the
# payload (:241-266), a UDP checksum of 0 is not checked (:259), ICMPv4 is
# always summed without pseudo-header (:267-273), IPv6 sums UDP and UDPLite over
# the UDP length (:184-198).  The validator (pc.vld, no flags) keeps the first
# error added (validation.go:59-66).
PCAP_IP_HDR_BAD = 1    # ErrBadCRC appended to the IPv4 frame's Errors (:229-231)
PCAP_PROTO_BAD = 2     # ipProtoErr == ErrBadCRC (attached to the transport frame, :297-299)
IPPROTO_UDPLITE = 136  # definitions.go:178


def _pcap_ipv4(ip: bytes) -> int:
    if len(ip) < 20:                                   # ipv4.NewFrame (:208-211)
        return ERR_TRUNCATED_FRAME << 2
    tl, ihl = _be16(ip, 2), ip[0] & 0xF
    errs = []                                          # ipv4 ValidateSize (ipv4/frame.go:214-227), :212-215
    if tl < 20:
        errs.append(ERR_INVALID_LENGTH_FIELD)
    if tl > len(ip):
        errs.append(ERR_TRUNCATED_FRAME)
    if ihl < 5 or ihl * 4 > tl:
        errs.append(ERR_INVALID_LENGTH_FIELD)
    if errs:
        return errs[0] << 2
    st = PCAP_IP_HDR_BAD if ipv4_header_sum16(ip) != 0 else 0
    proto, payload = ip[9], ip[ihl * 4:tl]
    if proto == IPPROTO_TCP:
        if len(payload) >= 20:                         # tcp.NewFrame (tcp/frame.go) accepts it
            doff = (payload[12] >> 4) * 4              # tcp ValidateSize: the error ends the capture (:243-246)
            if doff < 20:
                return st | ERR_INVALID_LENGTH_FIELD << 2
            if doff > len(payload):
                return st | ERR_TRUNCATED_FRAME << 2
            if ipv4_tcp_pseudo(ip).payload_sum16(payload) != 0:
                st |= PCAP_PROTO_BAD
    elif proto == IPPROTO_UDP:
        if len(payload) >= 8:                          # udp.NewFrame accepts it
            ul = _be16(payload, 4)                     # udp ValidateSize (:255-258)
            if ul < 8:
                return st | ERR_INVALID_LENGTH_FIELD << 2
            if ul > len(payload):
                return st | ERR_TRUNCATED_FRAME << 2
            if _be16(payload, 6) != 0 and ipv4_udp_pseudo(ip, ul).payload_sum16(payload[:ul]) != 0:
                st |= PCAP_PROTO_BAD
    elif proto == IPPROTO_ICMP:
        if len(payload) >= 8 and CRC791().payload_sum16(payload) != 0:   # icmpv4.NewFrame, :267-273
            st |= PCAP_PROTO_BAD
    return st


def _pcap_ipv6(ip6: bytes) -> int:
    if len(ip6) < 40:                                  # ipv6.NewFrame (:164-167)
        return ERR_TRUNCATED_FRAME << 2
    pl = _be16(ip6, 4)
    if pl + 40 > len(ip6):                             # ValidateSize (:168-171)
        return ERR_INVALID_LENGTH_FIELD << 2
    proto, payload = ip6[6], ip6[40:40 + pl]
    if proto == IPPROTO_TCP:
        if ipv6_pseudo(ip6).payload_sum16(payload) != 0:
            return PCAP_PROTO_BAD
    elif proto in (IPPROTO_UDP, IPPROTO_UDPLITE):
        # a size error here is ipProtoErr (:185-194); CaptureUDP over the rest of
        # the packet then fails with the same code or records it on the UDP frame
        if len(payload) < 8:
            return ERR_TRUNCATED_FRAME << 2
        ul = _be16(payload, 4)
        if ul < 8:
            return ERR_INVALID_LENGTH_FIELD << 2
        if ul > len(payload):
            return ERR_TRUNCATED_FRAME << 2
        if ipv6_pseudo(ip6).payload_sum16(payload[:ul]) != 0:   # :195-198, the UDP length
            return PCAP_PROTO_BAD
    return 0


def pcap_checksums(frame: bytes) -> int:
    """What pcap's PacketBreakdown.CaptureEthernet records about one Ethernet
    frame's checksums (internet/pcap/capture.go:67-277), as a status byte:
    bit 0 PCAP_IP_HDR_BAD, bit 1 PCAP_PROTO_BAD, bits 2-7 the errGeneric code of
    a size error met on the way to (or, for IPv6 UDP / UDPLite, in place of) the
    transport check, else 0.  Frames that are 802.3 length frames, VLAN-tagged or
    of another EtherType have no checksum stage in pcap: 0 unless their Ethernet
    size check fails."""
    if len(frame) < 14:                                # ethernet.NewFrame (:74-77)
        return ERR_TRUNCATED_FRAME << 2
    et = _be16(frame, 12)
    if et <= 1500 and len(frame) < et:                 # ValidateSize (ethernet/frame.go:119-127), :78-81
        return ERR_INVALID_LENGTH_FIELD << 2
    if et == ETHERTYPE_VLAN and len(frame) < 18:
        return ERR_TRUNCATED_FRAME << 2
    if et == ETHERTYPE_IPV4:                           # :98-104 (size / VLAN frames returned at :88-97)
        return _pcap_ipv4(frame[14:])
    if et == ETHERTYPE_IPV6:
        return _pcap_ipv6(frame[14:])
    return 0


# ------------------------------------------------- TX checksum generate (a16)


def _put16(b: bytearray, i: int, v: int) -> None:
    b[i:i + 2] = struct.pack(">H", v & 0xFFFF)


def tx_checksum(frame: bytes) -> tuple[bytes, int]:
    """The checksum-generate step of the transmit path for one Ethernet frame
    (Ethernet header + IP packet, before padding and FCS), as encapsulate4 /
    encapsulate6 and the ICMP clients run it once the child has written its
    n-byte payload:

    IPv4 (internet/stack-ip4.go:202-228): SetTotalLength(n + hl); SetCRC(0);
      SetCRC(CalculateHeaderCRC()) (first 20 bytes only, ipv4/frame.go:138-146);
      TCP: CRCWriteTCPPseudo, tcp SetCRC(0), SetCRC(PayloadSum16(payload));
      UDP: CRCWriteUDPPseudo(n), SetLength(n), SetCRC(0),
           SetCRC(NeverZeroSum(PayloadSum16(payload))) (crc.go:65-71);
      ICMP (ipv4/icmpv4/client.go:210-214): SetCRC(0), SetCRC(CRC791{}.PayloadSum16(msg)).
    IPv6 (internet/stack-ip6.go:167-181): SetPayloadLength(n); TCP / UDP as
      above with CRCWritePseudo (ipv6/frame.go:104-108); ICMPv6
      (ipv6/icmpv6/client.go:135-148): SetCRC(0), WriteEven(src, dst),
      AddUint32(n), AddUint32(58), PayloadSum16(msg).
    The header length is the frame's own IHL (encapsulate4 writes 5).
    Returns (new frame, status): 0 when written (other EtherTypes / protocols
    are left as they are), else the frame unchanged with ErrTruncatedFrame (18)
    when it is too short for a header the step writes (ipv4.NewFrame, tcp /
    udp / icmp NewFrame: 20, 20, 8, 8 bytes; the reference would panic on the
    transport ones, whose error it discards) or ErrInvalidLengthField (15) for
    IHL < 5 or a length that does not fit 16 bits."""
    f = bytearray(frame)
    if len(f) < 14:
        return bytes(frame), ERR_TRUNCATED_FRAME
    et = _be16(f, 12)
    if et == ETHERTYPE_IPV4:
        if len(f) < 34:
            return bytes(frame), ERR_TRUNCATED_FRAME
        hl = (f[14] & 0xF) * 4
        if hl < 20:
            return bytes(frame), ERR_INVALID_LENGTH_FIELD
        if 14 + hl > len(f):
            return bytes(frame), ERR_TRUNCATED_FRAME
        tl = len(f) - 14
        if tl > 0xFFFF:
            return bytes(frame), ERR_INVALID_LENGTH_FIELD
        n, proto, la = tl - hl, f[23], 14 + hl
        need = {IPPROTO_TCP: 20, IPPROTO_UDP: 8, IPPROTO_ICMP: 8}.get(proto, 0)
        if n < need:
            return bytes(frame), ERR_TRUNCATED_FRAME
        _put16(f, 16, tl)
        _put16(f, 24, 0)
        _put16(f, 24, ipv4_header_sum16(bytes(f[14:34])))
        ip = bytes(f[14:])
        if proto == IPPROTO_TCP:
            _put16(f, la + 16, 0)
            _put16(f, la + 16, ipv4_tcp_pseudo(ip).payload_sum16(bytes(f[la:])))
        elif proto == IPPROTO_UDP:
            c = ipv4_udp_pseudo(ip, n)
            _put16(f, la + 4, n)
            _put16(f, la + 6, 0)
            _put16(f, la + 6, never_zero_sum(c.payload_sum16(bytes(f[la:]))))
        elif proto == IPPROTO_ICMP:
            _put16(f, la + 2, 0)
            _put16(f, la + 2, CRC791().payload_sum16(bytes(f[la:])))
        return bytes(f), 0
    if et == ETHERTYPE_IPV6:
        if len(f) < 54:
            return bytes(frame), ERR_TRUNCATED_FRAME
        n, proto = len(f) - 54, f[20]
        if n > 0xFFFF:
            return bytes(frame), ERR_INVALID_LENGTH_FIELD
        need = {IPPROTO_TCP: 20, IPPROTO_UDP: 8, IPPROTO_ICMPV6: 8}.get(proto, 0)
        if n < need:
            return bytes(frame), ERR_TRUNCATED_FRAME
        _put16(f, 18, n)
        if proto in (IPPROTO_TCP, IPPROTO_UDP, IPPROTO_ICMPV6):
            c = ipv6_pseudo(bytes(f[14:54]))
            at = {IPPROTO_TCP: 16, IPPROTO_UDP: 6, IPPROTO_ICMPV6: 2}[proto]
            if proto == IPPROTO_UDP:
                _put16(f, 58, n)
            _put16(f, 54 + at, 0)
            s = c.payload_sum16(bytes(f[54:]))
            _put16(f, 54 + at, never_zero_sum(s) if proto == IPPROTO_UDP else s)
        return bytes(f), 0
    return bytes(frame), 0


def fix_ip_tcp_crcs(frame: bytes) -> tuple[bytes, bool]:
    """fixIPTCPCRCs of lneto's stack fuzz test (x/xnet/xnet_fuzz_test.go:150-185),
    which regenerates the checksums of a fuzzed frame before the stack sees it:
    for an IPv4 EtherType with version 4, IHL >= 5, IHL*4 <= total length <=
    len(frame), the header CRC over the first 20 bytes (ipv4/frame.go:144-146);
    then, for TCP with a >= 20-byte IP payload (ipv4 Frame.Payload, frame.go:188-192:
    bytes [IHL*4, total length) of the Ethernet payload; tcp.NewFrame), the TCP
    CRC = CRCWriteTCPPseudo + PayloadSum16 of that payload with its CRC field
    zeroed.  Returns (the frame as the harness leaves it, fixable).  A total
    length past len(frame) - 14 makes the Go slice run past the frame into the
    harness's buffer: such a frame is returned unchanged with None (its result
    depends on bytes outside it)."""
    f = bytearray(frame)
    if len(f) < 14 or _be16(f, 12) != ETHERTYPE_IPV4 or len(f) - 14 < 20:  # ethernet / ipv4 NewFrame
        return bytes(frame), False
    v, ihl, tl = f[14] >> 4, f[14] & 0xF, _be16(f, 16)
    if v != 4 or ihl < 5 or tl < ihl * 4 or tl > len(f):
        return bytes(frame), False
    if 14 + tl > len(f):
        return bytes(frame), None
    _put16(f, 24, 0)
    _put16(f, 24, ipv4_header_sum16(bytes(f[14:34])))
    if f[23] != IPPROTO_TCP:
        return bytes(f), False
    la = 14 + ihl * 4
    payload = f[la:14 + tl]
    if len(payload) < 20:                              # tcp.NewFrame (tcp/frame.go:19-24)
        return bytes(f), False
    _put16(f, la + 16, 0)
    _put16(f, la + 16, ipv4_tcp_pseudo(bytes(f[14:])).payload_sum16(bytes(f[la:14 + tl])))
    return bytes(f), True


# ------------------------------------------------------------ TX FCS append
ERR_SHORT_BUFFER = 6


def fcs_append(frame: bytes, capacity: int) -> tuple[bytes, int]:
    """Tail of StackEthernet.Encapsulate with the CRC32Update hook set
    (internet/stack-ethernet.go:200-214): zero-pad to 60 bytes, append
    LE32(crc32.Update(0, IEEETable, frame)).  A frame that would outgrow
    `capacity` is returned unchanged with ErrShortBuffer (the per-frame form of
    the destination-size check at internet/stack-ethernet.go:170-179)."""
    padded = frame + bytes(max(0, 60 - len(frame)))
    if len(padded) + 4 > capacity:
        return frame, ERR_SHORT_BUFFER
    return padded + struct.pack("<I", crc32_update(0, padded)), 0


# ----------------------------------------------------------------- C oracle
_lib = None


def lib():
    """ctypes handle of oracle/liboracle.so (built by `make -C oracle`)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise FileNotFoundError(f"{LIB_PATH} missing: run `make -C oracle`")
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.oracle_crc32.restype = ctypes.c_uint32
        L.oracle_crc32.argtypes = [u8p, ctypes.c_size_t]
        L.oracle_crc32_update.restype = ctypes.c_uint32
        L.oracle_crc32_update.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.oracle_crc32_update_simple.restype = ctypes.c_uint32
        L.oracle_crc32_update_simple.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.oracle_crc32_search.restype = ctypes.c_int64
        L.oracle_crc32_search.argtypes = [u8p, ctypes.c_size_t, ctypes.c_int64]
        L.oracle_payload_sum16.restype = ctypes.c_uint16
        L.oracle_payload_sum16.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.oracle_crc32_frames.restype = ctypes.c_int
        L.oracle_crc32_frames.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                          ctypes.c_void_p, ctypes.c_int]
        L.oracle_crc32_frames_amd64.restype = ctypes.c_int
        L.oracle_crc32_frames_amd64.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint64,
                                                ctypes.c_void_p, ctypes.c_int]
        L.oracle_crc32_update_amd64.restype = ctypes.c_uint32
        L.oracle_crc32_update_amd64.argtypes = [ctypes.c_uint32, u8p, ctypes.c_size_t]
        L.oracle_has_clmul.restype = ctypes.c_int
        L.oracle_has_clmul.argtypes = []
        L.oracle_sum16_segments.restype = None
        L.oracle_sum16_segments.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                            ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        _lib = L
    return _lib


def _u8p(b: bytes):
    buf = (ctypes.c_uint8 * max(len(b), 1)).from_buffer_copy(bytes(b) if len(b) else b"\0")
    return buf


def c_crc32(p: bytes) -> int:
    return lib().oracle_crc32(_u8p(p), len(p))


def c_crc32_simple(p: bytes, crc: int = 0) -> int:
    return lib().oracle_crc32_update_simple(crc, _u8p(p), len(p))


def c_crc32_search(p: bytes, min_off: int) -> int:
    return lib().oracle_crc32_search(_u8p(p), len(p), min_off)


def c_payload_sum16(seed: int, p: bytes) -> int:
    return lib().oracle_payload_sum16(seed, _u8p(p), len(p))


def crc32_frames(data: np.ndarray, off: np.ndarray, threads: int = 1, amd64: bool = False) -> np.ndarray:
    """CRC32 of every frame data[off[i]:off[i+1]] (C oracle, `threads` threads).
    amd64: Go's amd64 fast path (PCLMULQDQ folding + slicing-by-8 tail), the CPU
    baseline's form; the table form otherwise."""
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    n = len(off) - 1
    out = np.zeros(max(n, 1), dtype=np.uint32)
    fn = lib().oracle_crc32_frames_amd64 if amd64 else lib().oracle_crc32_frames
    fn(data.ctypes.data, off.ctypes.data, n, out.ctypes.data, threads)
    return out[:n]


def has_clmul() -> bool:
    return bool(lib().oracle_has_clmul())


def c_crc32_update_amd64(crc: int, p: bytes) -> int:
    return lib().oracle_crc32_update_amd64(crc, _u8p(p), len(p))


def sum16_segments(data: np.ndarray, off: np.ndarray, length: np.ndarray,
                   seed: np.ndarray | None) -> np.ndarray:
    data = np.ascontiguousarray(data, dtype=np.uint8)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    length = np.ascontiguousarray(length, dtype=np.uint32)
    n = len(off)
    out = np.zeros(max(n, 1), dtype=np.uint16)
    sp = None
    if seed is not None:
        seed = np.ascontiguousarray(seed, dtype=np.uint32)
        sp = seed.ctypes.data
    lib().oracle_sum16_segments(data.ctypes.data, off.ctypes.data, length.ctypes.data, sp, n,
                                out.ctypes.data)
    return out[:n]
