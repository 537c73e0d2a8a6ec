"""Synthetic Ethernet/IPv4/IPv6/TCP/UDP frames with valid or broken checksums,
shaped like lneto's own test generators (internal/ltesto/ltesto.go:99-135,209-228:
Ethernet + IPv4 (IHL 5) + TCP/UDP with the checksums filled in), widened with IP
options, IPv6, other protocols and the malformed cases demux4 / demux6 reject.

Checksum fields are filled with the oracle restatement of crc.go / ipv4/frame.go /
ipv6/frame.go (tests/test_oracle.py pins it on lneto_test.go:119-160)."""
from __future__ import annotations

import struct

import numpy as np

from oracle import oracle as O


def ether(et: int, payload: bytes) -> bytes:
    return bytes.fromhex("c0ffee00dead") + bytes.fromhex("4e8b3af9fb6b") + struct.pack(">H", et) + payload


IP4_DST = bytes([192, 168, 10, 2])
IP6_DST = bytes(range(0x30, 0x40))


def ipv4(proto: int, l4: bytes, opts: bytes = b"", flags: int = 0x4000, fix_l4: bool = True,
         dst: bytes = IP4_DST) -> bytes:
    ihl = 5 + len(opts) // 4
    tl = ihl * 4 + len(l4)
    hdr = bytearray(struct.pack(">BBHHHBBH4s4s", 0x40 | ihl, 0, tl, 0x1234, flags, 64, proto, 0,
                                bytes([192, 168, 10, 1]), dst)) + opts
    hdr[10:12] = struct.pack(">H", O.ipv4_header_sum16(bytes(hdr)))  # covers 20 bytes only
    l4 = bytearray(l4)
    if fix_l4 and proto == O.IPPROTO_TCP and len(l4) >= 18:
        l4[16:18] = b"\0\0"
        l4[16:18] = struct.pack(">H", O.ipv4_tcp_pseudo(bytes(hdr)).payload_sum16(bytes(l4)))
    if fix_l4 and proto == O.IPPROTO_ICMP and len(l4) >= 8:  # no pseudo-header (ltesto.go:224-227)
        l4[2:4] = b"\0\0"
        l4[2:4] = struct.pack(">H", O.CRC791().payload_sum16(bytes(l4)))
    if fix_l4 and proto == O.IPPROTO_UDP and len(l4) >= 8:
        ul = struct.unpack(">H", l4[4:6])[0]
        l4[6:8] = b"\0\0"
        if ul <= len(l4):
            l4[6:8] = struct.pack(">H", O.ipv4_udp_pseudo(bytes(hdr), ul).payload_sum16(bytes(l4[:ul])))
    return bytes(hdr) + bytes(l4)


def ipv6(proto: int, l4: bytes, fix_l4: bool = True, dst: bytes = IP6_DST) -> bytes:
    hdr = bytearray(struct.pack(">IHBB", 0x60000000, len(l4), proto, 64)) + bytes(range(0x20, 0x30)) + dst
    l4 = bytearray(l4)
    if fix_l4 and proto == O.IPPROTO_TCP and len(l4) >= 18:
        l4[16:18] = b"\0\0"
        l4[16:18] = struct.pack(">H", O.ipv6_pseudo(bytes(hdr)).payload_sum16(bytes(l4)))
    if fix_l4 and proto == O.IPPROTO_ICMPV6 and len(l4) >= 8:  # ipv6/icmpv6/client.go:141-148
        l4[2:4] = b"\0\0"
        l4[2:4] = struct.pack(">H", O.ipv6_pseudo(bytes(hdr)).payload_sum16(bytes(l4)))
    if fix_l4 and proto == O.IPPROTO_UDP and len(l4) >= 8:
        l4[6:8] = b"\0\0"  # the stack sums the whole payload (stack-ip6.go:133-134)
        l4[6:8] = struct.pack(">H", O.ipv6_pseudo(bytes(hdr)).payload_sum16(bytes(l4)))
    return bytes(hdr) + bytes(l4)


def tcp(payload: bytes) -> bytes:
    return struct.pack(">HHIIBBHHH", 0xE70A, 80, 0x4060D5CC, 0, 0x50, 0x18, 0xFAF0, 0, 0) + payload


def udp(payload: bytes, length: int | None = None) -> bytes:
    ul = 8 + len(payload) if length is None else length
    return struct.pack(">HHHH", 5353, 53, ul, 0) + payload


def icmp(type_: int, payload: bytes, ident: int = 0x1234, seq: int = 1) -> bytes:
    """An ICMPv4 / ICMPv6 message with an echo-shaped header (type, code 0,
    checksum, identifier, sequence number); ipv4() / ipv6() fill the checksum."""
    return struct.pack(">BBHHH", type_, 0, 0, ident, seq) + payload


def ltesto_icmp_echo(payload: bytes, ident: int, seq: int) -> bytes:
    """ltesto.PacketGen.AppendIPv4ICMPEcho (internal/ltesto/ltesto.go:175-231)
    with the addresses of TestStackAsync_ICMPEchoChecksum
    (x/xnet/xnet_test.go:1015-1045): IHL 5, ID 0, flags 0, TTL 64, protocol
    ICMP, header CRC; echo request (type 8, code 0) whose checksum covers the
    whole ICMP message."""
    tl = 20 + 8 + len(payload)
    hdr = bytearray(struct.pack(">BBHHHBBH4s4s", 0x45, 0, tl, 0, 0, 64, O.IPPROTO_ICMP, 0,
                                bytes([192, 168, 1, 1]), bytes([192, 168, 1, 99])))
    hdr[10:12] = struct.pack(">H", O.ipv4_header_sum16(bytes(hdr)))
    msg = bytearray(struct.pack(">BBHHH", 8, 0, 0, ident, seq) + payload)
    msg[2:4] = struct.pack(">H", O.CRC791().payload_sum16(bytes(msg)))
    return bytes([0xAA, 0xBB, 0xCC, 0xDD, 0xEE, 0xFF, 0x00, 0x11, 0x22, 0x33, 0x44, 0x55, 0x08, 0x00]) \
        + bytes(hdr) + bytes(msg)


def icmp_frames(seed: int = 3, count: int = 1200) -> list[bytes]:
    """ICMPv4 / ICMPv6 frames for the ICMP clients' checks (LNX_VERIFY_ICMP):
    echo and echo reply, other types (ICMPv4 drops them before the sum), one
    flipped byte, messages under 8 bytes, trailing bytes past tl / pl + 40
    (ignored), IPv4 options, and a broken IPv4 header in front of a non-echo
    type (the header sum comes first)."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        pay = rng.integers(0, 256, size=int(rng.integers(0, 1400)), dtype=np.uint8).tobytes()
        kind = i % 12
        if kind in (0, 1):
            f = ether(0x0800, ipv4(1, icmp(8 if kind == 0 else 0, pay)))
        elif kind == 2:
            f = ether(0x0800, ipv4(1, icmp(int(rng.choice([3, 5, 11, 13, 14, 42, 255])), pay)))
        elif kind == 3:
            b = bytearray(ether(0x0800, ipv4(1, icmp(8, pay))))
            b[int(rng.integers(34, len(b)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(b)
        elif kind == 4:
            f = ether(0x0800, ipv4(1, rng.integers(0, 256, size=int(rng.integers(0, 8)), dtype=np.uint8).tobytes()))
        elif kind == 5:
            f = ether(0x0800, ipv4(1, icmp(0, pay))) + bytes.fromhex("deadbeef")
        elif kind == 6:
            f = ether(0x86DD, ipv6(58, icmp(int(rng.choice([1, 128, 129, 135, 136, 200])), pay)))
        elif kind == 7:
            b = bytearray(ether(0x86DD, ipv6(58, icmp(128, pay))))
            b[int(rng.integers(54, len(b)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(b)
        elif kind == 8:
            f = ether(0x86DD, ipv6(58, rng.integers(0, 256, size=int(rng.integers(0, 8)), dtype=np.uint8).tobytes()))
        elif kind == 9:
            f = ether(0x86DD, ipv6(58, icmp(129, pay))) + rng.integers(1, 256, size=20, dtype=np.uint8).tobytes()
        elif kind == 10:
            b = bytearray(ether(0x0800, ipv4(1, icmp(3, pay))))
            b[22] ^= 0x01  # TTL
            f = bytes(b)
        else:
            f = ether(0x0800, ipv4(1, icmp(8, pay), opts=bytes(4 * int(rng.integers(1, 11)))))
        out.append(f)
    return out


def short_tcp6(rng) -> bytes:
    """0..7 payload bytes under IPv6 next-header TCP; demux6 does no size check
    for TCP (internet/stack-ip6.go:116-121), so the verdict is the sum alone.
    Half of the >= 2-byte ones carry their own checksum in the first word."""
    raw = bytearray(rng.integers(0, 256, size=int(rng.integers(0, 8)), dtype=np.uint8).tobytes())
    if len(raw) >= 2 and rng.integers(0, 2):
        hdr = struct.pack(">IHBB", 0x60000000, len(raw), O.IPPROTO_TCP, 64) + bytes(range(0x20, 0x40))
        raw[0:2] = b"\0\0"
        raw[0:2] = struct.pack(">H", O.ipv6_pseudo(hdr).payload_sum16(bytes(raw)))
    return bytes(raw)


def trailing_frames(seed: int = 7, count: int = 600) -> list[bytes]:
    """Frames whose transport data ends before the frame does, followed by
    non-zero bytes the receive path must ignore: IPv4 TCP / UDP with bytes past
    tl (internet/stack-ip4.go:100-107 slices the frame to tl), IPv4 UDP whose
    UDP length is below the IP payload (the sum covers ufrm.RawData()[:Length()],
    stack-ip4.go:161-163), and IPv6 with bytes past pl + 40 (ipv6 payload is
    sliced by PayloadLength, stack-ip6.go:86-138).  Transport payloads of
    150-1200 B so the ignored bytes land in the middle of a row's batch;
    a third of the frames carry one flipped byte inside the covered range."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(count):
        n = int(rng.integers(150, 1200))
        pay = rng.integers(0, 256, size=n, dtype=np.uint8).tobytes()
        tail = (rng.integers(1, 256, size=int(rng.integers(16, 300)), dtype=np.uint8)).tobytes()
        kind = i % 5
        if kind == 0:
            f = ether(0x0800, ipv4(6, tcp(pay))) + tail
        elif kind == 1:
            f = ether(0x0800, ipv4(17, udp(pay))) + tail
        elif kind == 2:  # UDP length < IP payload: the rest of the IP payload is outside the sum
            ul = 8 + int(rng.integers(0, n))
            f = ether(0x0800, ipv4(17, udp(pay, length=ul)))
        elif kind == 3:
            f = ether(0x86DD, ipv6(6, tcp(pay))) + tail
        else:
            f = ether(0x86DD, ipv6(17, udp(pay))) + tail
        if i % 3 == 0:
            b = bytearray(f)
            end = 14 + (struct.unpack(">H", b[16:18])[0] if kind < 3 else 40 + struct.unpack(">H", b[18:20])[0])
            if kind == 2:
                end = 14 + 20 + struct.unpack(">H", b[38:40])[0]
            b[int(rng.integers(min(60, end - 1), end))] ^= 0x04
            f = bytes(b)
        out.append(f)
    return out


def frames(seed: int = 1, count: int = 3000) -> list[bytes]:
    """A mixed batch: valid frames of every kind plus every malformation the
    receive path distinguishes, with random payload sizes (odd ones too)."""
    rng = np.random.default_rng(seed)

    def pay(lo=0, hi=1400):
        return rng.integers(0, 256, size=int(rng.integers(lo, hi)), dtype=np.uint8).tobytes()

    out = []
    for i in range(count):
        kind = i % 24
        if kind == 0:
            f = ether(0x0800, ipv4(6, tcp(pay())))
        elif kind == 1:
            f = ether(0x0800, ipv4(17, udp(pay())))
        elif kind == 2:  # IP options: the header sum still covers 20 bytes only (ipv4/frame.go:144-146)
            f = ether(0x0800, ipv4(6, tcp(pay()), opts=bytes(4 * int(rng.integers(1, 11)))))
        elif kind == 3 and (i // 24) % 2:  # IPv6 TCP shorter than a TCP header: demux6 sums it anyway
            f = ether(0x86DD, ipv6(6, short_tcp6(rng)))
        elif kind == 3:
            f = ether(0x86DD, ipv6(6, tcp(pay())))
        elif kind == 4:
            f = ether(0x86DD, ipv6(17, udp(pay())))
        elif kind == 5:  # corrupted payload byte
            b = bytearray(ether(0x0800, ipv4(int(rng.choice([6, 17])), tcp(pay(1)))))
            b[int(rng.integers(34, len(b)))] ^= 1 << int(rng.integers(0, 8))
            f = bytes(b)
        elif kind == 6:  # corrupted IPv4 header byte (not the length/version fields)
            b = bytearray(ether(0x0800, ipv4(6, tcp(pay()))))
            b[int(rng.choice([15, 18, 19, 22, 26, 27, 30, 33]))] ^= 0x10
            f = bytes(b)
        elif kind == 7:  # corrupted IPv6 payload
            b = bytearray(ether(0x86DD, ipv6(int(rng.choice([6, 17])), udp(pay(1)))))
            b[int(rng.integers(54, len(b)))] ^= 0x80
            f = bytes(b)
        elif kind == 8:  # UDP checksum 0 on IPv4: NOT special-cased by the stack (stack-ip4.go:152-167)
            b = bytearray(ether(0x0800, ipv4(17, udp(pay()))))
            b[40:42] = b"\0\0"
            f = bytes(b)
        elif kind == 9:  # other IP protocols: no transport sum
            f = ether(0x0800, ipv4(1, pay(8)))
        elif kind == 10:
            f = ether(0x86DD, ipv6(58, pay(8)))
        elif kind == 11:  # truncated total length: tl > buffer
            b = bytearray(ether(0x0800, ipv4(6, tcp(pay()))))
            b = b[: int(rng.integers(34, len(b)))]
            f = bytes(b)
        elif kind == 12:  # trailing bytes past tl (Ethernet padding): ignored
            f = ether(0x0800, ipv4(17, udp(pay(0, 10)))) + bytes(int(rng.integers(1, 30)))
        elif kind == 13:  # bad IHL / tl / version fields
            b = bytearray(ether(0x0800, ipv4(6, tcp(pay()))))
            m = int(rng.integers(0, 4))
            if m == 0:
                b[14] = 0x40 | int(rng.integers(0, 5))   # ihl < 5
            elif m == 1:
                b[16:18] = struct.pack(">H", int(rng.integers(0, 20)))  # tl < 20
            elif m == 2:
                b[14] = 0x60 | (b[14] & 15)              # version 6
            else:
                b[14] = 0x4F                             # ihl*4 = 60 > tl possibly
            f = bytes(b)
        elif kind == 14:  # evil bit (only rejected with VERIFY_EVIL_BIT)
            f = ether(0x0800, ipv4(6, tcp(pay()), flags=0x2000))
        elif kind == 15:  # UDP length field broken
            ul = int(rng.choice([0, 3, 7, 9000]))
            f = ether(0x0800, ipv4(17, udp(pay(), length=ul)))
        elif kind == 16:  # IPv6 payload length too large / UDP too short
            b = bytearray(ether(0x86DD, ipv6(17, udp(pay(0, 6)))))
            if rng.integers(0, 2):
                b[18:20] = struct.pack(">H", len(b))
            else:
                b = b[: 14 + 40 + int(rng.integers(0, 8))]
                b[18:20] = struct.pack(">H", len(b) - 54)
            f = bytes(b)
        elif kind == 17:  # short frames
            f = pay(0, 60)
        elif kind == 18:  # VLAN, size-type, ARP EtherTypes
            et = int(rng.choice([0x8100, 0x0806, 46, 1500, 0x88CC]))
            f = ether(et, pay(0, 100))
            if et == 0x8100 and rng.integers(0, 2):
                f = f[: int(rng.integers(14, 18))]
        elif kind == 19:  # IPv4 with a UDP payload shorter than the UDP header
            f = ether(0x0800, ipv4(17, pay(0, 8), fix_l4=False))
        elif kind == 20:  # random bytes behind IPv4 / IPv6 EtherTypes
            f = ether(int(rng.choice([0x0800, 0x86DD])), pay(0, 200))
        elif kind == 21:  # odd-length TCP segment (trailing byte weighted << 8)
            f = ether(0x0800, ipv4(6, tcp(pay(1, 50) + b"\x7f")))
        elif kind == 22:  # jumbo-ish
            f = ether(0x0800, ipv4(6, tcp(pay(3000, 8900))))
        else:  # minimum-size frame with Ethernet padding
            f = ether(0x0800, ipv4(17, udp(b"")))
            f = f + bytes(max(0, 60 - len(f)))
        out.append(f)
    return out


MAC_US = bytes.fromhex("c0ffee00dead")  # ether()'s destination: the stack's own MAC in filter_frames


def filter_frames(seed: int = 21, count: int = 2400) -> list[bytes]:
    """Frames for the stack filter (lnx_rx_filter / oracle.StackFilter): every
    destination class at each layer (the stack's MAC / broadcast / another
    unicast MAC / a multicast MAC; the stack's IPv4 address / another / 224/4 /
    255.255.255.255; the stack's IPv6 address / another / ff02::1), EtherTypes
    and IP protocols with and without a handler, crossed with broken sums and
    sizes, so a frame the stack would drop also carries an error that a later
    check would report (the precedence is the test)."""
    rng = np.random.default_rng(seed)
    macs = [MAC_US, b"\xff" * 6, bytes.fromhex("02aabbccddee"), bytes.fromhex("01005e000001")]
    ip4s = [IP4_DST, bytes([192, 168, 10, 77]), bytes([224, 0, 0, 251]), b"\xff" * 4]
    ip6s = [IP6_DST, bytes(range(0x50, 0x60)), bytes.fromhex("ff020000000000000000000000000001")]
    out = []
    for i in range(count):
        pay = rng.integers(0, 256, size=int(rng.integers(0, 600)), dtype=np.uint8).tobytes()
        fam = i % 5
        if fam in (0, 1):
            proto = int(rng.choice([6, 17, 1, 47]))
            l4 = tcp(pay) if proto == 6 else udp(pay) if proto == 17 else icmp(8, pay) if proto == 1 else pay
            f = ether(0x0800, ipv4(proto, l4, dst=ip4s[int(rng.integers(0, 4))]))
        elif fam in (2, 3):
            proto = int(rng.choice([6, 17, 58, 47]))
            l4 = tcp(pay) if proto == 6 else udp(pay) if proto == 17 else icmp(128, pay) if proto == 58 else pay
            f = ether(0x86DD, ipv6(proto, l4, dst=ip6s[int(rng.integers(0, 3))]))
        else:
            et = int(rng.choice([0x0806, 0x88CC, 0x8100, 46]))
            f = ether(et, pay + bytes(46))
        b = bytearray(f)
        b[0:6] = macs[int(rng.choice(4, p=[0.55, 0.15, 0.15, 0.15]))]
        r = rng.random()
        if r < 0.2 and len(b) > 34:          # a broken sum somewhere past the Ethernet header
            b[int(rng.integers(14, len(b)))] ^= 1 << int(rng.integers(0, 8))
        elif r < 0.27:                       # a size error
            b = b[: int(rng.integers(14, max(15, len(b) - 1)))]
        out.append(bytes(b))
    return out


def _udp6_pcap(proto: int, pay: bytes, extra: bytes = b"") -> bytes:
    """An IPv6 UDP / UDPLite packet whose checksum covers the UDP length only,
    as pcap sums it (internet/pcap/capture.go:184-198), followed by `extra`
    bytes inside the IPv6 payload but outside the UDP length."""
    l4 = bytearray(udp(pay)) + extra
    hdr = bytearray(struct.pack(">IHBB", 0x60000000, len(l4), proto, 64)) + bytes(range(0x20, 0x30)) + IP6_DST
    ul = 8 + len(pay)
    l4[6:8] = struct.pack(">H", O.ipv6_pseudo(bytes(hdr)).payload_sum16(bytes(l4[:ul])))
    return bytes(hdr) + bytes(l4)


def pcap_frames(seed: int = 31, count: int = 2400) -> list[bytes]:
    """Frames for pcap's checksum re-verification (oracle.pcap_checksums):
    the receive-path mix (frames()) plus what pcap treats differently — a bad
    IPv4 header sum in front of a good / bad transport sum, IPv4 UDP with a
    zero checksum, ICMPv4 of any type (good / flipped), IPv6 UDP and UDPLite
    summed over the UDP length with bytes after it, TCP data offsets below 5 or
    past the payload, IPv4 TCP payloads under 20 bytes and UDP under 8."""
    rng = np.random.default_rng(seed)

    def pay(lo=0, hi=1400):
        return rng.integers(0, 256, size=int(rng.integers(lo, hi)), dtype=np.uint8).tobytes()

    def flip(f: bytes, lo: int, hi: int | None = None) -> bytes:
        b = bytearray(f)
        b[int(rng.integers(lo, len(b) if hi is None else hi))] ^= 1 << int(rng.integers(0, 8))
        return bytes(b)

    out = []
    base = frames(seed=seed + 1, count=count // 2)
    for i in range(count - len(base)):
        kind = i % 12
        if kind == 0:    # bad header sum (TTL / ID byte), transport good
            f = flip(ether(0x0800, ipv4(int(rng.choice([1, 6, 17])), tcp(pay()))), 18, 24)
        elif kind == 1:  # bad header sum and bad transport sum
            f = flip(flip(ether(0x0800, ipv4(6, tcp(pay(1)))), 22, 23), 34)
        elif kind == 2:  # IPv4 UDP with checksum 0: not checked, whatever the payload
            b = bytearray(flip(ether(0x0800, ipv4(17, udp(pay(1)))), 42))
            b[40:42] = b"\0\0"
            f = bytes(b)
        elif kind == 3:  # ICMPv4 of any type, good or flipped
            f = ether(0x0800, ipv4(1, icmp(int(rng.integers(0, 256)), pay())))
            if rng.integers(0, 2):
                f = flip(f, 34)
        elif kind == 4:  # ICMPv4 under 8 bytes: icmpv4.NewFrame refuses it, no check
            f = ether(0x0800, ipv4(1, pay(0, 8), fix_l4=False))
        elif kind == 5:  # IPv6 UDP / UDPLite over the UDP length, bytes after it
            f = ether(0x86DD, _udp6_pcap(int(rng.choice([17, 136])), pay(), pay(0, 40)))
            if rng.integers(0, 2):
                f = flip(f, 54, 54 + 8 + ((f[58] << 8) | f[59]) - 8)
        elif kind == 6:  # IPv6 UDPLite / UDP size errors
            b = bytearray(ether(0x86DD, _udp6_pcap(int(rng.choice([17, 136])), pay(0, 30))))
            m = int(rng.integers(0, 3))
            if m == 0:
                b[58:60] = struct.pack(">H", int(rng.integers(0, 8)))        # ul < 8
            elif m == 1:
                b[58:60] = struct.pack(">H", len(b) - 54 + int(rng.integers(1, 100)))  # ul > pl
            else:
                b = b[:54 + int(rng.integers(0, 8))]                        # pl < 8
                b[18:20] = struct.pack(">H", len(b) - 54)
            f = bytes(b)
        elif kind == 7:  # TCP data offset < 5 or past the payload (the capture ends)
            b = bytearray(ether(0x0800, ipv4(6, tcp(pay(0, 40)))))
            b[46] = (int(rng.integers(0, 5)) if rng.integers(0, 2) else 15) << 4
            f = flip(bytes(b), 22, 23) if rng.integers(0, 2) else bytes(b)
        elif kind == 8:  # IPv4 TCP payload under 20 bytes: tcp.NewFrame refuses it, no check
            f = ether(0x0800, ipv4(6, pay(0, 20), fix_l4=False))
        elif kind == 9:  # IPv4 UDP length errors behind a bad header sum
            f = flip(ether(0x0800, ipv4(17, udp(pay(), length=int(rng.choice([0, 7, 4000]))))), 22, 23)
        elif kind == 10:  # IPv6 TCP, any length from 0 (no NewFrame check there)
            f = ether(0x86DD, ipv6(6, short_tcp6(rng) if rng.integers(0, 2) else tcp(pay())))
            if rng.integers(0, 3) == 0 and len(f) > 54:
                f = flip(f, 54)
        else:            # IPv6 UDP summed the receive path's way (whole payload): pcap's differs
            f = ether(0x86DD, ipv6(17, udp(pay())) + pay(1, 20))
            b = bytearray(f)
            b[18:20] = struct.pack(">H", len(b) - 54)  # the trailing bytes inside pl
            f = bytes(b)
        out.append(f)
    return base + out
