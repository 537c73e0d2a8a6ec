// host_path.cpp — per-frame host forms of the receive verdict and the
// transmit steps (round 5).
//
// netdev's Runner hands the stack ONE buffer per IngressPackets /
// EgressPackets call (lneto x/netdev/runner.go:358-359,432-433,469-470).  A
// GPU round trip costs tens of microseconds (pinned gather, H2D, launches,
// D2H, a sync: DESIGN.md §4 "per-call latency"), a host verdict of a 1500-byte
// frame about a microsecond, so the packet entries (rx_ring.hip) fold batches
// below the measured crossover here and never launch for them.  These are the
// product's own restatements of the reference (the oracle in oracle/ is the
// checker of both paths), and the same functions are exported per frame:
// lnx_ingress_verdict, lnx_pcap_checksums, lnx_tx_checksum, lnx_fcs_append
// (include/lneto_amd.h).
#include <cstdint>
#include <cstring>
#include "../../include/lneto_amd.h"
#include "rx_filter.hpp"

namespace lnx {

namespace {

constexpr uint8_t kErrPacketDrop = 2, kErrBadCRC = 3, kErrShortBuffer = 6, kErrInvalidField = 14,
                  kErrInvalidLengthField = 15, kErrTruncatedFrame = 18;  // lneto errors.go:6-28
constexpr uint32_t kVerifyEvilBit = LNX_VERIFY_EVIL_BIT, kVerifyIcmp = LNX_VERIFY_ICMP;

inline uint32_t be16(const uint8_t* p) { return (uint32_t)p[0] << 8 | p[1]; }
inline void put16(uint8_t* p, uint32_t v) { p[0] = (uint8_t)(v >> 8), p[1] = (uint8_t)v; }

// lneto.CRC791 (crc.go:13-59)
struct Crc791 {
  uint32_t sum = 0;
  void write_even(const uint8_t* p, size_t n) { sum = lnx_sum_write_even(sum, p, n); }
  void add16(uint32_t v) { sum += v & 0xFFFFu; }
  void add32(uint32_t v) { sum += v >> 16, sum += v & 0xFFFFu; }
  uint16_t payload_sum16(const uint8_t* p, size_t n) const { return lnx_sum16_payload(sum, p, n); }
};

bool proto_bit(const uint32_t (&m)[8], uint32_t p) { return (m[p >> 5] >> (p & 31u)) & 1u; }

// demux4 up to its checksum checks (internet/stack-ip4.go:100-164); ip = the
// IPv4 packet as the Ethernet payload (frame[14:]), n bytes
uint8_t ipv4_verdict(const uint8_t* ip, size_t n, uint32_t flags, const RxFilter& f) {
  if (n < 20) return kErrTruncatedFrame;  // ipv4.NewFrame (ipv4/frame.go:15-20)
  if (f.on && f.ip4 != 0 && le32_of(ip + 16) != f.ip4) {  // stack-ip4.go:108-119
    const bool mc = (ip[16] & 0xF0u) == 0xE0u;                                       // ipv4/definitions.go:17-19
    const bool bc = ip[16] == 0xFF && ip[17] == 0xFF && ip[18] == 0xFF && ip[19] == 0xFF;  // :34-36
    if (!(f.ip4_mc && mc) && !(f.ip4_bc && bc)) return kErrPacketDrop;
  }
  // ValidateExceptCRC (ipv4/frame.go:214-238): the first error added wins
  const uint32_t tl = be16(ip + 2), ihl = ip[0] & 15u, version = ip[0] >> 4;
  if (tl < 20) return kErrInvalidLengthField;
  if (tl > n) return kErrTruncatedFrame;
  if (ihl < 5 || ihl * 4 > tl) return kErrInvalidLengthField;
  if (version != 4) return kErrInvalidField;
  if ((flags & kVerifyEvilBit) && (be16(ip + 6) & (1u << 13))) return kErrPacketDrop;  // ipv4/definitions.go:68-87
  {
    Crc791 h;  // CalculateHeaderCRC: the first 20 bytes only (ipv4/frame.go:138-146)
    h.write_even(ip, 20);
    if (lnx_sum16(h.sum) != 0) return kErrBadCRC;
  }
  const uint32_t hl = ihl * 4, proto = ip[9];
  const uint8_t* pay = ip + hl;  // Frame.Payload (ipv4/frame.go:188-192)
  const uint32_t pn = tl - hl;
  if (f.on && !proto_bit(f.p4, proto)) return kErrPacketDrop;  // nodeByProto nil (stack-ip4.go:135-141)
  if (proto == 6) {
    Crc791 c;  // CRCWriteTCPPseudo (ipv4/frame.go:154-158)
    c.write_even(ip + 12, 8);
    c.add16(tl - hl);
    c.add16(proto);
    if (c.payload_sum16(pay, pn) != 0) return kErrBadCRC;
  } else if (proto == 17) {
    if (pn < 8) return kErrTruncatedFrame;  // udp.NewFrame (udp/frame.go:15-20)
    const uint32_t ul = be16(pay + 4);
    if (ul < 8) return kErrInvalidLengthField;  // udp ValidateSize (udp/frame.go:96-104)
    if (ul > pn) return kErrTruncatedFrame;
    Crc791 c;  // CRCWriteUDPPseudo(crc, ul) (ipv4/frame.go:166-170)
    c.write_even(ip + 12, 8);
    c.add16(ul);
    c.add16(proto);
    if (c.payload_sum16(pay, ul) != 0) return kErrBadCRC;
  } else if (proto == 1 && (flags & kVerifyIcmp)) {
    // the ICMPv4 client's Demux (ipv4/icmpv4/client.go:89-102)
    if (pn < 8) return kErrTruncatedFrame;  // icmpv4.NewFrame
    if (pay[0] != 0 && pay[0] != 8) return kErrPacketDrop;  // echo reply / echo only
    if (Crc791{}.payload_sum16(pay, pn) != 0) return kErrBadCRC;  // no pseudo-header
  }
  return 0;
}

// demux6 up to its checksum checks (internet/stack-ip6.go:86-138)
uint8_t ipv6_verdict(const uint8_t* ip, size_t n, uint32_t flags, const RxFilter& f) {
  if (n < 40) return kErrTruncatedFrame;  // ipv6.NewFrame (ipv6/frame.go:13-18)
  if (f.on && (f.ip6[0] | f.ip6[1] | f.ip6[2] | f.ip6[3]) != 0) {  // stack-ip6.go:93-98
    const bool mine = le32_of(ip + 24) == f.ip6[0] && le32_of(ip + 28) == f.ip6[1] && le32_of(ip + 32) == f.ip6[2] &&
                      le32_of(ip + 36) == f.ip6[3];
    if (!mine && !(f.ip6_mc && ip[24] == 0xFF)) return kErrPacketDrop;  // internal/ip.go:30-35
  }
  const uint32_t pl = be16(ip + 4);
  if (pl + 40 > n) return kErrInvalidLengthField;  // ValidateSize (ipv6/frame.go:123-128)
  const uint32_t proto = ip[6];
  if (f.on && !proto_bit(f.p6, proto)) return kErrPacketDrop;  // nodeByProto nil (stack-ip6.go:107-111)
  const uint8_t* pay = ip + 40;
  auto pseudo = [&] {  // CRCWritePseudo (ipv6/frame.go:104-108)
    Crc791 c;
    c.write_even(ip + 8, 32);
    c.add32(pl);
    c.add32(proto);
    return c;
  };
  if (proto == 6) {
    if (pseudo().payload_sum16(pay, pl) != 0) return kErrBadCRC;
  } else if (proto == 17) {
    if (pl < 8) return kErrTruncatedFrame;
    const uint32_t ul = be16(pay + 4);
    if (ul < 8) return kErrInvalidLengthField;
    if (ul > pl) return kErrTruncatedFrame;
    // the IPv6 UDP sum covers the whole payload, not the UDP length (stack-ip6.go:133-134)
    if (pseudo().payload_sum16(pay, pl) != 0) return kErrBadCRC;
  } else if (proto == 58 && (flags & kVerifyIcmp)) {
    // the ICMPv6 client's Demux (ipv6/icmpv6/client.go:100-115): size, then the pseudo-header sum
    if (pl < 8) return kErrTruncatedFrame;
    if (pseudo().payload_sum16(pay, pl) != 0) return kErrBadCRC;
  }
  return 0;
}

// pcap's CaptureIPv4 checksum findings (internet/pcap/capture.go:203-277):
// status bits as lnx_pcap_verify_batch
uint8_t pcap_ipv4(const uint8_t* ip, size_t n) {
  if (n < 20) return kErrTruncatedFrame << 2;  // ipv4.NewFrame
  const uint32_t tl = be16(ip + 2), ihl = ip[0] & 15u;  // ValidateSize (ipv4/frame.go:214-227), :212-215
  if (tl < 20) return kErrInvalidLengthField << 2;
  if (tl > n) return kErrTruncatedFrame << 2;
  if (ihl < 5 || ihl * 4 > tl) return kErrInvalidLengthField << 2;
  uint8_t st = 0;
  {
    Crc791 h;  // a bad header sum is recorded and the capture goes on (:229-231)
    h.write_even(ip, 20);
    if (lnx_sum16(h.sum) != 0) st |= LNX_PCAP_IP_HDR_BAD;
  }
  const uint32_t hl = ihl * 4, proto = ip[9], pn = tl - hl;
  const uint8_t* pay = ip + hl;
  if (proto == 6 && pn >= 20) {  // tcp.NewFrame accepts it; ValidateSize ends the capture (:241-251)
    const uint32_t doff = (uint32_t)(pay[12] >> 4) * 4;
    if (doff < 20) return st | kErrInvalidLengthField << 2;
    if (doff > pn) return st | kErrTruncatedFrame << 2;
    Crc791 c;
    c.write_even(ip + 12, 8);
    c.add16(pn);
    c.add16(proto);
    if (c.payload_sum16(pay, pn) != 0) st |= LNX_PCAP_PROTO_BAD;
  } else if (proto == 17 && pn >= 8) {  // udp.NewFrame accepts it (:252-266)
    const uint32_t ul = be16(pay + 4);
    if (ul < 8) return st | kErrInvalidLengthField << 2;
    if (ul > pn) return st | kErrTruncatedFrame << 2;
    if (be16(pay + 6) != 0) {  // a zero UDP checksum is not checked (:259)
      Crc791 c;
      c.write_even(ip + 12, 8);
      c.add16(ul);
      c.add16(proto);
      if (c.payload_sum16(pay, ul) != 0) st |= LNX_PCAP_PROTO_BAD;
    }
  } else if (proto == 1 && pn >= 8) {  // icmpv4.NewFrame; summed with no pseudo-header (:267-273)
    if (Crc791{}.payload_sum16(pay, pn) != 0) st |= LNX_PCAP_PROTO_BAD;
  }
  return st;
}

// pcap's CaptureIPv6 checksum findings (internet/pcap/capture.go:159-201)
uint8_t pcap_ipv6(const uint8_t* ip, size_t n) {
  if (n < 40) return kErrTruncatedFrame << 2;  // ipv6.NewFrame
  const uint32_t pl = be16(ip + 4), proto = ip[6];
  if (pl + 40 > n) return kErrInvalidLengthField << 2;  // ValidateSize
  Crc791 c;  // CRCWritePseudo (ipv6/frame.go:104-108)
  c.write_even(ip + 8, 32);
  c.add32(pl);
  c.add32(proto);
  const uint8_t* pay = ip + 40;
  if (proto == 6) {
    if (c.payload_sum16(pay, pl) != 0) return LNX_PCAP_PROTO_BAD;
  } else if (proto == 17 || proto == 136) {  // UDP and UDPLite (:184-198)
    if (pl < 8) return kErrTruncatedFrame << 2;
    const uint32_t ul = be16(pay + 4);
    if (ul < 8) return kErrInvalidLengthField << 2;
    if (ul > pl) return kErrTruncatedFrame << 2;
    if (c.payload_sum16(pay, ul) != 0) return LNX_PCAP_PROTO_BAD;  // over the UDP length
  }
  return 0;
}

}  // namespace

// The receive path's checksum-stage verdict of one Ethernet frame without its
// FCS: StackEthernet.Demux (internet/stack-ethernet.go:139-165), then demux4 /
// demux6 by EtherType; the same value as ingress_verify_kernel.
uint8_t host_verdict(const uint8_t* fr, size_t L, uint32_t flags, const RxFilter& f) {
  if (L < 14) return kErrTruncatedFrame;  // ethernet.NewFrame (ethernet/frame.go:13-18)
  const uint32_t et = be16(fr + 12);
  bool et_handler = true;
  if (f.on) {
    // before ValidateSize: neither broadcast nor for the MAC, unless multicast is accepted (stack-ethernet.go:146-152)
    const bool bcast = le32_of(fr) == 0xFFFFFFFFu && fr[4] == 0xFF && fr[5] == 0xFF;
    const bool mine = le32_of(fr) == f.mac_lo && (uint32_t)(fr[4] | fr[5] << 8) == f.mac_hi;
    if (!bcast && !mine && !(f.eth_mc && (fr[0] & 1u))) return kErrPacketDrop;
    et_handler = false;  // handlers.demuxByProto (stack-ethernet.go:158-161)
    for (uint32_t i = 0; i < f.n_et; ++i) et_handler = et_handler || f.et[i] == et;
  }
  if (et <= 1500 && L < et) return kErrInvalidLengthField;  // ValidateSize (ethernet/frame.go:119-127)
  if (et == 0x8100 && L < 18) return kErrTruncatedFrame;
  if (!et_handler) return kErrPacketDrop;
  if (et == 0x0800) return ipv4_verdict(fr + 14, L - 14, flags, f);
  if (et == 0x86DD) return ipv6_verdict(fr + 14, L - 14, flags, f);
  return 0;
}

// pcap's CaptureEthernet checksum findings (internet/pcap/capture.go:67-110):
// the same status as pcap_verify_kernel
uint8_t host_pcap(const uint8_t* fr, size_t L) {
  if (L < 14) return kErrTruncatedFrame << 2;  // ethernet.NewFrame
  const uint32_t et = be16(fr + 12);
  if (et <= 1500 && L < et) return kErrInvalidLengthField << 2;  // ValidateSize
  if (et == 0x8100 && L < 18) return kErrTruncatedFrame << 2;
  if (et == 0x0800) return pcap_ipv4(fr + 14, L - 14);  // size and VLAN frames end at :88-97
  if (et == 0x86DD) return pcap_ipv6(fr + 14, L - 14);
  return 0;
}

// The transmit checksum step for one frame (Ethernet header + IP packet, before
// padding and FCS), in place: the semantics of lnx_tx_checksum_batch
// (encapsulate4 / encapsulate6 / the ICMP clients, internet/stack-ip4.go:202-228,
// internet/stack-ip6.go:167-181, ipv4/icmpv4/client.go:210-214,
// ipv6/icmpv6/client.go:135-148).  Returns the status (0, 18 or 15).
uint8_t host_tx_checksum(uint8_t* f, size_t L) {
  if (L < 14) return kErrTruncatedFrame;
  const uint32_t et = be16(f + 12);
  if (et == 0x0800) {
    if (L < 34) return kErrTruncatedFrame;
    const uint32_t hl = (f[14] & 15u) * 4;
    if (hl < 20) return kErrInvalidLengthField;
    if (14 + hl > L) return kErrTruncatedFrame;
    const size_t tl = L - 14;
    if (tl > 0xFFFF) return kErrInvalidLengthField;
    const uint32_t n = (uint32_t)tl - hl, proto = f[23];
    const uint32_t need = proto == 6 ? 20u : (proto == 17 || proto == 1) ? 8u : 0u;
    if (n < need) return kErrTruncatedFrame;
    uint8_t* ip = f + 14;
    uint8_t* t = ip + hl;
    put16(ip + 2, (uint32_t)tl);  // SetTotalLength(n + hl)
    put16(ip + 10, 0);
    Crc791 h;
    h.write_even(ip, 20);  // CalculateHeaderCRC (ipv4/frame.go:138-146)
    put16(ip + 10, lnx_sum16(h.sum));
    if (proto == 6) {
      Crc791 c;  // CRCWriteTCPPseudo
      c.write_even(ip + 12, 8);
      c.add16(n);
      c.add16(proto);
      put16(t + 16, 0);
      put16(t + 16, c.payload_sum16(t, n));
    } else if (proto == 17) {
      Crc791 c;  // CRCWriteUDPPseudo(crc, n), SetLength(n)
      c.write_even(ip + 12, 8);
      c.add16(n);
      c.add16(proto);
      put16(t + 4, n);
      put16(t + 6, 0);
      put16(t + 6, lnx_never_zero_sum(c.payload_sum16(t, n)));  // crc.go:65-71
    } else if (proto == 1) {
      put16(t + 2, 0);
      put16(t + 2, Crc791{}.payload_sum16(t, n));
    }
    return 0;
  }
  if (et == 0x86DD) {
    if (L < 54) return kErrTruncatedFrame;
    const size_t n64 = L - 54;
    if (n64 > 0xFFFF) return kErrInvalidLengthField;
    const uint32_t n = (uint32_t)n64, proto = f[20];
    const uint32_t need = proto == 6 ? 20u : (proto == 17 || proto == 58) ? 8u : 0u;
    if (n < need) return kErrTruncatedFrame;
    uint8_t* ip = f + 14;
    uint8_t* t = f + 54;
    put16(ip + 4, n);  // SetPayloadLength(n)
    if (proto == 6 || proto == 17 || proto == 58) {
      Crc791 c;  // CRCWritePseudo (ipv6/frame.go:104-108)
      c.write_even(ip + 8, 32);
      c.add32(n);
      c.add32(proto);
      const uint32_t at = proto == 6 ? 16u : proto == 17 ? 6u : 2u;
      if (proto == 17) put16(t + 4, n);
      put16(t + at, 0);
      const uint16_t s = c.payload_sum16(t, n);
      put16(t + at, proto == 17 ? lnx_never_zero_sum(s) : s);
    }
    return 0;
  }
  return 0;
}

// The tail of StackEthernet.Encapsulate with the CRC32Update hook set
// (internet/stack-ethernet.go:200-214): zero-pad to 60 bytes, append the LE
// FCS, *len grows; ErrShortBuffer (6) with the frame untouched when it would
// outgrow `capacity`.
uint8_t host_fcs_append(uint8_t* f, uint32_t* len, uint32_t capacity) {
  const uint32_t n = *len, pad = n < 60 ? 60 - n : 0;
  if ((uint64_t)n + pad + 4 > capacity) return kErrShortBuffer;
  if (pad) std::memset(f + n, 0, pad);
  const uint32_t crc = lnx_crc32(f, n + pad);
  for (int i = 0; i < 4; ++i) f[n + pad + i] = (uint8_t)(crc >> (8 * i));
  *len = n + pad + 4;
  return 0;
}

// FCS check of a received frame carrying its LE FCS (the residue test)
uint8_t host_fcs_ok(const uint8_t* f, size_t L) {
  return L >= 4 && lnx_crc32(f, L) == LNX_CRC32_RESIDUE ? 1 : 0;
}

}  // namespace lnx

extern "C" {

int lnx_ingress_verdict(const uint8_t* frame, size_t len, uint32_t flags, const lnx_rx_filter* filter) {
  lnx::RxFilter f;
  if (!lnx::rx_filter_of(filter, &f)) return LNX_EINVAL;
  if (len > 0 && !frame) return LNX_EINVAL;
  return lnx::host_verdict(frame, len, flags & (LNX_VERIFY_EVIL_BIT | LNX_VERIFY_ICMP), f);
}

int lnx_pcap_checksums(const uint8_t* frame, size_t len) {
  if (len > 0 && !frame) return LNX_EINVAL;
  return lnx::host_pcap(frame, len);
}

int lnx_tx_checksum(uint8_t* frame, size_t len) {
  if (len > 0 && !frame) return LNX_EINVAL;
  return lnx::host_tx_checksum(frame, len);
}

int lnx_fcs_append(uint8_t* frame, uint32_t* len, uint32_t capacity) {
  if (!len || !frame) return LNX_EINVAL;
  return lnx::host_fcs_append(frame, len, capacity);
}

}  // extern "C"
