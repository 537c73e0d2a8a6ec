// lneto_amd.hpp — C++ host mirror of lneto's checksum API over the C-ABI.
//
// Same names, argument meaning and error behaviour as the Go reference, so a
// C++ caller (and the C++ tests) read like lneto's own code:
//
//   Go (reference)                                   C++ (this header)
//   ethernet.CRC32(data) uint32          crc.go:19   ethernet::CRC32(data)
//   ethernet.CRC32Search(data, min) int  crc.go:28   ethernet::CRC32Search(data, min)
//   crc32.Update(crc, IEEETable, p)      hook type   ethernet::CRC32Update (a CRC32UpdateFunc)
//   lneto.CRC791{...}                    crc.go:13   lneto::CRC791
//   lneto.NeverZeroSum                   crc.go:65   lneto::NeverZeroSum
//   lneto.ErrBadCRC                      errors.go:10 lneto::Err::BadCRC
//   ipv4.Frame.CRCWrite{Header,TCPPseudo,UDPPseudo}   ipv4::CRCWrite*
//   ipv6.Frame.CRCWritePseudo                          ipv6::CRCWritePseudo
//   internet.StackEthernetConfig{AppendCRC32,CRC32Update} + the FCS append of
//   StackEthernet.Encapsulate (internet/stack-ethernet.go:203-215)
//                                                      internet::AppendFCS
//
// Batch extensions (device-resident, HIP): ethernet::CRC32Batch,
// ethernet::VerifyFCSBatch, lneto::PayloadSum16Batch.  They return LNX_OK or a
// negative LNX_E* code (the Go side would wrap these into an error value).
#pragma once
#include <cstddef>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "lneto_amd.h"

namespace lneto {

// Mirrors lneto's error convention for this path: a checksum mismatch makes
// the caller drop the frame with ErrBadCRC (errors.go:10).
enum class Err : int { None = 0, BadCRC = 3 };

// Non-owning byte view (the Go []byte of the reference API).
struct Bytes {
  const uint8_t* p = nullptr;
  size_t n = 0;
  Bytes() = default;
  Bytes(const uint8_t* p_, size_t n_) : p(p_), n(n_) {}
  Bytes(const std::vector<uint8_t>& v) : p(v.data()), n(v.size()) {}  // NOLINT
  Bytes sub(size_t lo, size_t hi) const { return Bytes(p + lo, hi - lo); }
};

// lneto.CRC791 (crc.go:13-62).  The zero value is ready to use.
struct CRC791 {
  uint32_t sum = 0;
  // Panics in Go on odd length (crc.go:30); here the trailing byte is ignored
  // and callers must pass even lengths, as the reference requires.
  void WriteEven(Bytes b) { sum = lnx_sum_write_even(sum, b.p, b.n); }
  void AddUint32(uint32_t v) {
    AddUint16(uint16_t(v >> 16));
    AddUint16(uint16_t(v));
  }
  void AddUint16(uint16_t v) { sum += v; }
  uint16_t Sum16() const { return lnx_sum16(sum); }
  uint16_t PayloadSum16(Bytes b) const { return lnx_sum16_payload(sum, b.p, b.n); }
  void Reset() { sum = 0; }
};

inline uint16_t NeverZeroSum(uint16_t s) { return lnx_never_zero_sum(s); }

// Batch: out[i] = CRC791{seed[i]}.PayloadSum16(bytes[off[i] : off[i]+len[i]]) on the GPU.
inline int PayloadSum16Batch(const uint8_t* d_bytes, const uint64_t* d_off, const uint32_t* d_len,
                             const uint32_t* d_seed, uint64_t n, uint16_t* d_out, void* stream = nullptr) {
  return lnx_sum16_batch(d_bytes, d_off, d_len, d_seed, n, d_out, stream);
}

}  // namespace lneto

namespace ethernet {
using lneto::Bytes;

// The plugin-hook signature of StackEthernetConfig.CRC32Update
// (internet/stack-ethernet.go:31-32): func(crc uint32, p []byte) uint32.
using CRC32UpdateFunc = uint32_t (*)(uint32_t crc, const uint8_t* p, size_t n);

// Go crc32.Update(crc, crc32.IEEETable, p): pass as CRC32Update.
inline uint32_t CRC32Update(uint32_t crc, const uint8_t* p, size_t n) { return lnx_crc32_update(crc, p, n); }

inline uint32_t CRC32(Bytes data) { return lnx_crc32(data.p, data.n); }

inline int CRC32Search(Bytes data, int minOffCRC) {
  return (int)lnx_crc32_search(data.p, data.n, minOffCRC);
}

// Batch extensions over packed frames (device pointers).
// flags: LNX_BATCH_SHORT_FRAMES for a short-frame mix (the staged lane-stream kernel).
inline int CRC32Batch(const uint8_t* d_frames, const uint64_t* d_off, uint64_t n, uint32_t* d_crc,
                      void* stream = nullptr, uint32_t flags = 0) {
  return flags ? lnx_crc32_batch_ex(d_frames, d_off, n, d_crc, flags, stream)
               : lnx_crc32_batch(d_frames, d_off, n, d_crc, stream);
}
inline int VerifyFCSBatch(const uint8_t* d_frames, const uint64_t* d_off, uint64_t n, uint8_t* d_ok,
                          void* stream = nullptr, uint32_t flags = 0) {
  return flags ? lnx_fcs_verify_batch_ex(d_frames, d_off, n, d_ok, flags, stream)
               : lnx_fcs_verify_batch(d_frames, d_off, n, d_ok, stream);
}
// Frames in ring slots: CRC32 of bytes[start[i] : start[i] + len[i]].
inline int CRC32Segments(const uint8_t* d_bytes, const uint64_t* d_start, const uint32_t* d_len, uint64_t n,
                         uint32_t* d_crc, void* stream = nullptr) {
  return lnx_crc32_segments(d_bytes, d_start, d_len, n, d_crc, stream);
}
// CRC32Search over every capture bytes[off[i] : off[i+1]] (ethernet/crc.go:28-47).
inline int CRC32SearchBatch(const uint8_t* d_bytes, const uint64_t* d_off, const int64_t* d_minOffCRC, uint64_t n,
                            int64_t* d_found, void* stream = nullptr) {
  return lnx_crc32_search_batch(d_bytes, d_off, d_minOffCRC, n, d_found, stream);
}

}  // namespace ethernet

namespace ipv4 {
using lneto::Bytes;
using lneto::CRC791;
// ipv4/frame.go:144-146 — the header sum covers exactly 20 bytes (options are not covered).
inline void CRCWriteHeader(Bytes ip, CRC791& c) { c.WriteEven(ip.sub(0, 20)); }
// ipv4/frame.go:138-142
inline uint16_t CalculateHeaderCRC(Bytes ip) {
  CRC791 c;
  CRCWriteHeader(ip, c);
  return c.Sum16();
}
inline uint16_t TotalLength(Bytes ip) { return uint16_t(ip.p[2] << 8 | ip.p[3]); }
inline uint8_t HeaderLength(Bytes ip) { return uint8_t((ip.p[0] & 0xF) * 4); }
// ipv4/frame.go:154-158
inline void CRCWriteTCPPseudo(Bytes ip, CRC791& c) {
  c.WriteEven(ip.sub(12, 20));
  c.AddUint16(uint16_t(TotalLength(ip) - HeaderLength(ip)));
  c.AddUint16(ip.p[9]);
}
// ipv4/frame.go:166-170
inline void CRCWriteUDPPseudo(Bytes ip, CRC791& c, uint16_t udpLength) {
  c.WriteEven(ip.sub(12, 20));
  c.AddUint16(udpLength);
  c.AddUint16(ip.p[9]);
}
}  // namespace ipv4

namespace ipv6 {
using lneto::Bytes;
using lneto::CRC791;
// ipv6/frame.go:104-108
inline void CRCWritePseudo(Bytes ip6, CRC791& c) {
  c.WriteEven(ip6.sub(8, 40));
  c.AddUint32(uint32_t(ip6.p[4] << 8 | ip6.p[5]));
  c.AddUint32(ip6.p[6]);
}
}  // namespace ipv6

namespace internet {
// The CRC-related fields of StackEthernetConfig (internet/stack-ethernet.go:28-32).
struct StackEthernetConfig {
  bool AppendCRC32 = false;
  ethernet::CRC32UpdateFunc CRC32Update = nullptr;
};

// Config validation of StackEthernet.Configure (internet/stack-ethernet.go:92-93):
// AppendCRC32 without a CRC32Update is an invalid configuration.
inline bool ValidCRCConfig(const StackEthernetConfig& c) { return !(c.AppendCRC32 && c.CRC32Update == nullptr); }

// Tail of StackEthernet.Encapsulate (internet/stack-ethernet.go:203-215): pad the
// frame to 60 bytes, then, if configured, append CRC32Update(0, frame) little-endian.
// `frame` must have room for max(n, 60) + 4 bytes.  Returns the new length.
inline size_t AppendFCS(uint8_t* frame, size_t n, const StackEthernetConfig& c) {
  const size_t minFrameSize = 60;
  while (n < minFrameSize) frame[n++] = 0;
  if (c.CRC32Update != nullptr) {
    const uint32_t crc = c.CRC32Update(0, frame, n);
    frame[n] = uint8_t(crc);
    frame[n + 1] = uint8_t(crc >> 8);
    frame[n + 2] = uint8_t(crc >> 16);
    frame[n + 3] = uint8_t(crc >> 24);
    n += 4;
  }
  return n;
}

// Batch form of AppendFCS with CRC32Update set, in place on frames in ring
// slots of `capacity` bytes (status 6 = lneto.ErrShortBuffer).
inline int AppendFCSBatch(uint8_t* d_bytes, const uint64_t* d_start, uint32_t* d_len, uint64_t n,
                          uint32_t capacity, uint8_t* d_status, void* stream = nullptr) {
  return lnx_fcs_append_batch(d_bytes, d_start, d_len, n, capacity, d_status, stream);
}

// The checksum step of encapsulate4 / encapsulate6 and the ICMP clients
// (internet/stack-ip4.go:202-228, internet/stack-ip6.go:167-181) for every
// frame in ring slots: IPv4 total length / IPv6 payload length, IPv4 header
// CRC, TCP / UDP (NeverZeroSum) / ICMP CRCs, in place; status 0, 18 or 15.
inline int GenerateChecksumsBatch(uint8_t* d_bytes, const uint64_t* d_start, const uint32_t* d_len, uint64_t n,
                                  uint8_t* d_status, void* stream = nullptr) {
  return lnx_tx_checksum_batch(d_bytes, d_start, d_len, n, d_status, stream);
}

// The transmit tail in one read of each frame (lnx_tx_finish_batch): the
// checksum step above (flags & LNX_TX_CHECKSUM), then StackEthernet.Encapsulate's
// padding to 60 bytes and LE FCS (flags & LNX_TX_FCS, internet/stack-ethernet.go:
// 200-214) within `capacity` bytes of each start; d_len updated in place;
// status: the checksum step's 18 / 15 if non-zero, else 0 or 6 (ErrShortBuffer).
inline int FinishBatch(uint8_t* d_bytes, const uint64_t* d_start, uint32_t* d_len, uint64_t n, uint32_t capacity,
                       uint8_t* d_status, uint32_t flags = LNX_TX_CHECKSUM | LNX_TX_FCS, void* stream = nullptr) {
  return lnx_tx_finish_batch(d_bytes, d_start, d_len, n, capacity, flags, d_status, stream);
}

// The stack configuration the receive path consults before and between its
// checksum checks (lnx_rx_filter): the Ethernet stack's MAC and multicast
// acceptance (internet/stack-ethernet.go:56-58,146-152), the EtherTypes with a
// handler (RegisterEthernet, :158-161), the IPv4 / IPv6 stacks' addresses,
// multicast / broadcast acceptance and protocol handlers
// (internet/stack-ip4.go:88-93,108-141, internet/stack-ip6.go:74,93-111).
struct StackFilter {
  uint8_t MAC[6] = {};
  bool AcceptMulticastEthernet = false, AcceptMulticast4 = false, AcceptBroadcast4 = false,
       AcceptMulticast6 = false;
  uint8_t Addr4[4] = {};   // 0.0.0.0: every destination accepted (stack-ip4.go:108)
  uint8_t Addr6[16] = {};  // ::: every destination accepted
  std::vector<uint16_t> EtherTypes{0x0800, 0x86DD, 0x0806};
  std::vector<uint8_t> Protocols4{1, 6, 17}, Protocols6{6, 17, 58};

  // The C-ABI form; false for more than 8 EtherTypes or one RegisterEthernet
  // rejects (proto <= 1500 -> ErrInvalidConfig, internet/stack-ethernet.go:131-135).
  bool ToC(lnx_rx_filter* f) const {
    if (EtherTypes.size() > 8) return false;
    for (uint16_t et : EtherTypes)
      if (et <= 1500) return false;
    *f = lnx_rx_filter{};
    for (int i = 0; i < 6; ++i) f->mac[i] = MAC[i];
    f->eth_accept_multicast = AcceptMulticastEthernet, f->ip4_accept_multicast = AcceptMulticast4;
    f->ip4_accept_broadcast = AcceptBroadcast4, f->ip6_accept_multicast = AcceptMulticast6;
    for (int i = 0; i < 4; ++i) f->ip4[i] = Addr4[i];
    for (int i = 0; i < 16; ++i) f->ip6[i] = Addr6[i];
    f->n_ethertypes = uint32_t(EtherTypes.size());
    for (size_t i = 0; i < EtherTypes.size(); ++i) f->ethertypes[i] = EtherTypes[i];
    for (uint8_t p : Protocols4) f->ip4_protocols[p >> 3] |= uint8_t(1u << (p & 7));
    for (uint8_t p : Protocols6) f->ip6_protocols[p >> 3] |= uint8_t(1u << (p & 7));
    return true;
  }
};

// Receive-path checksum verdicts of every Ethernet frame (0 or the lneto
// errGeneric code), StackEthernet.Demux -> demux4 / demux6.
// icmp: the ICMP clients' checks too (LNX_VERIFY_ICMP).  With a StackFilter,
// frames the stack would not accept get ErrPacketDrop where lneto drops them.
inline int VerifyIngressBatch(const uint8_t* d_frames, const uint64_t* d_off, uint64_t n, uint8_t* d_verdict,
                              bool evilBit = false, void* stream = nullptr, bool icmp = false,
                              const StackFilter* filter = nullptr) {
  const uint32_t flags = (evilBit ? LNX_VERIFY_EVIL_BIT : 0u) | (icmp ? LNX_VERIFY_ICMP : 0u);
  if (!filter) return lnx_ingress_verify_batch(d_frames, d_off, n, flags, d_verdict, stream);
  lnx_rx_filter f;
  if (!filter->ToC(&f)) return LNX_EINVAL;
  return lnx_ingress_verify_batch_filtered(d_frames, d_off, n, flags, &f, d_verdict, stream);
}
}  // namespace internet

namespace netdev {
// Receive ring: bufferSelect-style pinned slots
// (x/netdev/buffer.go:25-37) whose batches run through FCS verify and the
// receive-path verdicts on the GPU.  IngressPackets mirrors
// netdev.Stack.IngressPackets(bufs [][]byte, offset int) (x/netdev/interface.go:82-89):
// frame k = bufs[k][offset:], FCS included; per frame fcsOK and verdict.
class RxRing {
 public:
  RxRing() = default;
  RxRing(const RxRing&) = delete;
  RxRing& operator=(const RxRing&) = delete;
  ~RxRing() { lnx_rx_ring_destroy(r_); }
  int Open(int device, uint32_t nslots, uint32_t slotCap, uint32_t batchSlots = 0, uint32_t depth = 3) {
    lnx_rx_ring_destroy(r_);
    r_ = nullptr;
    nslots_ = nslots, cap_ = slotCap;
    return lnx_rx_ring_create(device, nslots, slotCap, batchSlots, depth, &r_);
  }
  // Slot i's pinned buffer (slotCap bytes) and its length, for a producer.
  uint8_t* Slot(uint32_t i) { return lnx_rx_ring_slots(r_) + size_t(i) * cap_; }
  uint32_t& Len(uint32_t i) { return lnx_rx_ring_lengths(r_)[i]; }
  // The stack's destination and handler configuration for the verdicts
  // (nullptr: accept-all), and whether the device strips the FCS
  // (x/netdev/interface.go:34-40: then no FCS check, verdicts on whole frames).
  int SetFilter(const internet::StackFilter* f) {
    if (!f) return lnx_rx_ring_set_filter(r_, nullptr);
    lnx_rx_filter c;
    if (!f->ToC(&c)) return LNX_EINVAL;
    return lnx_rx_ring_set_filter(r_, &c);
  }
  void SetDeviceStripsFCS(bool v) { noFCS_ = v; }
  // Slots [first, first + count) as IngressPackets(slots, offset).
  int Ingress(uint32_t first, uint32_t count, uint32_t offset, uint8_t* fcsOK, uint8_t* verdict,
              bool evilBit = false) {
    return lnx_rx_ring_ingress(r_, first, count, offset, flags(evilBit), fcsOK, verdict);
  }
  // Caller-owned buffers (gathered into pinned staging for the call only,
  // read in place when they are the ring's slots: SlotBuffers).
  int IngressPackets(const uint8_t* const* bufs, const uint32_t* lens, uint64_t n, uint32_t offset, uint8_t* fcsOK,
                     uint8_t* verdict, bool evilBit = false) {
    return lnx_ingress_packets(r_, bufs, lens, n, offset, flags(evilBit), fcsOK, verdict);
  }
  // IngressPackets(bufs [][]byte, offset int) with the Go slice shape: the
  // buffers' addresses and lengths are staged in the ring object for the call
  // only and dropped after it (the Go binding pins them with runtime.Pinner
  // for exactly that span); fcsOK / verdict are resized.
  int IngressPackets(const std::vector<lneto::Bytes>& bufs, uint32_t offset, std::vector<uint8_t>& fcsOK,
                     std::vector<uint8_t>& verdict, bool evilBit = false) {
    ptrs_.resize(bufs.size());
    lens_.resize(bufs.size());
    for (size_t k = 0; k < bufs.size(); ++k) {
      ptrs_[k] = bufs[k].p;
      lens_[k] = uint32_t(bufs[k].n);
    }
    fcsOK.resize(bufs.size());
    verdict.resize(bufs.size());
    const int rc = lnx_ingress_packets(r_, ptrs_.data(), lens_.data(), bufs.size(), offset, flags(evilBit),
                                       fcsOK.data(), verdict.data());
    ptrs_.clear();  // unpinned: nothing refers to the caller's buffers after the call
    lens_.clear();
    return rc;
  }
  // netdev.Stack.EgressPackets(bufs, sizes, offset) (x/netdev/interface.go:85)
  // for the device's part of the transmit path: frame k = bufs[k][offset :
  // offset + lens[k]] gets its checksums (checksum) and its padding + FCS
  // (fcs) in place; lens[k] is updated, status[k] = 0, 18, 15 or 6.
  int EgressPackets(uint8_t* const* bufs, uint32_t* lens, uint64_t n, uint32_t offset, uint32_t capacity,
                    uint8_t* status, bool checksum = true, bool fcs = true) {
    return lnx_egress_packets(r_, bufs, lens, n, offset, capacity,
                              (checksum ? LNX_TX_CHECKSUM : 0u) | (fcs ? LNX_TX_FCS : 0u), status);
  }
  uint32_t Slots() const { return nslots_; }
  uint32_t SlotCap() const { return cap_; }
  // The slots as netdev RunnerConfig.Buffers (x/netdev/runner.go:92-94): a
  // Runner built on these hands IngressPackets / EgressPackets views of the
  // ring's own pinned memory, which the kernels read (and patch) in place.
  std::vector<lneto::Bytes> SlotBuffers() {
    std::vector<lneto::Bytes> b;
    for (uint32_t k = 0; k < nslots_; ++k) b.emplace_back(Slot(k), cap_);
    return b;
  }
  // In-place access to the slots (default) or copies through staging.
  int SetZeroCopy(bool on) { return lnx_rx_ring_set_zero_copy(r_, on ? 1 : 0); }
  // Batches below `frames` run on the host (no launch); 0 = always the GPU.
  int SetHostThreshold(uint32_t frames) { return lnx_rx_ring_set_host_threshold(r_, frames); }
  lnx_rx_ring_counters Stats() const {
    lnx_rx_ring_counters c{};
    (void)lnx_rx_ring_stats(r_, &c);
    return c;
  }

 private:
  uint32_t flags(bool evilBit) const { return (evilBit ? LNX_VERIFY_EVIL_BIT : 0u) | (noFCS_ ? LNX_RX_NO_FCS : 0u); }
  lnx_rx_ring* r_ = nullptr;
  uint32_t nslots_ = 0, cap_ = 0;
  bool noFCS_ = false;
  std::vector<const uint8_t*> ptrs_;
  std::vector<uint32_t> lens_;
};

// The batching half of a netdev Runner (x/netdev/runner.go:420-476) for the
// ring: the reference's Runner hands IngressPackets ONE buffer per call
// (r.bufsaux = [1][]byte{buf}, :432-433,469-470) and releases it at once.
// RxBatcher keeps the receive handler's shape — Put copies an incoming frame
// into the next free pinned slot, as bufferSelect.goroPutRx copies it into a
// free buffer (x/netdev/buffer.go:77-98) — but Drain hands every pending slot
// to ONE Ingress call (up to Slots() frames), then frees them all; Put drains
// by itself when the slots are full.  The callback gets each frame's index in
// Put order, its FCS verdict and its receive verdict.  INTEGRATION.md §2.2
// has the same loop in Go.
class RxBatcher {
 public:
  using OnFrame = void (*)(void* ctx, uint64_t index, uint8_t fcsOK, uint8_t verdict);
  RxBatcher(RxRing& ring, OnFrame on, void* ctx) : ring_(ring), on_(on), ctx_(ctx) {}
  // false: frame longer than a slot (dropped, as goroPutRx drops it)
  bool Put(const uint8_t* frame, uint32_t len) {
    if (len > ring_.SlotCap()) return false;
    if (pending_ == ring_.Slots() && Drain() != LNX_OK) return false;
    std::memcpy(ring_.Slot(pending_), frame, len);
    ring_.Len(pending_) = len;
    ++pending_;
    return true;
  }
  int Drain() {
    if (pending_ == 0) return LNX_OK;
    ok_.resize(pending_);
    verdict_.resize(pending_);
    const int rc = ring_.Ingress(0, pending_, 0, ok_.data(), verdict_.data());
    if (rc == LNX_OK)
      for (uint32_t k = 0; k < pending_; ++k) on_(ctx_, next_ + k, ok_[k], verdict_[k]);
    next_ += pending_;
    pending_ = 0;
    return rc;
  }
  uint32_t Pending() const { return pending_; }

 private:
  RxRing& ring_;
  OnFrame on_;
  void* ctx_;
  uint32_t pending_ = 0;
  uint64_t next_ = 0;
  std::vector<uint8_t> ok_, verdict_;
};
}  // namespace netdev
