// ingress_kernel.hip — fused receive-path checksum verification, gfx950
// (SURVEY.md §8(f).2).
//
// For every received Ethernet frame (FCS stripped) the verdict lneto's receive
// path reaches at its checksum stage, as one kernel:
//   StackEthernet.Demux size checks (internet/stack-ethernet.go:139-165,
//   ethernet/frame.go:13-18,119-127), then by EtherType
//   0x0800 demux4 (internet/stack-ip4.go:100-164): ipv4.NewFrame, the first
//          error of ValidateExceptCRC (ipv4/frame.go:214-238), the header sum
//          over the first 20 bytes only (ipv4/frame.go:138-146), TCP / UDP
//          checksums with the pseudo-header seeds (ipv4/frame.go:154-170) and
//          the UDP size checks (udp/frame.go:15-20,96-104);
//   0x86DD demux6 (internet/stack-ip6.go:86-138): ipv6.NewFrame, ValidateSize
//          (ipv6/frame.go:123-128), TCP / UDP sums with CRCWritePseudo
//          (ipv6/frame.go:104-108); the UDP sum covers the whole IPv6 payload;
//   with kVerifyIcmp, ICMP messages also take their client's Demux checks up to
//          the checksum (ipv4/icmpv4/client.go:89-102: size, echo types,
//          sum with no pseudo-header; ipv6/icmpv6/client.go:100-115: size,
//          sum with the pseudo-header, as CRCWritePseudo with proto 58).
// The verdict is 0 (every check passed, or none applies) or the errGeneric
// code the reference returns (errors.go:6-28).  Destination filtering and
// handler lookup depend on stack configuration: taken as accept-all.
//
// Layout: one 16-lane row per frame, four frames per wave.  The row's first
// batch of dword loads (frame offsets from 12 on) also carries every header
// field: they are gathered from the row's lanes with ds_bpermute and realigned
// with v_alignbyte, so a frame costs one round trip before its sums start.  The sums use the identity of
// sum16_kernel.hip: the uint32 sum of big-endian 16-bit words of a segment that
// starts at an even frame offset is 256*E + O (E / O = sums of the bytes at
// even / odd frame offsets), and every segment here starts at an even offset
// (14, 22, 26, 14 + 4*IHL, 54).  One pass over the frame's aligned dwords
// accumulates two (E, O) pairs with v_dot4_u32_u8: the IPv4 header [14, 34)
// and the transport sum = pseudo-header addresses + transport segment.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include "rx_filter.hpp"

namespace lnx {

constexpr int kIngBlock = 256;
// dwords per lane in flight: 24 (1536 B per row) reads a 1500-B frame in one
// batch; 0.283 ms against 0.291 for 8 and 0.313 for 16 on 1 M x 1500 B
// (bench.py --op ingress, LNX_PROF_INGRESS_UNROLL; profiles/r1g_ingress_unroll.txt)
[[maybe_unused]] constexpr int kIngUnroll = 24;
// qword lanes (r1h product): 12 qwords per lane in flight, again 1536 B per row
constexpr int kIngUnrollQ = 12;
constexpr uint32_t kErrPacketDrop = 2, kErrBadCRC = 3, kErrInvalidField = 14, kErrInvalidLengthField = 15,
                   kErrTruncatedFrame = 18;
constexpr uint32_t kVerifyEvilBit = 1, kVerifyIcmp = 2;

// bit `proto` of a 256-bit mask held in kernel-argument words (a select chain:
// no indexed scratch)
__device__ __forceinline__ bool proto_bit(const uint32_t (&m)[8], uint32_t proto) {
  const uint32_t w = proto >> 5;
  const uint32_t word = w == 0 ? m[0] : w == 1 ? m[1] : w == 2 ? m[2] : w == 3 ? m[3] : w == 4 ? m[4]
                        : w == 5 ? m[5] : w == 6 ? m[6] : m[7];
  return (word >> (proto & 31u)) & 1u;
}

__device__ __forceinline__ uint32_t ing_keep_from(int32_t lo) {
  lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
  return (uint32_t)(0xFFFFFFFFull << (8 * lo));
}
// byte mask of the frame offsets [a, b) inside the word whose byte 0 is at o0
__device__ __forceinline__ uint32_t range_mask(int32_t o0, int32_t a, int32_t b) {
  return ing_keep_from(a - o0) & ~ing_keep_from(b - o0);
}

__device__ __forceinline__ uint32_t row_add(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return v;
}

__device__ __forceinline__ uint16_t ing_sum16(uint32_t sum) {  // crc.go:17-21
  sum = (sum & 0xffffu) + (sum >> 16);
  return (uint16_t)~(uint16_t)(sum + (sum >> 16));
}

// QW: lanes load qwords (global_load_dwordx2: a 16-lane row reads a whole
// 128-byte line per instruction), UNR qwords per lane in flight; otherwise
// dwords (a 64-byte half line per row instruction), UNR dwords in flight
//
// GEN (tx_checksum_batch): the same rows GENERATE the
// checksums instead (encapsulate4 / encapsulate6 / the ICMP clients after the
// child wrote its n payload bytes, internet/stack-ip4.go:202-228,
// internet/stack-ip6.go:167-181, ipv4/icmpv4/client.go:210-214,
// ipv6/icmpv6/client.go:135-148): the length fields are set from the frame
// length, and the sums are taken over the bytes as loaded with the old field
// values subtracted (uint32 wrap: the same value as summing with the fields
// zeroed); lanes 0..7 of the row then store the 2-byte fields (IPv4 total
// length / IPv6 payload length, header CRC, transport CRC, UDP length) and
// `verdict` receives the status (0, or 18 / 15 with the frame untouched).
// (the generate form writes the frames: its byte pointer is not const)
template <bool GEN>
using IngBytes = std::conditional_t<GEN, uint8_t, const uint8_t>;

// FILT = false: the instance for batches without a stack filter (the filter
// checks compiled out; the r3 code path and its speed)
template <int UNR, bool QW, bool GEN = false, bool FILT = true>
__global__ void __launch_bounds__(kIngBlock)
ingress_verify_kernel(IngBytes<GEN>* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t n,
                      uint32_t flags, uint8_t* __restrict__ verdict, const uint32_t* __restrict__ seg_len,
                      uint32_t trim, RxFilter filt, uint32_t* __restrict__ gate, uint32_t epoch, uint64_t short_mean) {
  static_assert(!GEN || QW, "generate runs on the qword rows");
  // lnx_ingress_verify_batch (offsets mode): a batch whose mean frame is
  // shorter than short_mean bytes (or whose offsets end below their start)
  // is the receive check's without its CRC (rx_verify_kernel, launched behind
  // this one: one lane per frame for the headers, 0.50 against 0.69 ms on 4 M
  // x 128 B, 2.06 against 2.61 on configs[3]'s Zipf mix; this kernel wins from
  // ~1280 B, tools/prof/ingress_vs_rv.py): every workgroup reads the batch's
  // two ends, and workgroup 0 leaves the call's epoch in the gate word
  // lnx_tx_checksum_batch (segment mode, GEN) likewise goes to tx_finish with
  // LNX_TX_CHECKSUM only below its crossover: tx_gate_probe_kernel (below, one wave
  // launched first) has left the epoch in the gate word then
  if (gate) {
    if (seg_len) {
      if (*gate == epoch) return;
    } else {
      const uint64_t a = off[0], b = off[n];
      if (b < a || b - a < short_mean * n) {
        if (blockIdx.x == 0 && threadIdx.x == 0) *gate = epoch;
        return;
      }
    }
  }
  // offsets mode (seg_len null): frame f = bytes[off[f] : off[f+1] - trim];
  // segment mode (the receive ring): frame f = bytes[off[f] : off[f] + seg_len[f] - trim],
  // i.e. the FCS (trim = 4) is stripped, empty if the buffer is shorter than trim
  const uint32_t lane = threadIdx.x & 63u, p = lane & 15u, row = lane >> 4;
  const uint64_t nwaves = (uint64_t)gridDim.x * (kIngBlock / 64);
  for (uint64_t q = (uint64_t)blockIdx.x * (kIngBlock / 64) + (threadIdx.x >> 6); q * 4 < n; q += nwaves) {
    const uint64_t f = q * 4 + row;
    const bool live = f < n;
    const uint64_t s = live ? off[f] : 0;
    const uint32_t sl = live && seg_len ? seg_len[f] : 0u;
    const uint64_t e1 = live && !seg_len ? off[f + 1] : 0;
    const uint64_t e = !live ? 0 : (seg_len ? s + (sl > trim ? sl - trim : 0u) : (e1 > s + trim ? e1 - trim : s));
    const uint64_t len64 = e > s ? e - s : 0;
    const uint32_t L = len64 < 0x7FFFFFFFull ? (uint32_t)len64 : 0x7FFFFFFFu;
    IngBytes<GEN>* fr = bytes + s;
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(fr) & (QW ? 7u : 3u));
    const uint32_t* base = reinterpret_cast<const uint32_t*>(fr - mis);
    // dword k of base holds frame offsets 4k - mis .. 4k - mis + 3
    const int32_t kstart = (int32_t)((12 + mis) >> 2);          // dword holding frame offset 12
    const int32_t kfend = (int32_t)((L + mis + 3) >> 2);         // dwords touching the frame

    // ---- first batch: dwords kstart + p + 16u (QW: qwords qstart + p + 16u,
    // qword Q = dwords 2Q, 2Q + 1); it also holds every header field.
    // (Round 3 A/B: the same loads through one raw buffer descriptor per wave,
    // out-of-range offsets in place of the guards, cost 8 more VGPRs, one
    // wave per SIMD and 9 % of the time: 0.2696 against 0.2476 ms,
    // profiles/r3n_ingress_buffer_loads_rejected.txt.)
    const uint2* base2 = reinterpret_cast<const uint2*>(base);
    const int32_t qstart = kstart >> 1, qfend = (kfend + 1) >> 1;
    uint32_t x[UNR];
    uint2 y[QW ? UNR : 1];
#pragma unroll
    for (int u = 0; u < UNR; ++u) {
      if constexpr (QW) {
        const int32_t q = qstart + (int32_t)p + 16 * u;
        y[u] = L >= 14 && q < qfend ? base2[q] : make_uint2(0u, 0u);
      } else {
        const int32_t k = kstart + (int32_t)p + 16 * u;
        x[u] = L >= 14 && k < kfend ? base[k] : 0u;
      }
    }
    // dword kstart + kk of this row (kk < 31) from the lane that loaded it
    auto rowword = [&](int32_t kk) -> uint32_t {
      if constexpr (QW) {
        const uint32_t rel = (uint32_t)(kstart - 2 * qstart + kk);  // dword of the row's first qword batch
        const int addr = (int)((row * 16u + ((rel >> 1) & 15u)) * 4u);
        const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)y[0].x);
        const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)y[0].y);
        return (rel & 1u) ? b : a;
      } else {
        const int addr = (int)((row * 16u + ((uint32_t)kk & 15u)) * 4u);
        const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)x[0]);
        const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)x[1]);
        return kk < 16 ? a : b;
      }
    };
    const uint32_t sh = (12 + mis) & 3u;  // byte of frame offset 12 inside dword kstart
    const uint32_t w0 = rowword(0), w1 = rowword(1), w2 = rowword(2), w3 = rowword(3);
    const uint32_t H0 = __builtin_amdgcn_alignbyte(w1, w0, sh);  // frame bytes 12..15
    const uint32_t H1 = __builtin_amdgcn_alignbyte(w2, w1, sh);  // 16..19
    const uint32_t H2 = __builtin_amdgcn_alignbyte(w3, w2, sh);  // 20..23
    auto byt = [](uint32_t w, int i) -> uint32_t { return (w >> (8 * i)) & 0xFFu; };
    auto be = [&](uint32_t w, int i) -> uint32_t { return (byt(w, i) << 8) | byt(w, i + 1); };
    // big-endian 16-bit field at frame offset o (o + 1 < L, o >= 12)
    auto field16 = [&](uint32_t o) -> uint32_t {
      const int32_t kk = (int32_t)((o + mis) >> 2) - kstart;
      const uint32_t lo = rowword(kk), hi = rowword(kk + 1);
      const uint32_t v2 = __builtin_amdgcn_alignbyte(hi, lo, (o + mis) & 3u);
      return ((v2 & 0xFFu) << 8) | ((v2 >> 8) & 0xFFu);
    };

    // ---- header parse: row-uniform; v = verdict so far, sums requested below
    uint32_t v = 0;
    uint32_t v_udp4 = 0;  // IPv4 UDP / ICMP size verdict: demux4 reports it only after the header sum passed
    bool hdr_sum = false, l4_sum = false;
    int32_t pa = 0, pb = 0, la = 0, lb = 0;  // pseudo-address bytes [pa, pb), transport [la, lb)
    uint32_t lseed = 0;                       // length + protocol words of the pseudo-header
    // A 16-bit big-endian field value v at an even frame offset adds cv(v) to
    // the qword rows' little-endian half-word sum S (see the sums below): its
    // high byte sits at address parity mis & 1
    auto cv = [&](uint32_t v) -> uint32_t { return (mis & 1u) ? v : (((v & 0xFFu) << 8) | (v >> 8)); };
    // GEN: the fields the step writes (frame offset, new value; 0 = none)
    uint32_t g_off[4] = {0, 0, 0, 0}, g_val[4] = {0, 0, 0, 0};
    uint32_t g_fix_h = 0, g_fix_t = 0;  // cv(new) - cv(old) of the summed fields (header, transport), mod 2^32
    bool g_nz = false;                   // UDP: NeverZeroSum (crc.go:65-71)
    if constexpr (GEN) {
      if (L < 14) {
        v = kErrTruncatedFrame;
      } else {
        const uint32_t et = be(H0, 0);
        if (et == 0x0800) {
          const uint32_t ihl = byt(H0, 2) & 15u, hl = 4 * ihl;
          if (L < 34) v = kErrTruncatedFrame;
          else if (ihl < 5) v = kErrInvalidLengthField;
          else if (14 + hl > L) v = kErrTruncatedFrame;
          else if (L - 14 > 0xFFFFu) v = kErrInvalidLengthField;
          if (v == 0) {
            const uint32_t tl = L - 14, nn = tl - hl, proto = byt(H2, 3);
            const uint32_t need = proto == 6 ? 20u : (proto == 17 || proto == 1) ? 8u : 0u;
            if (nn < need) v = kErrTruncatedFrame;
            if (v == 0) {
              hdr_sum = true;
              g_off[0] = 16, g_val[0] = tl;   // SetTotalLength(n + hl)
              g_off[1] = 24;                  // SetCRC(CalculateHeaderCRC()), value after the sums
              g_fix_h = cv(tl) - cv(be(H1, 0)) - cv(field16(24));
              if (need) {
                l4_sum = true;
                la = 14 + hl, lb = L;
                const uint32_t at = proto == 6 ? 16u : proto == 17 ? 6u : 2u;
                g_off[2] = la + at;
                g_fix_t = 0u - cv(field16(la + at));
                if (proto != 1) pa = 26, pb = 34, lseed = nn + proto;  // CRCWriteTCPPseudo / CRCWriteUDPPseudo(n)
                if (proto == 17) {
                  g_off[3] = la + 4, g_val[3] = nn;  // SetLength(n)
                  g_fix_t += cv(nn) - cv(field16(la + 4));
                  g_nz = true;
                }
              }
            }
          }
        } else if (et == 0x86DD) {
          const uint32_t nn = L - 54, proto = byt(H2, 0);
          if (L < 54) v = kErrTruncatedFrame;
          else if (nn > 0xFFFFu) v = kErrInvalidLengthField;
          const uint32_t need = proto == 6 ? 20u : (proto == 17 || proto == 58) ? 8u : 0u;
          if (v == 0 && nn < need) v = kErrTruncatedFrame;
          if (v == 0) {
            g_off[0] = 18, g_val[0] = nn;  // SetPayloadLength(n)
            if (need) {
              l4_sum = true;
              pa = 22, pb = 54, la = 54, lb = L;  // CRCWritePseudo: AddUint32(n), AddUint32(proto)
              lseed = nn + proto;
              const uint32_t at = proto == 6 ? 16u : proto == 17 ? 6u : 2u;
              g_off[2] = 54 + at;
              g_fix_t = 0u - cv(field16(54 + at));
              if (proto == 17) {
                g_off[3] = 58, g_val[3] = nn;
                g_fix_t += cv(nn) - cv(field16(58));
                g_nz = true;
              }
            }
          }
        }
      }
    } else {
      // bytes o .. o + 3 of the frame (o >= 12, o + 3 < L), little-endian packed
      auto field32 = [&](uint32_t o) -> uint32_t {
        const int32_t kk = (int32_t)((o + mis) >> 2) - kstart;
        return __builtin_amdgcn_alignbyte(rowword(kk + 1), rowword(kk), (o + mis) & 3u);
      };
      if (L < 14) {
        v = kErrTruncatedFrame;
      } else {
        const uint32_t et = be(H0, 0);
        bool eth_drop = false, et_handler = true;
        if (FILT && filt.on) {
          // StackEthernet.Demux (internet/stack-ethernet.go:146-152), before
          // ValidateSize: a frame neither broadcast nor for the stack's MAC is
          // dropped unless multicast frames are accepted and the group bit is set
          const uint32_t* w = base + (mis >> 2);
          const uint32_t sm = mis & 3u, m0 = w[0], m1 = w[1], m2 = w[2];
          const uint32_t D0 = __builtin_amdgcn_alignbyte(m1, m0, sm), D1 = __builtin_amdgcn_alignbyte(m2, m1, sm) & 0xFFFFu;
          const bool bcast = D0 == 0xFFFFFFFFu && D1 == 0xFFFFu;
          const bool mine = D0 == filt.mac_lo && D1 == filt.mac_hi;
          eth_drop = !bcast && !mine && !(filt.eth_mc && (D0 & 1u));
          // handlers.demuxByProto(etype) (stack-ethernet.go:158-161): no handler -> drop
          et_handler = false;
#pragma unroll
          for (int i = 0; i < 8; ++i) et_handler = et_handler || (i < (int)filt.n_et && filt.et[i] == et);
        }
        if (eth_drop) {
          v = kErrPacketDrop;
        } else if (et <= 1500 && L < et) {
          v = kErrInvalidLengthField;
        } else if (et == 0x8100 && L < 18) {
          v = kErrTruncatedFrame;
        } else if (!et_handler) {
          v = kErrPacketDrop;
        } else if (et == 0x0800) {
          const uint32_t M = L - 14;
          if (M < 20) {
            v = kErrTruncatedFrame;
          } else {
            const uint32_t b0 = byt(H0, 2), tl = be(H1, 0), ihl = b0 & 15u;
            if (FILT && filt.on && filt.ip4 != 0u) {
              // demux4's destination check (internet/stack-ip4.go:108-119), before ValidateExceptCRC
              const uint32_t dst = field32(30);
              const bool mc = (dst & 0xF0u) == 0xE0u, bc = dst == 0xFFFFFFFFu;  // ipv4/definitions.go:17-36
              if (dst != filt.ip4 && !(filt.ip4_mc && mc) && !(filt.ip4_bc && bc)) v = kErrPacketDrop;
            }
            if (v != 0) {
            } else if (tl < 20) v = kErrInvalidLengthField;
            else if (tl > M) v = kErrTruncatedFrame;
            else if (ihl < 5 || ihl * 4 > tl) v = kErrInvalidLengthField;
            else if ((b0 >> 4) != 4) v = kErrInvalidField;
            else if ((flags & kVerifyEvilBit) && (be(H2, 0) & (1u << 13))) v = kErrPacketDrop;
            if (v == 0) {
              hdr_sum = true;
              const uint32_t hl = ihl * 4, proto = byt(H2, 3), P = tl - hl;
              if (FILT && filt.on && !proto_bit(filt.p4, proto)) {
                v_udp4 = kErrPacketDrop;  // nodeByProto nil (stack-ip4.go:135-141), after the header sum
              } else if (proto == 6) {
                l4_sum = true;
                pa = 26, pb = 34, la = 14 + hl, lb = 14 + tl;
                lseed = ((tl - hl) & 0xFFFFu) + 6u;
              } else if (proto == 17) {
                if (P < 8) {
                  v_udp4 = kErrTruncatedFrame;
                } else {
                  const uint32_t ul = field16(14 + hl + 4);
                  if (ul < 8) v_udp4 = kErrInvalidLengthField;
                  else if (ul > P) v_udp4 = kErrTruncatedFrame;
                  else {
                    l4_sum = true;
                    pa = 26, pb = 34, la = 14 + hl, lb = 14 + hl + ul;
                    lseed = ul + 17u;
                  }
                }
              } else if (proto == 1 && (flags & kVerifyIcmp)) {
                if (P < 8) {
                  v_udp4 = kErrTruncatedFrame;
                } else {
                  const uint32_t type = field16(14 + hl) >> 8;
                  if (type != 0 && type != 8) {
                    v_udp4 = kErrPacketDrop;
                  } else {
                    l4_sum = true;  // no pseudo-header: [pa, pb) empty, lseed 0
                    la = 14 + hl, lb = 14 + tl;
                  }
                }
              }
            }
          }
        } else if (et == 0x86DD) {
          const uint32_t M = L - 14;
          if (M < 40) {
            v = kErrTruncatedFrame;
          } else {
            const uint32_t pl = be(H1, 2), proto = byt(H2, 0);
            if (FILT && filt.on && (filt.ip6[0] | filt.ip6[1] | filt.ip6[2] | filt.ip6[3]) != 0u) {
              // demux6's destination check (internet/stack-ip6.go:93-98), before ValidateSize
              const uint32_t d0 = field32(38), d1 = field32(42), d2 = field32(46), d3 = field32(50);
              const bool mine = d0 == filt.ip6[0] && d1 == filt.ip6[1] && d2 == filt.ip6[2] && d3 == filt.ip6[3];
              if (!mine && !(filt.ip6_mc && (d0 & 0xFFu) == 0xFFu)) v = kErrPacketDrop;  // internal/ip.go:30-35
            }
            if (v != 0) {
            } else if (pl + 40 > M) {
              v = kErrInvalidLengthField;
            } else if (FILT && filt.on && !proto_bit(filt.p6, proto)) {
              v = kErrPacketDrop;  // nodeByProto nil (stack-ip6.go:107-111), before the sums
            } else if (proto == 6 || proto == 17 || (proto == 58 && (flags & kVerifyIcmp))) {
              // demux6 size-checks the UDP header only; TCP goes straight to the
              // sum (internet/stack-ip6.go:116-137), whatever pl is.  ICMPv6:
              // icmpv6.NewFrame's size check, then the same pseudo-header sum.
              if (proto == 58 && pl < 8) v = kErrTruncatedFrame;
              if (proto == 17) {
                if (pl < 8) v = kErrTruncatedFrame;
                else if (field16(58) < 8) v = kErrInvalidLengthField;
                else if (field16(58) > pl) v = kErrTruncatedFrame;
              }
              if (v == 0) {
                l4_sum = true;
                pa = 22, pb = 54, la = 54, lb = 54 + pl;  // AddUint32(pl), AddUint32(proto): high halves 0
                lseed = pl + proto;
              }
            }
          }
        }
      }
    }

    // ---- the sums: the first batch is in x; later batches while the summed
    // range [14, end) goes on (kIngUnroll dwords per lane in flight)
    uint32_t hE = 0, hO = 0, tE = 0, tO = 0;
    // qword rows: S = the sum of the little-endian 16-bit halves of the
    // aligned dwords, one v_dot2_u32_u16 per dword (the dword rows keep the
    // even / odd byte sums E, O of two v_dot4 per dword).  S = Σ bytes at even
    // addresses + 256 Σ bytes at odd addresses; with the frame starting at an
    // odd address that is 256 E + O itself, at an even one E + 256 O, which is
    // 256 E + O times 256 modulo 65535 (a byte rotation of the folded sum).
    // The sums of a frame under 64 KiB never wrap 2^32, so sum16 of the
    // rotated fold equals sum16 of 256 E + O (RFC 1071 §2(B)).
    uint32_t hS = 0, tS = 0;
    auto dot2 = [](uint32_t w, uint32_t acc) -> uint32_t {
      typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
      const u16x2 ones = {1, 1};
      return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w), ones, acc, false);
    };
    const bool any_sum = hdr_sum || l4_sum;
    const int32_t end = l4_sum ? lb : (hdr_sum ? 34 : 0);
    const int32_t kend = any_sum ? (end + (int32_t)mis + 3) >> 2 : 0;
    const uint32_t wE = (mis & 1u) ? 0x01000100u : 0x00010001u;  // bytes at even frame offsets
    const uint32_t wO = wE << 8 | wE >> 24;
    const int32_t ha = hdr_sum ? 14 : 0, hb = hdr_sum ? 34 : 0;
    if constexpr (QW) {
      // Only the first qword of the first batch can hold header, pseudo-header
      // or transport-start bytes: every later qword starts at frame offset
      // >= 8 * (qstart + 16) - mis >= 126, past hb = 34, pb <= 54 and
      // la <= 74. There the transport mask is the end bound alone and the
      // header sum takes nothing.
      const int32_t qend = (kend + 1) >> 1;
      // The first batch was loaded up to the frame end (qfend), before the
      // header parse knew the transport end: its qwords at or past qend (bytes
      // after tl, after the UDP length, after pl + 40) are not summed.  Only
      // rows whose frame runs past the transport end take this branch.
      if (qend < qfend) {
#pragma unroll
        for (int u = 1; u < UNR; ++u) {
          const bool past = qstart + (int32_t)p + 16 * u >= qend;
          y[u].x = past ? 0u : y[u].x;
          y[u].y = past ? 0u : y[u].y;
        }
      }
      bool first = true;
      uint2 yl = make_uint2(0u, 0u);  // the row's last qword, on the lane that loaded it (outside the first qwords)
      // A wave-uniform trip count (the most any row of the wave needs): a
      // loop bounded per row, with dwordx2 loads in it, is the shape that
      // returned wrong sums in round 1; lanes past their
      // row's end load nothing (q < qend) and add zeros.
      int32_t nit = qend > qstart ? (qend - qstart + 16 * UNR - 1) / (16 * UNR) : 0;
      nit = max(nit, __shfl_xor(nit, 16));
      nit = max(nit, __shfl_xor(nit, 32));
      nit = __builtin_amdgcn_readfirstlane(nit);
      for (int32_t it = 0; it < nit; ++it) {
        const int32_t q0 = qstart + (int32_t)p + 16 * UNR * it;
        if (!first) {
#pragma unroll
          for (int u = 0; u < UNR; ++u) {
            const int32_t q = q0 + 16 * u;
            y[u] = q < qend ? base2[q] : make_uint2(0u, 0u);
          }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const uint32_t w = h ? y[u].y : y[u].x;
            const int32_t o0 = 4 * (2 * (q0 + 16 * u) + h) - (int32_t)mis;
            if (u == 0 && first) {
              const uint32_t xh = w & range_mask(o0, ha, hb);
              const uint32_t xt = w & (range_mask(o0, pa, pb) | range_mask(o0, la, lb));
              hS = dot2(xh, hS);
              tS = dot2(xt, tS);
            } else {
              // summed whole: every qword here lies below qend (later batches
              // load under q < qend; the first batch's qwords at or past qend
              // were zeroed above), so only qword qend - 1 can hold bytes at
              // or past lb; the lane holding it keeps it and takes those bytes
              // back out after the loop
              tS = dot2(w, tS);
            }
          }
        }
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const bool isl = q0 + 16 * u == qend - 1 && !(u == 0 && first);
          yl.x = isl ? y[u].x : yl.x;
          yl.y = isl ? y[u].y : yl.y;
        }
        first = false;
      }
      // bytes at or past lb of the last qword (zero unless this lane kept it)
      const int32_t ol = 8 * (qend - 1) - (int32_t)mis;  // frame offset of its first byte
      const uint32_t j0 = yl.x & ing_keep_from(lb - ol), j1 = yl.y & ing_keep_from(lb - ol - 4);
      tS -= dot2(j0, dot2(j1, 0u));
    }
    for (int32_t k0 = kstart + (int32_t)p; !QW && k0 < kend; k0 += 16 * UNR) {
      if (k0 != kstart + (int32_t)p) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
          const int32_t k = k0 + 16 * u;
          x[u] = k < kend ? base[k] : 0u;
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int32_t o0 = 4 * (k0 + 16 * u) - (int32_t)mis;
        const uint32_t xh = x[u] & range_mask(o0, ha, hb);
        const uint32_t xt = x[u] & (range_mask(o0, pa, pb) | range_mask(o0, la, lb));
        hE = __builtin_amdgcn_udot4(xh, wE, hE, false);
        hO = __builtin_amdgcn_udot4(xh, wO, hO, false);
        tE = __builtin_amdgcn_udot4(xt, wE, tE, false);
        tO = __builtin_amdgcn_udot4(xt, wO, tO, false);
      }
    }
    // hX, tX: 256 E + O of the header and transport bytes, or (qword rows) a
    // value congruent to it modulo 65535 that is zero exactly when it is
    uint32_t hX, tX;
    if constexpr (QW) {
      // GEN: the field fixes are row-uniform, added on lane 0 of the row only
      hS = row_add(hS + (p == 0 ? g_fix_h : 0u)), tS = row_add(tS + (p == 0 ? g_fix_t : 0u));
      auto conv = [&](uint32_t S) -> uint32_t {
        if (mis & 1u) return S;
        uint32_t f = (S & 0xFFFFu) + (S >> 16);
        f = (f & 0xFFFFu) + (f >> 16);
        return ((f << 8) | (f >> 8)) & 0xFFFFu;
      };
      hX = conv(hS), tX = conv(tS);
    } else {
      hE = row_add(hE), hO = row_add(hO), tE = row_add(tE), tO = row_add(tO);
      hX = 256u * hE + hO, tX = 256u * tE + tO;
    }
    if constexpr (GEN) {
      g_val[1] = ing_sum16(hX);
      const uint32_t tc = ing_sum16(tX + lseed);
      g_val[2] = g_nz && tc == 0 ? 0xFFFFu : tc;
      // lane k < 4 stores field k (big-endian): one 16-bit store when the
      // field's address is even, else its two bytes
      const uint32_t k = p;
      const uint32_t fo = k == 0 ? g_off[0] : k == 1 ? g_off[1] : k == 2 ? g_off[2] : g_off[3];
      const uint32_t fv = k == 0 ? g_val[0] : k == 1 ? g_val[1] : k == 2 ? g_val[2] : g_val[3];
      if (live && v == 0 && k < 4 && fo != 0) {
        uint8_t* q = fr + fo;
        if ((reinterpret_cast<uintptr_t>(q) & 1u) == 0) {
          *reinterpret_cast<uint16_t*>(q) = (uint16_t)(((fv & 0xFFu) << 8) | ((fv >> 8) & 0xFFu));
        } else {
          q[0] = (uint8_t)(fv >> 8);
          q[1] = (uint8_t)fv;
        }
      }
    } else {
      if (v == 0 && hdr_sum && ing_sum16(hX) != 0) v = kErrBadCRC;
      if (v == 0) v = v_udp4;  // udp.NewFrame / ValidateSize follow CalculateHeaderCRC (stack-ip4.go:128-159)
      if (v == 0 && l4_sum && ing_sum16(tX + lseed) != 0) v = kErrBadCRC;
    }
    if (live && p == 0) verdict[f] = (uint8_t)v;
  }
}

hipError_t launch_ingress_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t flags,
                                 uint8_t* verdict, int num_cus, hipStream_t stream, const uint32_t* seg_len,
                                 uint32_t trim, const RxFilter* filter, uint32_t* gate, uint32_t epoch,
                                 uint64_t short_mean) {
  RxFilter filt{};
  if (filter) filt = *filter;
  if (n == 0) return hipSuccess;
  const uint64_t frames_per_block = (kIngBlock / 64) * 4;
  uint64_t grid = (n + frames_per_block - 1) / frames_per_block;
  // 128 workgroups per CU (2 passes of 16 frames each at 1 M frames): 0.2594 ms against
  // 0.272 for 32, 0.2645 for 256 (profiles/r1h_grid_sweep.txt).
#ifdef LNX_RESEARCH
  // research library: LNX_PROF_INGRESS_WG_PER_CU overrides it;
  // LNX_PROF_INGRESS_UNROLL=8|16|24 selects the dword-lane form with that
  // batch depth (24 = the r1g product)
  static const uint64_t wg_per_cu = [] {
    const char* e = getenv("LNX_PROF_INGRESS_WG_PER_CU");
    const int v = e ? atoi(e) : 0;
    return (uint64_t)(v > 0 ? v : 128);
  }();
  const uint64_t cap = (uint64_t)num_cus * wg_per_cu;
  if (grid > cap) grid = cap;
  static const int unr = [] {
    const char* e = getenv("LNX_PROF_INGRESS_UNROLL");
    return e ? atoi(e) : 0;
  }();
  if (unr == 8)
    hipLaunchKernelGGL((ingress_verify_kernel<8, false>), dim3((unsigned)grid), dim3(kIngBlock), 0, stream, bytes,
                       off, n, flags, verdict, seg_len, trim, filt, gate, epoch, short_mean);
  else if (unr == 16)
    hipLaunchKernelGGL((ingress_verify_kernel<16, false>), dim3((unsigned)grid), dim3(kIngBlock), 0, stream, bytes,
                       off, n, flags, verdict, seg_len, trim, filt, gate, epoch, short_mean);
  else if (unr == kIngUnroll)
    hipLaunchKernelGGL((ingress_verify_kernel<kIngUnroll, false>), dim3((unsigned)grid), dim3(kIngBlock), 0, stream, bytes,
                       off, n, flags, verdict, seg_len, trim, filt, gate, epoch, short_mean);
  else
#else
  const uint64_t cap = (uint64_t)num_cus * 128;
  if (grid > cap) grid = cap;
#endif
  if (filt.on)
    hipLaunchKernelGGL((ingress_verify_kernel<kIngUnrollQ, true>), dim3((unsigned)grid), dim3(kIngBlock), 0, stream,
                       bytes, off, n, flags, verdict, seg_len, trim, filt, gate, epoch, short_mean);
  else
    hipLaunchKernelGGL((ingress_verify_kernel<kIngUnrollQ, true, false, false>), dim3((unsigned)grid),
                       dim3(kIngBlock), 0, stream, bytes, off, n, flags, verdict, seg_len, trim, filt, gate, epoch, short_mean);
  return hipGetLastError();
}

// lnx_tx_checksum_batch's choice (0.57 against 0.75 ms on 4 M x 128 B, 2.44
// against 2.87 on the Zipf mix for tx_finish's checksum step; the generate
// rows win from ~900 B, tools/prof/ingress_vs_rv.py): the mean of 64 lengths
// sampled across the batch (both kernels give the same bytes and status: the
// sample only picks the faster).  One wave, so that the 32 K workgroups of
// the generate rows read one word instead of 64 scattered lengths each (that
// form cost 0.09 ms on 4 M x 1500 B: 8 M requests)
__global__ void __launch_bounds__(64) tx_gate_probe_kernel(const uint32_t* __restrict__ len, uint64_t n, uint64_t short_mean,
                                                    uint32_t* __restrict__ gate, uint32_t epoch) {
  const uint64_t i = ((uint64_t)threadIdx.x * n) >> 6;
  uint32_t l = len[i];
#pragma unroll
  for (int sft = 1; sft < 64; sft <<= 1) l += (uint32_t)__shfl_xor((int)l, sft);
  if (threadIdx.x == 0 && (uint64_t)l < 64u * short_mean) *gate = epoch;  // (64 lengths < 2^25: no wrap)
}

// Batched transmit checksum generate over ring slots: frame i =
// bytes[start[i] : start[i] + len[i]] (segment mode, trim 0), status[i] as
// lnx_tx_checksum_batch documents.
hipError_t launch_tx_checksum(uint8_t* bytes, const uint64_t* start, const uint32_t* len, uint64_t n,
                              uint8_t* status, int num_cus, hipStream_t stream, uint32_t* gate, uint32_t epoch,
                              uint64_t short_mean) {
  if (n == 0) return hipSuccess;
  const uint64_t frames_per_block = (kIngBlock / 64) * 4;
  uint64_t grid = (n + frames_per_block - 1) / frames_per_block;
  const uint64_t cap = (uint64_t)num_cus * 128;
  if (grid > cap) grid = cap;
  if (gate) hipLaunchKernelGGL(tx_gate_probe_kernel, dim3(1), dim3(64), 0, stream, len, n, short_mean, gate, epoch);
  hipLaunchKernelGGL((ingress_verify_kernel<kIngUnrollQ, true, true>), dim3((unsigned)grid), dim3(kIngBlock), 0,
                     stream, bytes, start, n, 0u, status, len, 0u, RxFilter{}, gate, epoch, short_mean);
  return hipGetLastError();
}

}  // namespace lnx
