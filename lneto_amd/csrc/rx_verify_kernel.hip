// rx_verify_kernel.hip — lneto's whole receive check in ONE pass over each
// frame, gfx950 (round 5): the FCS residue test
// (lnx_fcs_verify_batch) and the checksum-stage verdict
// (lnx_ingress_verify_batch_filtered, §8(f).2: StackEthernet.Demux,
// internet/stack-ethernet.go:139-168, then demux4 / demux6,
// internet/stack-ip4.go:100-167, internet/stack-ip6.go:86-138) from the same
// loads.  Two kernels read every frame from HBM twice (0.247 + 0.248 ms on
// 1 M x 1500 B); this one reads it once.
//
// Layout: the ingress kernel's qword rows (ingress_kernel.hip): one 16-lane
// row per frame, four frames per wave, lane p holding qwords qstart + p + 16u
// of the frame's 8-byte-aligned base (u < 12 per batch: 1536 bytes per row),
// the header fields gathered from the row's lanes by ds_bpermute, the sums by
// v_dot2 on the loaded qwords.  The CRC rides on the same qwords as an
// interleaved fold: lane p owns the 8-byte chunks p, p + 16, p + 32, ... of a
// window that starts 16 qwords before qstart (one extra load per lane, the
// "pre" qword, brings in the frame's first bytes: the MACs the ingress rows
// never load), and folds one chunk per 128-byte line:
//   r <- Z_128(r ^ w0) ^ Z_124(w1)
// (eight byte lookups in lane-private slicing tables, the staged kernel's
// 8-column layout).  After the row's NL lines, lane p's register sits 8p bytes
// past the window end W; the frame's register is
//   R = Z_{-b}( XOR_p Z_{-8(p + a)}(r_p) ),  W - Ltot = 8a + b  (b < 8, a <= 16),
// the first shift by the lane's own nibble tables F_{p+a}, the row XOR by DPP,
// the last by one of eight nibble tables.  The frame's first four bytes carry
// the CRC init (XOR 0xFF), bytes before the frame and past its end are masked
// to zero; FCS ok = Ltot >= 4 and ~R == the CRC-32 residue.
#include <hip/hip_runtime.h>
#include <cstdint>
#include "rx_filter.hpp"

namespace lnx {

namespace {

constexpr int kRvBlock = 1024;
constexpr int kRvUnroll = 12;  // qwords per lane per batch (1536 bytes per row, as the ingress kernel)
constexpr uint32_t kErrPacketDrop = 2, kErrBadCRC = 3, kErrInvalidField = 14, kErrInvalidLengthField = 15,
                   kErrTruncatedFrame = 18;
constexpr uint32_t kVerifyEvilBit = 1, kVerifyIcmp = 2;
// LDS (bytes): the slicing tables T_k (k < 4: Z_{128}(e << 8k); 4 + k: Z_{124}(e << 8k)) expanded into
// 8 bank columns (e << 8 | k << 5 | c << 2), then F_q = Z_{-8q} (q < 32) and B_b = Z_{-b} (b < 8) as
// nibble tables, entry (t, i, v) at 128 t + 16 i + v dwords
constexpr uint32_t kRvT = 0, kRvF = 65536, kRvB = kRvF + 32 * 512, kRvBytes = kRvB + 8 * 512;
// the compact image (api.cpp build_rx_image): T_k[e] at 256 k + e, then F, then B (dwords)
constexpr uint32_t kRvImgF = 2048;  // (then B at kRvImgF + 32 * 128; 2048 + 40 * 128 dwords in all)

__device__ __forceinline__ uint32_t rv_lds(const char* lds, uint32_t a) {
  return *reinterpret_cast<const uint32_t*>(lds + a);
}
struct RvLane {
  uint32_t base[8], sel[4];
  __device__ explicit RvLane(uint32_t lane) {
    const uint32_t g = (lane >> 3) & 3u, c = lane & 7u;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t k = (i + g) & 3u;
      base[i] = (k << 5) | (c << 2);
      base[4 + i] = ((4u + k) << 5) | (c << 2);
      sel[i] = 0x0c020400u + (k << 8);
    }
  }
};
// one 8-byte chunk and the 120 bytes of the other lanes: Z_128(v0) ^ Z_124(v1)
__device__ __forceinline__ uint32_t rv_unit(const char* lds, uint32_t v0, uint32_t v1, const RvLane& z) {
  uint32_t y[8];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) y[4 + i] = rv_lds(lds, kRvT + __builtin_amdgcn_perm(v1, z.base[4 + i], z.sel[i]));
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) y[i] = rv_lds(lds, kRvT + __builtin_amdgcn_perm(v0, z.base[i], z.sel[i]));
  const uint32_t t = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(y[4], y[5], y[6], 0x96), y[7], y[0], 0x96);
  return __builtin_amdgcn_bitop3_b32(t, y[1], y[2], 0x96) ^ y[3];
}
// a nibble-table map (table at byte address t)
__device__ __forceinline__ uint32_t rv_nib(const char* lds, uint32_t t, uint32_t v) {
  uint32_t a = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) a ^= rv_lds(lds, t + 64u * i + (__builtin_amdgcn_ubfe(v, 4 * i, 4) << 2));
  return a;
}
__device__ __forceinline__ uint32_t rv_row_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return v;
}
__device__ __forceinline__ uint32_t rv_row_add(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
  return v;
}
__device__ __forceinline__ bool rv_proto_bit(const uint32_t (&m)[8], uint32_t proto) {
  const uint32_t w = proto >> 5;
  const uint32_t word = w == 0 ? m[0] : w == 1 ? m[1] : w == 2 ? m[2] : w == 3 ? m[3] : w == 4 ? m[4]
                        : w == 5 ? m[5] : w == 6 ? m[6] : m[7];
  return (word >> (proto & 31u)) & 1u;
}
__device__ __forceinline__ uint32_t rv_keep_from(int32_t lo) {
  lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
  return (uint32_t)(0xFFFFFFFFull << (8 * lo));
}
// byte mask of the frame offsets [a, b) inside the word whose byte 0 is at o0
__device__ __forceinline__ uint32_t rv_range(int32_t o0, int32_t a, int32_t b) {
  return rv_keep_from(a - o0) & ~rv_keep_from(b - o0);
}
__device__ __forceinline__ uint16_t rv_sum16(uint32_t sum) {  // crc.go:17-21
  sum = (sum & 0xffffu) + (sum >> 16);
  return (uint16_t)~(uint16_t)(sum + (sum >> 16));
}
__device__ __forceinline__ uint32_t rv_dot2(uint32_t w, uint32_t acc) {
  typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
  const u16x2 ones = {1, 1};
  return __builtin_amdgcn_udot2(__builtin_bit_cast(u16x2, w), ones, acc, false);
}

}  // namespace

// frame f = bytes[off[f] : off[f+1]] (offsets mode) or bytes[off[f] :
// off[f] + seg_len[f]] (segment mode: the receive ring's whole slots); the
// last `trim` bytes are the FCS (trim 4) or none (LNX_RX_NO_FCS: trim 0, no
// CRC, ok = 1).  ok[f] = the FCS test, verdict[f] = the verdict of the frame
// without its FCS, as lnx_ingress_verify_batch_filtered.
template <bool CRC, bool FILT>
__global__ void __launch_bounds__(kRvBlock)
rx_verify_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t n, uint32_t flags,
                 uint8_t* __restrict__ okv, uint8_t* __restrict__ verdict, const uint32_t* __restrict__ seg_len,
                 const uint32_t* __restrict__ image, RxFilter filt) {
  __shared__ __attribute__((aligned(16))) char lds[CRC ? kRvBytes : 16];
  if constexpr (CRC) {
    const uint32_t t = threadIdx.x;
    for (uint32_t vi = t; vi < 2048u; vi += kRvBlock) {
      const uint32_t v = image[vi];
      uint4* row = reinterpret_cast<uint4*>(lds + kRvT + ((vi & 255u) << 8) + ((vi >> 8) << 5));
      const uint4 v4 = {v, v, v, v};
      row[0] = v4;
      row[1] = v4;
    }
    for (uint32_t i = t; i < 40u * 128u; i += kRvBlock) reinterpret_cast<uint32_t*>(lds + kRvF)[i] = image[kRvImgF + i];
    __syncthreads();
  }
  const uint32_t trim = CRC ? 4u : 0u;
  const uint32_t lane = threadIdx.x & 63u, p = lane & 15u, row = lane >> 4;
  const RvLane z(lane);
  const uint64_t nwaves = (uint64_t)gridDim.x * (kRvBlock / 64);
  for (uint64_t qg = (uint64_t)blockIdx.x * (kRvBlock / 64) + (threadIdx.x >> 6); qg * 4 < n; qg += nwaves) {
    const uint64_t f = qg * 4 + row;
    const bool live = f < n;
    const uint64_t s = live ? off[f] : 0;
    const uint32_t sl = live && seg_len ? seg_len[f] : 0u;
    const uint64_t e1 = live && !seg_len ? off[f + 1] : 0;
    const uint64_t et64 = !live ? 0 : (seg_len ? s + sl : (e1 > s ? e1 : s));
    const uint64_t lt64 = et64 - s;  // the whole frame, FCS included
    const uint32_t Lt = lt64 < 0x7FFFFFFFull ? (uint32_t)lt64 : 0x7FFFFFFFu;
    const uint32_t L = Lt > trim ? Lt - trim : 0u;  // the frame the verdict sees
    const uint8_t* fr = bytes + s;
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(fr) & 7u);
    const uint2* base2 = reinterpret_cast<const uint2*>(fr - mis);
    // qword Q of base2 holds frame offsets 8Q - mis .. 8Q - mis + 7
    const int32_t qstart = (int32_t)((12 + mis) >> 3);        // qword holding frame offset 12
    const int32_t QE = (int32_t)((Lt + mis + 7) >> 3);         // qwords touching the frame, FCS included
    const int32_t kstart = (int32_t)((12 + mis) >> 2);         // dword holding frame offset 12

    // ---- first batch (qwords qstart + p + 16 u) and the pre qword (qstart + p - 16)
    uint2 y[kRvUnroll];
#pragma unroll
    for (int u = 0; u < kRvUnroll; ++u) {
      const int32_t q = qstart + (int32_t)p + 16 * u;
      y[u] = q < QE ? base2[q] : make_uint2(0u, 0u);
    }
    const int32_t qpre = qstart + (int32_t)p - 16;
    uint2 yp = make_uint2(0u, 0u);
    if constexpr (CRC) yp = qpre >= 0 && qpre < QE ? base2[qpre] : make_uint2(0u, 0u);

    // dword kstart + kk of this row (kk < 31) from the lane that loaded it
    auto rowword = [&](int32_t kk) -> uint32_t {
      const uint32_t rel = (uint32_t)(kstart - 2 * qstart + kk);
      const int addr = (int)((row * 16u + ((rel >> 1) & 15u)) * 4u);
      const uint32_t a = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)y[0].x);
      const uint32_t b = (uint32_t)__builtin_amdgcn_ds_bpermute(addr, (int)y[0].y);
      return (rel & 1u) ? b : a;
    };
    const uint32_t sh = (12 + mis) & 3u;
    const uint32_t w0 = rowword(0), w1 = rowword(1), w2 = rowword(2), w3 = rowword(3);
    const uint32_t H0 = __builtin_amdgcn_alignbyte(w1, w0, sh);  // frame bytes 12..15
    const uint32_t H1 = __builtin_amdgcn_alignbyte(w2, w1, sh);  // 16..19
    const uint32_t H2 = __builtin_amdgcn_alignbyte(w3, w2, sh);  // 20..23
    auto byt = [](uint32_t w, int i) -> uint32_t { return (w >> (8 * i)) & 0xFFu; };
    auto be = [&](uint32_t w, int i) -> uint32_t { return (byt(w, i) << 8) | byt(w, i + 1); };
    auto field16 = [&](uint32_t o) -> uint32_t {
      const int32_t kk = (int32_t)((o + mis) >> 2) - kstart;
      const uint32_t lo = rowword(kk), hi = rowword(kk + 1);
      const uint32_t v2 = __builtin_amdgcn_alignbyte(hi, lo, (o + mis) & 3u);
      return ((v2 & 0xFFu) << 8) | ((v2 >> 8) & 0xFFu);
    };
    auto field32 = [&](uint32_t o) -> uint32_t {
      const int32_t kk = (int32_t)((o + mis) >> 2) - kstart;
      return __builtin_amdgcn_alignbyte(rowword(kk + 1), rowword(kk), (o + mis) & 3u);
    };

    // ---- header parse (ingress_kernel.hip's, FCS excluded: L bytes)
    uint32_t v = 0, v_udp4 = 0;
    bool hdr_sum = false, l4_sum = false;
    int32_t pa = 0, pb = 0, la = 0, lb = 0;
    uint32_t lseed = 0;
    if (L < 14) {
      v = kErrTruncatedFrame;
    } else {
      const uint32_t et = be(H0, 0);
      bool eth_drop = false, et_handler = true;
      if (FILT && filt.on) {
        // StackEthernet.Demux (internet/stack-ethernet.go:146-152), before ValidateSize; the
        // destination MAC (frame bytes 0..5) from the pre qwords and the first batch
        const uint32_t* w = reinterpret_cast<const uint32_t*>(fr - mis) + (mis >> 2);
        const uint32_t sm = mis & 3u, m0 = w[0], m1 = w[1], m2 = w[2];
        const uint32_t D0 = __builtin_amdgcn_alignbyte(m1, m0, sm), D1 = __builtin_amdgcn_alignbyte(m2, m1, sm) & 0xFFFFu;
        const bool bcast = D0 == 0xFFFFFFFFu && D1 == 0xFFFFu;
        const bool mine = D0 == filt.mac_lo && D1 == filt.mac_hi;
        eth_drop = !bcast && !mine && !(filt.eth_mc && (D0 & 1u));
        et_handler = false;  // handlers.demuxByProto(etype) (stack-ethernet.go:158-161)
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
            const uint32_t dst = field32(30);  // demux4's destination check (stack-ip4.go:108-119)
            const bool mc = (dst & 0xF0u) == 0xE0u, bc = dst == 0xFFFFFFFFu;
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
            if (FILT && filt.on && !rv_proto_bit(filt.p4, proto)) {
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
                  l4_sum = true;
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
            const uint32_t d0 = field32(38), d1 = field32(42), d2 = field32(46), d3 = field32(50);
            const bool mine = d0 == filt.ip6[0] && d1 == filt.ip6[1] && d2 == filt.ip6[2] && d3 == filt.ip6[3];
            if (!mine && !(filt.ip6_mc && (d0 & 0xFFu) == 0xFFu)) v = kErrPacketDrop;
          }
          if (v != 0) {
          } else if (pl + 40 > M) {
            v = kErrInvalidLengthField;
          } else if (FILT && filt.on && !rv_proto_bit(filt.p6, proto)) {
            v = kErrPacketDrop;
          } else if (proto == 6 || proto == 17 || (proto == 58 && (flags & kVerifyIcmp))) {
            if (proto == 58 && pl < 8) v = kErrTruncatedFrame;
            if (proto == 17) {
              if (pl < 8) v = kErrTruncatedFrame;
              else if (field16(58) < 8) v = kErrInvalidLengthField;
              else if (field16(58) > pl) v = kErrTruncatedFrame;
            }
            if (v == 0) {
              l4_sum = true;
              pa = 22, pb = 54, la = 54, lb = 54 + pl;
              lseed = pl + proto;
            }
          }
        }
      }
    }

    // ---- one pass over the frame's qwords: the sums (qwords below qend) and the CRC (every qword)
    const bool any_sum = hdr_sum || l4_sum;
    const int32_t end = l4_sum ? lb : (hdr_sum ? 34 : 0);
    const int32_t kend = any_sum ? (end + (int32_t)mis + 3) >> 2 : 0;
    const int32_t qend = (kend + 1) >> 1;
    const int32_t ha = hdr_sum ? 14 : 0, hb = hdr_sum ? 34 : 0;
    uint32_t hS = 0, tS = 0;
    // CRC: lines (16 qwords) from qword qstart - 16; the row needs NL of them
    const int32_t q0 = qstart - 16;
    const int32_t NL = (QE - q0 + 15) >> 4;  // >= 1
    const int32_t lastq = QE - 1;
    // the last qword's bytes at or past Lt are not the frame's
    const int32_t olast = 8 * lastq - (int32_t)mis;
    const uint32_t mlast0 = ~rv_keep_from((int32_t)Lt - olast), mlast1 = ~rv_keep_from((int32_t)Lt - olast - 4);
    uint32_t r = 0;
    if constexpr (CRC) {
      // the pre qword (line 0): bytes before the frame masked, the CRC init on frame bytes 0..3
      const int32_t o0 = 8 * qpre - (int32_t)mis;
      const int32_t ie = (int32_t)(Lt < 4 ? Lt : 4u);
      const uint32_t a0 = yp.x & rv_range(o0, 0, (int32_t)Lt), a1 = yp.y & rv_range(o0 + 4, 0, (int32_t)Lt);
      const uint32_t x0 = a0 ^ rv_range(o0, 0, ie), x1 = a1 ^ rv_range(o0 + 4, 0, ie);
      r = rv_unit(lds, x0, x1, z);  // (NL >= 1: line 0 is always the row's)
    }
    // a wave-uniform trip count (the most any row of the wave needs), as the ingress kernel
    const int32_t qneed = QE > qend ? QE : qend;
    int32_t nit = qneed > qstart ? (qneed - qstart + 16 * kRvUnroll - 1) / (16 * kRvUnroll) : 0;
    nit = max(nit, __shfl_xor(nit, 16));
    nit = max(nit, __shfl_xor(nit, 32));
    nit = __builtin_amdgcn_readfirstlane(nit);
    uint2 yl = make_uint2(0u, 0u);  // the sum's last qword, on the lane that holds it
    for (int32_t it = 0; it < nit; ++it) {
      const int32_t qb = qstart + (int32_t)p + 16 * kRvUnroll * it;
      if (it > 0) {
#pragma unroll
        for (int u = 0; u < kRvUnroll; ++u) {
          const int32_t q = qb + 16 * u;
          y[u] = q < QE ? base2[q] : make_uint2(0u, 0u);
        }
      }
#pragma unroll
      for (int u = 0; u < kRvUnroll; ++u) {
        const int32_t q = qb + 16 * u;
        // sums: qwords below qend only; the first qword of the first batch takes the header /
        // pseudo-header / transport-start masks (every later one lies past offset 126)
        const bool insum = q < qend;
        const uint32_t sx = insum ? y[u].x : 0u, sy = insum ? y[u].y : 0u;
        if (u == 0 && it == 0) {
          const int32_t o0 = 8 * q - (int32_t)mis;
          hS = rv_dot2(sx & rv_range(o0, ha, hb), hS);
          hS = rv_dot2(sy & rv_range(o0 + 4, ha, hb), hS);
          tS = rv_dot2(sx & (rv_range(o0, pa, pb) | rv_range(o0, la, lb)), tS);
          tS = rv_dot2(sy & (rv_range(o0 + 4, pa, pb) | rv_range(o0 + 4, la, lb)), tS);
        } else {
          tS = rv_dot2(sx, rv_dot2(sy, tS));
          const bool isl = q == qend - 1;
          yl.x = isl ? y[u].x : yl.x;
          yl.y = isl ? y[u].y : yl.y;
        }
        if constexpr (CRC) {
          // line 1 + u + kRvUnroll * it of the CRC window
          const bool inl = 1 + u + kRvUnroll * it < NL;
          const bool isl = q == lastq;
          const uint32_t c0 = isl ? y[u].x & mlast0 : y[u].x, c1 = isl ? y[u].y & mlast1 : y[u].y;
          const uint32_t nr = rv_unit(lds, r ^ c0, c1, z);
          r = inl ? nr : r;
        }
      }
    }
    // bytes at or past lb of the sum's last qword (zero unless this lane kept it)
    {
      const int32_t ol = 8 * (qend - 1) - (int32_t)mis;
      const uint32_t j0 = yl.x & rv_keep_from(lb - ol), j1 = yl.y & rv_keep_from(lb - ol - 4);
      tS -= rv_dot2(j0, rv_dot2(j1, 0u));
    }
    hS = rv_row_add(hS), tS = rv_row_add(tS);
    auto conv = [&](uint32_t S) -> uint32_t {  // ingress_kernel.hip: the byte rotation for even bases
      if (mis & 1u) return S;
      uint32_t fo = (S & 0xFFFFu) + (S >> 16);
      fo = (fo & 0xFFFFu) + (fo >> 16);
      return ((fo << 8) | (fo >> 8)) & 0xFFFFu;
    };
    const uint32_t hX = conv(hS), tX = conv(tS);
    if (v == 0 && hdr_sum && rv_sum16(hX) != 0) v = kErrBadCRC;
    if (v == 0) v = v_udp4;  // udp.NewFrame / ValidateSize follow CalculateHeaderCRC (stack-ip4.go:128-159)
    if (v == 0 && l4_sum && rv_sum16(tX + lseed) != 0) v = kErrBadCRC;
    uint32_t okf = 1;
    if constexpr (CRC) {
      // the window end W = 8 (q0 + 16 NL) - mis (frame offset); W - Lt = 8a + b
      const uint32_t pad = (uint32_t)(8 * (q0 + 16 * NL) - (int32_t)mis - (int32_t)Lt);
      const uint32_t a = pad >> 3, b = pad & 7u;
      const uint32_t x = rv_row_xor(rv_nib(lds, kRvF + 512u * (p + a), r));
      const uint32_t R = rv_nib(lds, kRvB + 512u * b, x);
      okf = Lt >= 4 && ~R == 0x2144DF1Cu;
    }
    if (live && p == 0) {
      okv[f] = (uint8_t)okf;
      verdict[f] = (uint8_t)v;
    }
  }
}

hipError_t launch_rx_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t flags, bool fcs,
                            uint8_t* ok, uint8_t* verdict, const uint32_t* seg_len, const RxFilter* filter,
                            const uint32_t* image, int num_cus, hipStream_t stream) {
  RxFilter filt{};
  if (filter) filt = *filter;
  if (n == 0) return hipSuccess;
  uint64_t grid = (n + (kRvBlock / 64) * 4 - 1) / ((kRvBlock / 64) * 4);
  if (grid > (uint64_t)num_cus) grid = (uint64_t)num_cus;
#define LNX_RV(C, F)                                                                                       \
  hipLaunchKernelGGL((rx_verify_kernel<C, F>), dim3((unsigned)grid), dim3(kRvBlock), 0, stream, bytes, off, n, \
                     flags, ok, verdict, seg_len, image, filt)
  if (fcs) {
    if (filt.on) LNX_RV(true, true); else LNX_RV(true, false);
  } else {
    if (filt.on) LNX_RV(false, true); else LNX_RV(false, false);
  }
#undef LNX_RV
  return hipGetLastError();
}

}  // namespace lnx
