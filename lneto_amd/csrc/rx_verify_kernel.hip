// rx_verify_kernel.hip — lneto's whole receive check in ONE pass over each
// frame, gfx950 (round 5): the FCS residue test
// (lnx_fcs_verify_batch) and the checksum-stage verdict
// (lnx_ingress_verify_batch_filtered, §8(f).2: StackEthernet.Demux,
// internet/stack-ethernet.go:139-168, then demux4 / demux6,
// internet/stack-ip4.go:100-167, internet/stack-ip6.go:86-138) from the same
// loads.  Two kernels read every frame from HBM twice (0.247 + 0.248 ms on
// 1 M x 1500 B); this one reads it once.
//
// The CRC is an interleaved fold over one 16-lane row per frame: lane p owns
// the 8-byte chunks p, p + 16, p + 32, ... of a qword window that starts at
// the qword holding the frame's first byte, and folds one chunk per 128-byte
// line:
//   r <- Z_128(r ^ w0) ^ Z_124(w1)
// (eight byte lookups in lane-private slicing tables, the staged kernel's
// 8-column layout).  After the row's NL lines, lane p's register sits 8p bytes
// past the window end W; the frame's register is
//   R = Z_{-b}( XOR_p Z_{-8(p + a)}(r_p) ),  W - Ltot = 8a + b  (b < 8, a < 16),
// the first shift by the lane's own nibble tables F_{p+a}, the row XOR by DPP,
// the last by one of eight nibble tables.  The frame's first four bytes carry
// the CRC init (XOR 0xFF); FCS ok = Ltot >= 4 and ~R == the CRC-32 residue.
// The verdicts come from a second phase with one lane per frame (below).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>
#include "rx_filter.hpp"

namespace lnx {

namespace {

#ifndef LNX_TX_BLOCK
#define LNX_TX_BLOCK 1024
#endif
constexpr int kRvBlock = 1024;
// Round 5: the transmit kernel wanted more registers than 16 waves of 128
// VGPRs give it (hipcc spilled 120-130 bytes per lane inside the row passes:
// traffic 1.57 x, 0.71 ms on 1 M x 1500 B), so it ran 12 waves of 168 VGPRs
// (1.035 x, 0.48 -> 0.434 ms; profiles/r5v_*).  Round 6: with 4 qwords of the
// next pass loaded ahead (kTxPf, was 8) and 48-frame groups (kTxGroup, was
// 64: the 16 waves' staging fits LDS beside the tables) it takes 126 VGPRs
// with no scratch, 16 waves: 0.436 -> 0.416 ms on 1 M x 1500 B, 4.50 -> 4.14
// ms on the 16 M Zipf mix (tools/prof/lib_ab.py).  Over host
// memory (the ring's zero-copy egress, PCIe-bound) 12 and 16 waves measured
// alike: 17.4-24.5 GiB/s on the Zipf mix (tools/prof/SESSIONS.md r5w, r5y).
constexpr int kTxBlock = LNX_TX_BLOCK;
#ifndef LNX_TX_BLOCK_HOST
#define LNX_TX_BLOCK_HOST 768
#endif
constexpr int kTxBlockHost = LNX_TX_BLOCK_HOST;
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

// A qword load through the global address space: the pointer is a select of
// a frame address and g_rv_zero, which hipcc would otherwise load with a FLAT
// instruction -- counted in lgkmcnt too, so every LDS wait of the fold would
// wait for the frame loads in flight (the prefetch included).
__device__ __forceinline__ uint2 rv_ld(const uint2* p) {
  const uint64_t v = *(const __attribute__((address_space(1))) uint64_t*)p;
  return make_uint2((uint32_t)v, (uint32_t)(v >> 32));
}
__device__ __forceinline__ uint32_t rv_ld32(const uint32_t* p) {
  return *(const __attribute__((address_space(1))) uint32_t*)p;
}
__device__ __forceinline__ uint32_t rv_lds(const char* lds, uint32_t a) {
  return *reinterpret_cast<const uint32_t*>(lds + a);
}
// the lane's table columns: T_k's entry for byte e of the chunk at e << 8 | k << 5 | c << 2
// (k rotated by the lane's 8-lane group, c its lane in the group); T_{4+k} is 128 bytes on
// (an address bit below e's: the lookup's immediate offset, no registers of its own)
struct RvLane {
  uint32_t base[4], sel[4];
  __device__ explicit RvLane(uint32_t lane) {
    const uint32_t g = (lane >> 3) & 3u, c = lane & 7u;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t k = (i + g) & 3u;
      base[i] = (k << 5) | (c << 2);
      sel[i] = 0x0c020400u + (k << 8);
    }
  }
};
// one 8-byte chunk and the 120 bytes of the other lanes: Z_128(v0) ^ Z_124(v1)
__device__ __forceinline__ uint32_t rv_unit(const char* lds, uint32_t v0, uint32_t v1, const RvLane& z) {
  uint32_t y[8];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) y[4 + i] = rv_lds(lds, kRvT + 128u + __builtin_amdgcn_perm(v1, z.base[i], z.sel[i]));
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) y[i] = rv_lds(lds, kRvT + __builtin_amdgcn_perm(v0, z.base[i], z.sel[i]));
  const uint32_t t = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(y[4], y[5], y[6], 0x96), y[7], y[0], 0x96);
  return __builtin_amdgcn_bitop3_b32(t, y[1], y[2], 0x96) ^ y[3];
}
// a nibble-table map (table at byte address t, a multiple of 64).  The entry's
// byte address is (v's nibble i, shifted into place and masked) OR the table's
// base, one v_and_or_b32 after the shift, and the 64 i (F: 2048 i) a ds_read
// offset: 2 VALU per nibble instead of 3
__device__ __forceinline__ uint32_t rv_nib(const char* lds, uint32_t t, uint32_t v) {
  uint32_t a = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t sh = i == 0 ? v << 2 : v >> (4 * i - 2);
    a ^= *reinterpret_cast<const uint32_t*>(lds + ((sh & 0x3Cu) | t) + 64u * i);
  }
  return a;
}
// the same for F_q in its banked layout (entry e of table q at dword 32 e + q)
__device__ __forceinline__ uint32_t rv_nib_f(const char* lds, uint32_t q, uint32_t v) {
  const uint32_t t = kRvF + 4u * q;  // (bits 2..6 and 16: clear of the entry's bits 7..10)
  uint32_t a = 0;
#pragma unroll
  for (uint32_t i = 0; i < 8; ++i) {
    const uint32_t sh = i == 0 ? v << 7 : i == 1 ? v << 3 : v >> (4 * i - 7);
    a ^= *reinterpret_cast<const uint32_t*>(lds + ((sh & 0x780u) | t) + 2048u * i);
  }
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
//
// A wave takes kRvGroup consecutive frames (a group) in two phases:
//  A. data: kRvGroup / 4 row passes of four frames (one 16-lane row each).
//     Lane p folds qwords p, p + 16, ... of the frame's qword window into its
//     CRC register (the first line masked to the frame, the init on its first
//     four bytes; the later lines unmasked, the last qword's bytes past the
//     frame taken out again by the lane holding it) and adds every qword into
//     a raw sum (no per-qword masks: qwords past the frame load as zero); the
//     lanes holding the FCS / the bytes past the frame take them out, so
//     S = the LE 16-bit sum of the frame's bytes [14, L).  The row's FCS test,
//     S and the frame's first kRvHead qwords go to LDS.
//  B. verdicts: one lane per frame parses the headers from its staged qwords,
//     takes the header, pseudo-header and head-of-segment sums there, and the
//     segment's sum as S minus the bytes before it minus the bytes from its
//     end to L (runt padding, trailing data: staged when short, else summed
//     from memory by the whole wave).
// Every qword load reads inside the frame or a zero qword (g_rv_zero), so no
// load crosses the frame's qwords and none is under a branch; the offsets of
// a group are loaded once, by the lane of each frame.
// the most frames per wave and group (LDS: tables + the waves' group staging
// <= 160 KiB): 56 for the receive kernel (16 waves: 154 KiB), 48 for the
// transmit kernel (16 waves: 152 KiB; 64 at its round-5 12 waves); the
// launchers pick the size per batch (balanced_group): on 1 M frames fixed
// sizes measured 0.331 / 0.310 / 0.322 / 0.340 ms (48 / 52 / 56 / 60,
// receive) and 0.462 / 0.467 / 0.435 / 0.454 ms (48 / 56 / 60 / 64, transmit
// at 12 waves) -- the rounds of groups times the group size
// (tools/prof/SESSIONS.md r6r, r6u)
constexpr uint32_t kRvGroup = 56;
#ifndef LNX_TX_GROUP
#define LNX_TX_GROUP 48
#endif
constexpr uint32_t kTxGroup = LNX_TX_GROUP;
constexpr uint32_t kRvHead = 9;    // staged qwords per frame: frame bytes [0, 72 - mis) >= [0, 65)
constexpr int kRvPf = 8;           // qwords per lane of the next pass loaded ahead (host memory)
#ifndef LNX_TX_PF
#define LNX_TX_PF 4
#endif
constexpr int kTxPf = LNX_TX_PF;   // ... (the transmit kernel over device memory)
#ifndef LNX_RV_PF_RX
#define LNX_RV_PF_RX 12
#endif
constexpr int kRvPfRx = LNX_RV_PF_RX;  // ... (receive: the whole next pass)
__device__ uint2 g_rv_zero[2];

typedef uint32_t rv_u4 __attribute__((ext_vector_type(4)));
#ifndef LNX_RV_R8_LINES
#define LNX_RV_R8_LINES 10
#endif
// lines of the 8-lane rows' window: frames of length class < kR8Lines (at
// most 128 (kR8Lines - 1) bytes, so a window of <= kR8Lines lines) take them.
// 10 (frames to 1152 B): against 4, 0.59 against 0.67 ms on 4 M x 768 B,
// 0.76 against 0.79 at 1024 B, the Zipf mix 1-3 % faster; 13 (MTU frames
// too) made the 1 M x 1500 B receive check 13 % slower (profiles/r8f)
constexpr int kR8Lines = LNX_RV_R8_LINES;
__device__ __attribute__((aligned(16))) uint32_t g_rv_zero4[4];
__device__ __forceinline__ rv_u4 rv_ld4(const rv_u4* p) {
  return *(const __attribute__((address_space(1))) rv_u4*)p;
}
// the XOR / sum over an 8-lane row (two quad steps, then the other quad of the half row)
__device__ __forceinline__ uint32_t rv_row8_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);  // row_half_mirror
  return v;
}
__device__ __forceinline__ uint32_t rv_row8_add(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x141, 0xF, 0xF, false);
  return v;
}

// Phase A for the group's short frames (round 6): positions [0, n8) of the
// passes' order, every frame there at most 128 (kR8Lines - 1) bytes (its
// window at most kR8Lines lines), in passes of EIGHT 8-lane rows.  Lane p of a
// row loads the 16-byte blocks p, p + 8, p + 16, p + 24 of a window that
// starts at the 16-byte block holding the frame's first byte (one dwordx4 a
// line: a row still reads a whole 128-byte line per instruction, and a block
// that holds a frame byte never leaves its page), i.e. qwords 2p and 2p + 1 of
// each line: lane p plays the lanes 2p and 2p + 1 of the 16-lane rows, with a
// CRC register each, the same fold, masks and end corrections (the window's
// misalignment m16 < 16 in place of mis < 8), the two registers shifted by
// F_{2p+a} and F_{2p+1+a} and XORed over the row.  The per-pass work of a row
// (the frame's start and length, its masks, the shifts) then serves eight
// frames a wave instead of four.
template <bool CRC, bool TX>
__device__ __forceinline__ void rv_rows8(const char* lds, uint2* res, uint2* head, const RvLane& z,
                                         const uint8_t* bytes, uint64_t sk, uint32_t Ltk, uint32_t n8, uint32_t trim,
                                         uint32_t capacity) {
  // (the lane index opaque here: values derived from it are computed where
  // they are used, not hoisted to the kernel's entry and held, or spilled,
  // through the 16-lane passes; this function is the receive kernel's
  // register peak)
  uint32_t lane = threadIdx.x & 63u;
  asm volatile("" : "+v"(lane));
  const uint32_t p = lane & 7u, row = lane >> 3;
  const rv_u4* zero4 = reinterpret_cast<const rv_u4*>(g_rv_zero4);
  auto wave_max = [&](int32_t x) -> int32_t {
    x = max(x, __shfl_xor(x, 8));
    x = max(x, __shfl_xor(x, 16));
    x = max(x, __shfl_xor(x, 32));
    return __builtin_amdgcn_readfirstlane(x);
  };
  auto row_frame = [&](uint32_t j, const uint8_t*& fr, uint32_t& Lt) {
    const uint32_t k = 8u * j + row;
    const uint32_t slo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)(uint32_t)sk);
    const uint32_t shi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)(uint32_t)(sk >> 32));
    Lt = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)Ltk);
    fr = bytes + (((uint64_t)shi << 32) | slo);
  };
  // a pass's four lines: the blocks some byte of the row's frame lies in (the
  // rest zero, without a load), the second qword of a block past the frame's
  // last qword zeroed (the 16-lane rows never load it)
  // (the next pass's first two lines are loaded a pass ahead, the other two
  // in the pass: four ahead spilled the receive kernel's registers)
  constexpr int PQ = 2;
  rv_u4 pf[PQ];
  const uint8_t* frn = bytes;
  uint32_t Ltn = 0;
  auto blocks = [&](const uint8_t* f, uint32_t Lt, const rv_u4*& b4, int32_t& QB, int32_t& um) {
    const uint32_t m16 = (uint32_t)(reinterpret_cast<uintptr_t>(f) & 15u);
    b4 = reinterpret_cast<const rv_u4*>(f - m16);
    QB = (int32_t)((Lt + m16 + 15u) >> 4);
    um = (wave_max(QB) + 7) >> 3;
  };
  auto prefetch = [&](uint32_t jn) {
    if (8u * jn >= n8) return;  // (wave-uniform)
    row_frame(jn, frn, Ltn);
    const rv_u4* b4;
    int32_t QB, um;
    blocks(frn, Ltn, b4, QB, um);
#pragma unroll
    for (int u = 0; u < PQ; ++u) {
      const int32_t b = (int32_t)p + 8 * u;
      pf[u] = u < um ? rv_ld4(b < QB ? b4 + b : zero4) : rv_u4{0u, 0u, 0u, 0u};
    }
  };
  prefetch(0);
  for (uint32_t j = 0; 8u * j < n8; ++j) {
    // (the row index made opaque in every pass: hoisted out of the loops, the
    // head and result addresses derived from it were spilled)
    uint32_t rw = row;
    asm volatile("" : "+v"(rw));
    const uint32_t k = 8u * j + rw;
    const uint8_t* fr = frn;
    const uint32_t Lt = Ltn;
    rv_u4 y[kR8Lines];
#pragma unroll
    for (int u = 0; u < PQ; ++u) y[u] = pf[u];
    {
      const rv_u4* b4;
      int32_t QB, um;
      blocks(fr, Lt, b4, QB, um);
#pragma unroll
      for (int u = PQ; u < kR8Lines; ++u) {
        const int32_t b = (int32_t)p + 8 * u;
        y[u] = u < um ? rv_ld4(b < QB ? b4 + b : zero4) : rv_u4{0u, 0u, 0u, 0u};
      }
    }
    prefetch(j + 1u);
    const uint32_t Lc = TX && CRC && (Lt < 60u ? 60u : Lt) + 4u <= capacity ? (Lt < 60u ? 60u : Lt) : Lt;
    const uint32_t L = TX ? Lt : (Lt > trim ? Lt - trim : 0u);
    const uint32_t m16 = (uint32_t)(reinterpret_cast<uintptr_t>(fr) & 15u);
    const int32_t QE = (int32_t)((Lt + m16 + 7u) >> 3);  // qwords holding frame bytes (from the 16-byte block)
    const int32_t NL = (int32_t)(((Lc + m16 + 7u) >> 3) + 15u) >> 4;  // lines of the CRC window (<= kR8Lines)
    const int32_t nlw = wave_max(NL);
    uint32_t S = 0, r[2] = {0u, 0u};
    // the frame's first qwords for phase B (from the 8-byte-aligned base it uses)
    const int32_t hsh = m16 >= 8u ? 1 : 0;
#pragma unroll
    for (int v = 0; v < 2; ++v) {
      const int32_t q2 = 2 * (int32_t)p + v - hsh;
      if (q2 >= 0 && q2 < (int32_t)kRvHead)  // (qwords past the frame as zero, as the 16-lane rows stage them)
        head[kRvHead * k + q2] = 2 * (int32_t)p + v >= QE ? make_uint2(0u, 0u)
                                 : v ? make_uint2(y[0][2], y[0][3]) : make_uint2(y[0][0], y[0][1]);
    }
    // every qword masked as it is folded (the sum to [14, L), the CRC to
    // [0, Lt) with the init on [0, 4)), so no end correction follows: the
    // 16-lane rows' reload of the end qwords and their junk unit kept more
    // registers live than the kernel has
#pragma unroll
    for (int u = 0; u < kR8Lines; ++u) {
      if (u > 0 && u >= nlw) break;  // (wave-uniform: no row's window reaches line u)
#pragma unroll
      for (int v = 0; v < 2; ++v) {
        const int32_t o = 8 * (2 * (int32_t)p + v + 16 * u) - (int32_t)m16;  // the qword's first frame offset
        const uint32_t c0 = y[u][2 * v], c1 = y[u][2 * v + 1];
        if (u == 0) {
          S = rv_dot2(c0 & rv_range(o, 14, (int32_t)L), rv_dot2(c1 & rv_range(o + 4, 14, (int32_t)L), S));
        } else {
          S = rv_dot2(c0 & ~rv_keep_from((int32_t)L - o), rv_dot2(c1 & ~rv_keep_from((int32_t)L - o - 4), S));
        }
        if constexpr (CRC) {
          const int32_t ie = (int32_t)(Lc < 4 ? Lc : 4u);
          uint32_t d0, d1;
          if (u == 0) {
            d0 = (c0 & rv_range(o, 0, (int32_t)Lt)) ^ rv_range(o, 0, ie);
            d1 = (c1 & rv_range(o + 4, 0, (int32_t)Lt)) ^ rv_range(o + 4, 0, ie);
          } else {
            d0 = c0 & ~rv_keep_from((int32_t)Lt - o);
            d1 = c1 & ~rv_keep_from((int32_t)Lt - o - 4);
          }
          const uint32_t nr = rv_unit(lds, r[v] ^ d0, d1, z);
          r[v] = u < NL ? nr : r[v];
        }
      }
    }
    uint32_t okf = 1;
    if constexpr (CRC) {
      // the window ends W = 128 NL - m16 past the frame start; W - Lc = 8a + b
      const uint32_t pad = (uint32_t)(128 * NL - (int32_t)m16 - (int32_t)Lc);
      const uint32_t a = pad >> 3, b = pad & 7u;
      const uint32_t x = rv_row8_xor(rv_nib_f(lds, 2u * p + a, r[0]) ^ rv_nib_f(lds, 2u * p + 1u + a, r[1]));
      const uint32_t R = rv_nib(lds, kRvB + 512u * b, x);
      okf = TX ? R : (uint32_t)(Lt >= 4 && ~R == 0x2144DF1Cu);
    }
    S = rv_row8_add(S);
    if (p == 0) res[k] = make_uint2(okf, S);
  }
}

// Phase A of a group (see above): kRvGroup / 4 passes of four 16-lane rows.
// Lane k < kRvGroup holds its frame's start sk and length Ltk.  Per frame the
// rows load the bytes [0, Ld), fold the CRC over them followed by zeros up to
// Lc >= Ld, and sum the LE 16-bit words of [14, Ls):
//   receive (TX = false): Ld = Lc = Ltk, Ls = Ltk - trim; res = (FCS ok, S);
//   transmit (TX = true): Ld = Ls = Ltk, Lc = the length padded to 60 when the
//     FCS is appended (Ltk otherwise); res = (the finished CRC register R of
//     the frame as it is, S).
// The frame's first kRvHead qwords go to head.  HOST (frames in pinned host
// memory, read over PCIe): the qwords past the frame's end are captured as the
// fold passes them instead of loaded again (a second PCIe round trip).
template <bool CRC, bool TX, bool HOST, int PF = kRvPf>
__device__ __forceinline__ uint32_t rv_rows(const char* lds, uint2* res, uint2* head, const RvLane& z,
                                            const uint8_t* bytes, uint64_t sk, uint32_t Ltk, uint32_t nrow,
                                            uint32_t trim, uint32_t capacity) {
  const uint32_t lane = threadIdx.x & 63u, p = lane & 15u, row = lane >> 4;
  const uint2* zero = g_rv_zero;
    // The passes take the group's frames in order of their length class (128-B
    // lines): a pass folds as many units as its longest frame needs, so four
    // frames of like length waste fewer of them on a mixed batch.  A counting
    // sort over the classes (stable; lanes past nrow stay last) gives each
    // lane its position `rank`, and the frames' starts and lengths move there
    // (ds_permute), so the passes below take position k = 4 j + row as
    // before and leave the frame's results at res[rank] / head[rank]: the
    // caller's lane-per-frame phase reads its frame there.  A uniform group
    // (MTU frames) skips the sort (rank = lane), and so do frames in host
    // memory: over PCIe the passes keep address order (the ring's zero-copy
    // receive on the Zipf mix ran 7.10 -> 7.44 ms per 1 M frames sorted).
    uint32_t rank = lane;
    uint32_t n8 = 0;  // positions [0, n8): the 8-lane rows (rv_rows8)
    if constexpr (!HOST) {
      const uint32_t key = lane < nrow ? ((Ltk + 127u) >> 7 < 14u ? (Ltk + 127u) >> 7 : 14u) : 15u;
      n8 = (uint32_t)__builtin_popcountll(__builtin_amdgcn_ballot_w64(key < (uint32_t)kR8Lines)) & ~7u;
      const uint32_t k0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)key);
      if (__builtin_amdgcn_ballot_w64(lane < nrow && key != k0) != 0) {
        uint32_t below = 0;
        uint64_t same = 0;
#pragma unroll 1
        for (uint32_t c = 0; c < 16u; ++c) {
          const uint64_t m = __builtin_amdgcn_ballot_w64(key == c);
          below += key > c ? (uint32_t)__builtin_popcountll(m) : 0u;
          same = key == c ? m : same;
        }
        // (the lanes of `same` below this one by mbcnt: no lane mask held in registers)
        rank = below + __builtin_amdgcn_mbcnt_hi((uint32_t)(same >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)same, 0u));
        const uint32_t slo = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank << 2), (int)(uint32_t)sk);
        const uint32_t shi = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank << 2), (int)(uint32_t)(sk >> 32));
        Ltk = (uint32_t)__builtin_amdgcn_ds_permute((int)(rank << 2), (int)Ltk);
        sk = ((uint64_t)shi << 32) | slo;
      }
    }
    // the short frames (length class < kR8Lines, sorted first) in 8-lane rows, the rest below
    if constexpr (!HOST) {
      if (n8 > 0) rv_rows8<CRC, TX>(lds, res, head, z, bytes, sk, Ltk, n8, trim, capacity);
    }
    // the row's frame of pass j: its start (from the lane that holds it) and length
    auto row_frame = [&](uint32_t j, const uint8_t*& fr, uint32_t& Lt) {
      const uint32_t k = n8 + 4u * j + row;
      const uint32_t slo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)(uint32_t)sk);
      const uint32_t shi = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)(uint32_t)(sk >> 32));
      Lt = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(k << 2), (int)Ltk);
      fr = bytes + (((uint64_t)shi << 32) | slo);
    };
    // the first PQ qwords of a pass's batch 0 are loaded PR passes before
    // (software pipelining: their latency overlaps the previous frames' folds)
    constexpr int PR = 1, PQ = PF;  // (two passes ahead for host memory measured no faster: 33.8 against 35-37 GiB/s)
    uint2 pf[PR][PQ];
    const uint8_t* frn[PR];
    uint32_t Ltn[PR];
    // (a unit whose qwords lie inside all four rows' frames -- the wave's least
    // qword count says so, wave-uniformly -- loads them at the frame's address
    // plus an immediate offset; else each lane selects its qword or the zero
    // qword: 4 VALU per load, 40 per pass of MTU frames saved)
    auto wave_min = [&](int32_t x) -> int32_t {
      x = min(x, __shfl_xor(x, 16));
      x = min(x, __shfl_xor(x, 32));
      return __builtin_amdgcn_readfirstlane(x);
    };
    auto wave_max = [&](int32_t x) -> int32_t {
      x = max(x, __shfl_xor(x, 16));
      x = max(x, __shfl_xor(x, 32));
      return __builtin_amdgcn_readfirstlane(x);
    };
    auto prefetch = [&](int slot, uint32_t jn) {
      if (n8 + 4u * jn >= nrow) return;  // (wave-uniform)
      row_frame(jn, frn[slot], Ltn[slot]);
      const uint32_t m2 = (uint32_t)(reinterpret_cast<uintptr_t>(frn[slot]) & 7u);
      const uint2* b2 = reinterpret_cast<const uint2*>(frn[slot] - m2);
      const int32_t Q2 = (int32_t)((Ltn[slot] + m2 + 7u) >> 3);
      const int32_t qm = wave_min(Q2);
      if (qm >= 16 * PQ) {
#pragma unroll
        for (int u = 0; u < PQ; ++u) pf[slot][u] = rv_ld(b2 + (int32_t)p + 16 * u);
        asm volatile("");  // (keeps the arms' loads apart: merged, every load takes the select)
      } else if (qm >= 16 * (PQ - 1)) {  // (MTU frames: the last unit alone may pass the frame's end)
#pragma unroll
        for (int u = 0; u < PQ - 1; ++u) pf[slot][u] = rv_ld(b2 + (int32_t)p + 16 * u);
        const int32_t q = (int32_t)p + 16 * (PQ - 1);
        pf[slot][PQ - 1] = rv_ld(q < Q2 ? b2 + q : zero);
        asm volatile("");
      } else {
        // short frames (the Zipf mix): only the units some row's frame reaches
        // are loaded (a wave-uniform count), the rest are zero without a load
        const int32_t um = (wave_max(Q2) + 15) >> 4;
#pragma unroll
        for (int u = 0; u < PQ; ++u) {
          const int32_t q = (int32_t)p + 16 * u;
          pf[slot][u] = u < um ? rv_ld(q < Q2 ? b2 + q : zero) : make_uint2(0u, 0u);
        }
      }
    };
#pragma unroll
    for (int a = 0; a < PR; ++a) prefetch(a, (uint32_t)a);
    for (uint32_t j = 0; n8 + 4u * j < nrow; ++j) {
      const uint32_t k = n8 + 4u * j + row;  // the row's frame in the group (its sorted position)
      const uint8_t* fr = frn[0];
      // Lt: the bytes loaded and folded; Lc: the CRC's length (zeros past Lt); L: the sum's end
      const uint32_t Lt = Ltn[0];
      const uint32_t Lc = TX && CRC && (Lt < 60u ? 60u : Lt) + 4u <= capacity ? (Lt < 60u ? 60u : Lt) : Lt;
      const uint32_t L = TX ? Lt : (Lt > trim ? Lt - trim : 0u);
      const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(fr) & 7u);
      const uint2* base2 = reinterpret_cast<const uint2*>(fr - mis);
      const int32_t QE = (int32_t)((Lt + mis + 7u) >> 3);  // qwords holding frame bytes
      const int32_t NL = (int32_t)(((Lc + mis + 7u) >> 3) + 15u) >> 4;  // lines of the CRC window
      int32_t nit = (QE + 16 * kRvUnroll - 1) / (16 * kRvUnroll), qmin = QE;
      nit = max(nit, __shfl_xor(nit, 16));
      nit = max(nit, __shfl_xor(nit, 32));
      nit = __builtin_amdgcn_readfirstlane(nit);
      qmin = wave_min(qmin);
      // the units (qwords per lane) any row's CRC window reaches: the later ones
      // fold nothing and are skipped (wave-uniform)
      const int32_t nlw = wave_max(NL), qmw = (wave_max(QE) + 15) >> 4;
      uint32_t r = 0, S = 0;
      // the qwords holding the bytes at or past L (the FCS, the last qword's
      // bytes past the frame) went into S, those past Lt into the CRC of lines
      // >= 1: the lanes that hold them (qwords qL .. QE - 1, at most two) take
      // them out again after the fold
      const int32_t lastq = QE - 1, qL = (int32_t)((L + mis) >> 3);
      const int32_t qme = (lastq & 15) == (int32_t)p ? lastq : (qL & 15) == (int32_t)p && qL < lastq ? qL : -1;
      uint2 ye = make_uint2(0u, 0u);
      // short passes (every row's window within 4 lines, the Zipf mix): the
      // qword(s) at the end are taken as the fold passes them, 8 selects,
      // rather than loaded again after it (an L2 round trip at the end of the
      // pass); MTU passes (12 lines: 24 selects) load it again.  Receive only:
      // in the transmit kernel it bought 0.9 % on Zipf and cost 0.4 % on MTU
      // frames (A/B x4, r8a); receive: Zipf -1.4 %, ingress's Zipf -2.7 %
      const bool cap4 = !HOST && !TX && nlw <= 4;
      auto capture = [&](const uint2 (&y)[kRvUnroll], int it) {
        if constexpr (HOST) {
#pragma unroll
          for (int u = 0; u < kRvUnroll; ++u) {
            const bool at = (int32_t)p + 16 * (u + kRvUnroll * it) == qme;
            ye.x = at ? y[u].x : ye.x;
            ye.y = at ? y[u].y : ye.y;
          }
        } else if (it == 0 && cap4) {
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const bool at = (int32_t)p + 16 * u == qme;
            ye.x = at ? y[u].x : ye.x;
            ye.y = at ? y[u].y : ye.y;
          }
        }
      };
      // one qword: the sum, and the CRC unit (in the window iff `in`)
      auto fold = [&](uint2 y, int u, int it, bool in) {
        uint32_t c0 = y.x, c1 = y.y;
        if (u == 0 && it == 0) {
          // line 0: the sum from frame offset 14 on; the CRC over the frame's bytes, init on 0..3
          const int32_t o0 = 8 * (int32_t)p - (int32_t)mis;
          S = rv_dot2(c0 & rv_keep_from(14 - o0), rv_dot2(c1 & rv_keep_from(10 - o0), S));
          if constexpr (CRC) {
            const int32_t ie = (int32_t)(Lc < 4 ? Lc : 4u);
            c0 = (c0 & rv_range(o0, 0, (int32_t)Lt)) ^ rv_range(o0, 0, ie);
            c1 = (c1 & rv_range(o0 + 4, 0, (int32_t)Lt)) ^ rv_range(o0 + 4, 0, ie);
          }
        } else {
          S = rv_dot2(c0, rv_dot2(c1, S));
        }
        if constexpr (CRC) {
          const uint32_t nr = rv_unit(lds, r ^ c0, c1, z);
          r = in ? nr : r;
        }
      };
      {
        // batch 0: the prefetched qwords, the rest loaded now, then the next pass's prefetch
        uint2 y[kRvUnroll];
#pragma unroll
        for (int u = 0; u < PQ; ++u) y[u] = pf[0][u];
        if constexpr (PQ < kRvUnroll) {
          if (qmin >= 16 * (kRvUnroll - 1)) {  // (MTU frames: the last unit alone may pass the frame's end)
#pragma unroll
            for (int u = PQ; u < kRvUnroll - 1; ++u) y[u] = rv_ld(base2 + (int32_t)p + 16 * u);
            const int32_t q = (int32_t)p + 16 * (kRvUnroll - 1);
            y[kRvUnroll - 1] = rv_ld(q < QE ? base2 + q : zero);
            asm volatile("");
          } else {
#pragma unroll
            for (int u = PQ; u < kRvUnroll; ++u) {
              const int32_t q = (int32_t)p + 16 * u;
              y[u] = u < qmw ? rv_ld(q < QE ? base2 + q : zero) : make_uint2(0u, 0u);
            }
          }
        }
        // the prefetch slots move down one; the last takes pass j + PR
#pragma unroll
        for (int a = 0; a + 1 < PR; ++a) {
          frn[a] = frn[a + 1];
          Ltn[a] = Ltn[a + 1];
#pragma unroll
          for (int u = 0; u < PQ; ++u) pf[a][u] = pf[a + 1][u];
        }
        prefetch(PR - 1, j + (uint32_t)PR);
        if (p < kRvHead) head[kRvHead * k + p] = y[0];  // the frame's first qwords for phase B
        capture(y, 0);
        if (qmin >= 16 * (kRvUnroll - 1) + 1) {  // (then NL >= 12: Lc >= Lt)
          // every row's window covers all twelve lines (MTU frames): no window test
#pragma unroll
          for (int u = 0; u < kRvUnroll; ++u) fold(y[u], u, 0, true);
        } else {
#pragma unroll
          for (int u = 0; u < kRvUnroll; ++u)
            if (u == 0 || u < nlw) fold(y[u], u, 0, u < NL);
        }
      }
      for (int32_t it = 1; it < nit; ++it) {
        uint2 y[kRvUnroll];
#pragma unroll
        for (int u = 0; u < kRvUnroll; ++u) {
          const int32_t q = (int32_t)p + 16 * (u + kRvUnroll * it);
          y[u] = rv_ld(q < QE ? base2 + q : zero);
        }
        capture(y, it);
#pragma unroll
        for (int u = 0; u < kRvUnroll; ++u) fold(y[u], u, it, u + kRvUnroll * it < NL);
      }
      if constexpr (!HOST) {
        if (!cap4) ye = rv_ld(qme >= 0 ? base2 + qme : zero);  // (an L2 hit: the fold just read it)
      }
      const int32_t oe = 8 * qme - (int32_t)mis;
      S -= rv_dot2(ye.x & rv_keep_from((int32_t)L - oe), rv_dot2(ye.y & rv_keep_from((int32_t)L - oe - 4), 0u)) &
           (qme >= 0 && L >= 14 ? ~0u : 0u);
      uint32_t okf = 1;
      if constexpr (CRC) {
        const bool junk = qme == lastq && lastq >= 16;
        r ^= rv_unit(lds, junk ? ye.x & rv_keep_from((int32_t)Lt - oe) : 0u,
                     junk ? ye.y & rv_keep_from((int32_t)Lt - oe - 4) : 0u, z);
        // the window ends W = 128 NL - mis (frame offsets) past the frame start; W - Lc = 8a + b
        const uint32_t pad = (uint32_t)(128 * NL - (int32_t)mis - (int32_t)Lc);
        const uint32_t a = pad >> 3, b = pad & 7u;
        const uint32_t x = rv_row_xor(rv_nib_f(lds, p + a, r));
        const uint32_t R = rv_nib(lds, kRvB + 512u * b, x);
        okf = TX ? R : (uint32_t)(Lt >= 4 && ~R == 0x2144DF1Cu);
      }
      S = rv_row_add(S);
      if (p == 0) res[k] = make_uint2(okf, S);
    }
    return rank;
}

template <bool CRC, bool FILT, bool HOST>
__global__ void __launch_bounds__(kRvBlock)
rx_verify_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t n, uint32_t flags,
                 uint8_t* __restrict__ okv, uint8_t* __restrict__ verdict, const uint32_t* __restrict__ seg_len,
                 const uint32_t* __restrict__ image, uint32_t gsz, RxFilter filt, const uint32_t* __restrict__ gate,
                 uint32_t epoch) {
  // behind the ingress launch (lnx_ingress_verify_batch on a short-frame
  // batch, launch_ingress_verify): nothing to do unless it left this call's
  // epoch in the gate word
  if (gate && *gate != epoch) return;
  constexpr uint32_t kTabBytes = CRC ? kRvBytes : 0u;
  constexpr uint32_t kWaveBytes = kRvGroup * 8u * (1u + kRvHead);
  __shared__ __attribute__((aligned(16))) char lds[kTabBytes + (kRvBlock / 64) * kWaveBytes];
  if constexpr (CRC) {
    const uint32_t t = threadIdx.x;
    for (uint32_t vi = t; vi < 2048u; vi += kRvBlock) {
      const uint32_t v = image[vi];
      uint4* row = reinterpret_cast<uint4*>(lds + kRvT + ((vi & 255u) << 8) + ((vi >> 8) << 5));
      const uint4 v4 = {v, v, v, v};
      row[0] = v4;
      row[1] = v4;
    }
    // F_q (q < 32): entry e of table q at dword 32 e + q, so the 16 lanes of a
    // row (16 different tables) read 16 different banks; B_b as in the image
    for (uint32_t i = t; i < 32u * 128u; i += kRvBlock)
      reinterpret_cast<uint32_t*>(lds + kRvF)[32u * (i & 127u) + (i >> 7)] = image[kRvImgF + i];
    for (uint32_t i = t; i < 8u * 128u; i += kRvBlock)
      reinterpret_cast<uint32_t*>(lds + kRvB)[i] = image[kRvImgF + 32u * 128u + i];
    __syncthreads();
  }
  const uint32_t trim = CRC ? 4u : 0u;
  const uint32_t lane = threadIdx.x & 63u, wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const RvLane z(lane);
  uint2* res = reinterpret_cast<uint2*>(lds + kTabBytes + kWaveBytes * wv);  // (FCS ok, S) per frame
  uint2* head = res + kRvGroup;                                                // kRvHead qwords per frame
  const uint2* zero = g_rv_zero;
  // gsz <= kRvGroup frames per group, a multiple of 4 (the launcher's choice:
  // every wave gets the same number of groups, launch_rx_verify)
  const uint64_t ngroups = (n + gsz - 1u) / gsz;
  for (uint64_t g = (uint64_t)blockIdx.x * (kRvBlock / 64) + wv; g < ngroups; g += (uint64_t)gridDim.x * (kRvBlock / 64)) {
    // the group's frames: lane k < gsz holds frame g * gsz + k's start and length (FCS included)
    const uint64_t fk = g * gsz + lane;
    // (32-bit compares on the scalar unit: the 64-bit one, which SALU lacks,
    // held gsz in a VGPR pair through the whole kernel)
    const uint64_t rem = n - g * gsz;
    const uint32_t nrow = (uint32_t)(rem >> 32) != 0u || (uint32_t)rem >= gsz ? gsz : (uint32_t)rem;
    const bool live = lane < nrow;
    const uint64_t fi = live ? fk : n - 1u;
    const uint64_t sk = off[fi];
    const uint64_t ek = seg_len ? sk + seg_len[fi] : off[fi + 1];
    const uint64_t ltk = live && ek > sk ? ek - sk : 0u;
    const uint32_t Ltk = ltk < 0x7FFFFFFFull ? (uint32_t)ltk : 0x7FFFFFFFu;

    // ---------------------------------------------------------------- A: data
    // (the whole next pass loaded ahead from HBM: 0.335 against 0.340-0.344 ms for 8 of
    // its 12 qwords; over PCIe 8 measured 34.4 against 33.7 GiB/s)
    // (the frame's results sit at its position in the passes' order: pos)
    const uint32_t pos = rv_rows<CRC, false, HOST, HOST ? kRvPf : kRvPfRx>(lds, res, head, z, bytes, sk, Ltk, nrow, trim,
                                                                           0u);
    __builtin_amdgcn_wave_barrier();  // (the wave's own LDS writes, read back in order below)

    // ---------------------------------------------------------------- B: verdicts
    const uint64_t f = fk;
    const uint32_t Lt = Ltk;
    const uint32_t L = Lt > trim ? Lt - trim : 0u;  // the frame the verdict sees
    const uint8_t* fr = bytes + sk;
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(fr) & 7u);
    const uint2* base2 = reinterpret_cast<const uint2*>(fr - mis);
    const int32_t QE = (int32_t)((Lt + mis + 7u) >> 3);
    const uint32_t kk = lane < gsz ? pos : 0u;
    // the staged qwords 0 .. kRvHead - 1 of the frame's window (frame offsets -mis .. 72 - mis),
    // then qwords 9, 10 from memory for the frames that need them (IPv4 options past offset 64)
    uint32_t dw[22];
#pragma unroll
    for (uint32_t i = 0; i < kRvHead; ++i) {
      const uint2 v = head[kRvHead * kk + i];
      dw[2 * i] = v.x;
      dw[2 * i + 1] = v.y;
    }
    // the frame's bytes 4k .. 4k + 3 as one dword, k < 15 (offsets < 60)
    const uint32_t sh = mis & 3u;
    uint32_t F[15];
#pragma unroll
    for (int k = 0; k < 15; ++k) {
      const uint32_t lo = mis >= 4 ? dw[k + 1] : dw[k], hi = mis >= 4 ? dw[k + 2] : dw[k + 1];
      F[k] = __builtin_amdgcn_alignbyte(hi, lo, sh);
    }
    auto byt = [](uint32_t w, int i) -> uint32_t { return (w >> (8 * i)) & 0xFFu; };
    auto be16 = [&](int o) -> uint32_t {  // the big-endian 16-bit field at static frame offset o (o < 59)
      const uint32_t w = (o & 3) == 3 ? __builtin_amdgcn_alignbyte(F[(o >> 2) + 1], F[o >> 2], 3) : F[o >> 2];
      const int i = (o & 3) == 3 ? 0 : (o & 3);
      return (byt(w, i) << 8) | byt(w, i + 1);
    };
    auto le32 = [&](int o) -> uint32_t {  // the frame's bytes o .. o + 3 (o % 4 == 2 or 0)
      return (o & 3) == 0 ? F[o >> 2] : __builtin_amdgcn_alignbyte(F[(o >> 2) + 1], F[o >> 2], (uint32_t)(o & 3));
    };
    // a field at a header-length-dependent offset o (o + 2 <= L checked by the caller): staged, else from memory
    auto dyn16 = [&](uint32_t o) -> uint32_t {
      const uint32_t a = o + mis;  // byte of the window
      uint32_t b0, b1;
      if (a + 2u <= 8u * kRvHead) {
        const uint8_t* hb = reinterpret_cast<const uint8_t*>(head + kRvHead * kk);
        b0 = hb[a];
        b1 = hb[a + 1u];
      } else {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(base2) + (a >> 2);
        const uint32_t lo = rv_ld32(w), hi = (a & 3u) == 3u ? rv_ld32(w + 1) : 0u;
        const uint32_t v2 = __builtin_amdgcn_alignbyte(hi, lo, a & 3u);
        b0 = v2 & 0xFFu;
        b1 = (v2 >> 8) & 0xFFu;
      }
      return (b0 << 8) | b1;
    };
    // LE 16-bit sum of the frame's bytes [a, b) among dwords D0 .. D1 - 1 of dw
    // (those that can hold them: frame offset o lies in dword (o + mis) / 4, mis < 8)
    auto hsum = [&](auto D0, auto D1, int32_t a, int32_t b) -> uint32_t {
      uint32_t acc = 0;
#pragma unroll
      for (int d = decltype(D0)::value; d < decltype(D1)::value; ++d)
        acc = rv_dot2(dw[d] & rv_range(4 * d - (int32_t)mis, a, b), acc);
      return acc;
    };
    using I3 = std::integral_constant<int, 3>;
    using I5 = std::integral_constant<int, 5>;
    using I8 = std::integral_constant<int, 8>;
    using I11 = std::integral_constant<int, 11>;
    using I16 = std::integral_constant<int, 16>;
    using I18 = std::integral_constant<int, 18>;
    using I22 = std::integral_constant<int, 22>;

    // ---- header parse (ingress_kernel.hip's, FCS excluded: L bytes)
    uint32_t v = 0, v_udp4 = 0;
    bool hdr_sum = false, l4_sum = false;
    int32_t pa = 0, pb = 0, la = 0, lb = 0;
    uint32_t lseed = 0;
    if (L < 14) {
      v = kErrTruncatedFrame;
    } else {
      const uint32_t et = be16(12);
      bool eth_drop = false, et_handler = true;
      if (FILT && filt.on) {
        // StackEthernet.Demux (internet/stack-ethernet.go:146-152), before ValidateSize
        const uint32_t D0 = F[0], D1 = F[1] & 0xFFFFu;
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
          const uint32_t b0 = byt(F[3], 2), tl = be16(16), ihl = b0 & 15u;
          if (FILT && filt.on && filt.ip4 != 0u) {
            const uint32_t dst = le32(30);  // demux4's destination check (stack-ip4.go:108-119)
            const bool mc = (dst & 0xF0u) == 0xE0u, bc = dst == 0xFFFFFFFFu;
            if (dst != filt.ip4 && !(filt.ip4_mc && mc) && !(filt.ip4_bc && bc)) v = kErrPacketDrop;
          }
          if (v != 0) {
          } else if (tl < 20) v = kErrInvalidLengthField;
          else if (tl > M) v = kErrTruncatedFrame;
          else if (ihl < 5 || ihl * 4 > tl) v = kErrInvalidLengthField;
          else if ((b0 >> 4) != 4) v = kErrInvalidField;
          else if ((flags & kVerifyEvilBit) && (be16(20) & (1u << 13))) v = kErrPacketDrop;
          if (v == 0) {
            hdr_sum = true;
            const uint32_t hl = ihl * 4, proto = byt(F[5], 3), P = tl - hl;
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
                const uint32_t ul = dyn16(14 + hl + 4);
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
                const uint32_t type = dyn16(14 + hl) >> 8;
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
          const uint32_t pl = be16(18), proto = byt(F[5], 0);
          if (FILT && filt.on && (filt.ip6[0] | filt.ip6[1] | filt.ip6[2] | filt.ip6[3]) != 0u) {
            const uint32_t d0 = le32(38), d1 = le32(42), d2 = le32(46), d3 = le32(50);
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
              else if (be16(58) < 8) v = kErrInvalidLengthField;
              else if (be16(58) > pl) v = kErrTruncatedFrame;
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

    // ---- the sums: header [14, 34) and pseudo-header [pa, pb) from the staged
    // bytes; the segment [la, lb) = S - [14, la) - [lb, L)
    // (IPv4 options past the staged bytes: qwords 9 and 10 from memory)
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int32_t q = (int32_t)kRvHead + i;
      const bool need = l4_sum && la + (int32_t)mis > 8 * (int32_t)kRvHead && q < QE;
      const uint2 v2 = rv_ld(need ? base2 + q : zero);
      dw[2 * q] = v2.x;
      dw[2 * q + 1] = v2.y;
    }
    const uint32_t hS = hdr_sum ? hsum(I3{}, I11{}, 14, 34) : 0u;  // bytes 14..33: dwords 3..10
    // the bytes from the segment's end to L: staged when they end inside the
    // staged qwords, else the whole wave sums them from memory (one frame at a time)
    const bool tail = l4_sum && lb < (int32_t)L;
    const bool tail_staged = tail && (int32_t)(L + mis) <= 8 * (int32_t)kRvHead;
    uint32_t tS = tail_staged ? hsum(I8{}, I18{}, lb, (int32_t)L) : 0u;  // lb >= 34, L + mis <= 72
    uint64_t longt = __builtin_amdgcn_ballot_w64(tail && !tail_staged);
    while (longt) {
      const uint32_t kf = (uint32_t)__builtin_ctzll(longt);
      longt &= longt - 1u;
      const int32_t a = __builtin_amdgcn_readlane(lb, kf), b = __builtin_amdgcn_readlane((int32_t)L, kf);
      const uint64_t s2 = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)sk, kf)) |
                          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(sk >> 32), kf) << 32);
      const uint8_t* fr2 = bytes + s2;
      const uint32_t m2 = (uint32_t)(reinterpret_cast<uintptr_t>(fr2) & 7u);
      const uint2* kb = reinterpret_cast<const uint2*>(fr2 - m2);
      const int32_t q0 = (a + (int32_t)m2) >> 3, q1 = (b + (int32_t)m2 + 7) >> 3;
      uint32_t acc = 0;
      for (int32_t qb = q0; qb < q1; qb += 64) {  // (a wave-uniform trip count)
        const int32_t q = qb + (int32_t)lane;
        const uint2 t = rv_ld(q < q1 ? kb + q : zero);
        const int32_t o0 = 8 * q - (int32_t)m2;
        acc = rv_dot2(t.x & rv_range(o0, a, b), rv_dot2(t.y & rv_range(o0 + 4, a, b), acc));
      }
#pragma unroll
      for (int sft = 1; sft < 64; sft <<= 1) acc += (uint32_t)__shfl_xor((int)acc, sft);
      tS += lane == kf ? acc : 0u;
    }
    const uint2 rk = res[kk];
    // [14, la): la <= 74; [pa, pb) within [22, 54)
    if (l4_sum) tS = rk.y - hsum(I3{}, I22{}, 14, la) - tS + hsum(I5{}, I16{}, pa, pb);
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
    if (live) {
      if (okv) okv[f] = (uint8_t)rk.x;  // (null: the verdicts alone, for lnx_ingress_verify_batch)
      verdict[f] = (uint8_t)v;
    }
    __builtin_amdgcn_wave_barrier();  // the next group rewrites res and head
  }
}

// ------------------------------------------------------------------ transmit
// tx_finish_kernel: lneto's transmit tail for frames in place, ONE read of each
// frame -- the checksum-generate step (lnx_tx_checksum_batch: encapsulate4 /
// encapsulate6 and the ICMP clients, internet/stack-ip4.go:202-228,
// internet/stack-ip6.go:167-181, ipv4/icmpv4/client.go:210-214,
// ipv6/icmpv6/client.go:135-148; ingress_kernel.hip GEN) and then the padding
// to 60 bytes and the LE FCS (lnx_fcs_append_batch, internet/stack-ethernet.go:
// 200-214).  Phase A is the receive kernel's (rv_rows<CRC, true>): the raw sum
// S of [14, L) and the CRC register R0 of the frame AS IT IS, padded with
// zeros.  Phase B, one lane per frame, parses the headers, sets the length
// fields and checksums exactly as the GEN rows do (sums over the bytes as
// loaded, the old field values taken out), and corrects the CRC for the fields
// it changed by linearity: a 16-bit change d at frame offset o changes the
// register after Lp bytes by Z_{Lp - o}(d) (d's first byte in the register's
// low byte); all such fields lie in the first 128 bytes, so
//   R = R0 ^ Z_{Lp - c}( XOR_f Z_{c - o_f}(d_f) ),  c = min(Lp, 128),
// the shifts by binary powers (nibble tables of Z_{2^m}, m < 16: every frame
// the step changes is shorter than 64 KiB).  Then the fields, the padding and
// the FCS are stored in place: a few 2- and 4-byte stores per frame, which is
// what the zero-copy egress of the ring wants (each store to host memory costs
// about a nanosecond, tools/ubench/host_write.hip).
// Segment form: frame f = bytes[start[f] : start[f] + len[f]], with room for
// the padding and FCS within `capacity` bytes of start[f]; len[f] is updated;
// st_ck[f] = the checksum step's status (0, 18, 15), st_ap[f] = the append's
// (0, or 6 ErrShortBuffer with the frame left unpadded).
constexpr uint32_t kTxP = kRvBytes;                    // Z_{2^m} nibble tables in LDS (after F, B)
constexpr uint32_t kTxTabBytes = kRvBytes + 16u * 512u;
constexpr uint32_t kTxImgP = kRvImgF + 40u * 128u;     // ... and in the image

// Z_k(x), k < 2^16, by binary powers (the steps some lane of the wave needs)
__device__ __forceinline__ uint32_t tx_zk(const char* lds, uint32_t k, uint32_t x) {
#pragma unroll 1
  for (uint32_t m = 0; m < 16u; ++m) {
    if (__builtin_amdgcn_ballot_w64((k >> m) & 1u) == 0) continue;
    const uint32_t y = rv_nib(lds, kTxP + 512u * m, x);
    x = (k >> m) & 1u ? y : x;
  }
  return x;
}
// XOR_f Z_{k_f}(x_f) over four fields: the four chains side by side (each step
// that some lane of the wave needs for some field maps all four)
__device__ __forceinline__ uint32_t tx_zk4(const char* lds, const uint32_t (&k)[4], uint32_t (&x)[4]) {
  const uint32_t ka = k[0] | k[1] | k[2] | k[3];
#pragma unroll 1
  for (uint32_t m = 0; m < 16u; ++m) {
    if (__builtin_amdgcn_ballot_w64((ka >> m) & 1u) == 0) continue;
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const uint32_t y = rv_nib(lds, kTxP + 512u * m, x[f]);
      x[f] = (k[f] >> m) & 1u ? y : x[f];
    }
  }
  return x[0] ^ x[1] ^ x[2] ^ x[3];
}

// store the big-endian 16-bit value v at frame address q (2 bytes)
__device__ __forceinline__ void tx_put16(uint8_t* q, uint32_t v) {
  if ((reinterpret_cast<uintptr_t>(q) & 1u) == 0) {
    *reinterpret_cast<uint16_t*>(q) = (uint16_t)(((v & 0xFFu) << 8) | ((v >> 8) & 0xFFu));
  } else {
    q[0] = (uint8_t)(v >> 8);
    q[1] = (uint8_t)v;
  }
}
// store the 4 bytes of w (little-endian) at q, by naturally aligned pieces
__device__ __forceinline__ void tx_put32(uint8_t* q, uint32_t w) {
  const uint32_t a = (uint32_t)(reinterpret_cast<uintptr_t>(q) & 3u);
  if (a == 0) {
    *reinterpret_cast<uint32_t*>(q) = w;
  } else if (a == 2) {
    reinterpret_cast<uint16_t*>(q)[0] = (uint16_t)w;
    reinterpret_cast<uint16_t*>(q)[1] = (uint16_t)(w >> 16);
  } else {
    q[0] = (uint8_t)w;
    *reinterpret_cast<uint16_t*>(q + 1) = (uint16_t)(w >> 8);
    q[3] = (uint8_t)(w >> 24);
  }
}

template <bool FCS, bool CK, bool HOST>
__global__ void __launch_bounds__(HOST ? kTxBlockHost : kTxBlock)
tx_finish_kernel(uint8_t* __restrict__ bytes, const uint64_t* __restrict__ start, uint32_t* __restrict__ len,
                 uint32_t n, uint32_t capacity, uint8_t* __restrict__ st_ck, uint8_t* __restrict__ st_ap,
                 const uint32_t* __restrict__ image, uint32_t gsz, const uint32_t* __restrict__ gate, uint32_t epoch) {
  // behind the generate rows (lnx_tx_checksum_batch on a short-frame batch,
  // launch_tx_checksum): nothing to do unless they left this call's epoch
  if (gate && *gate != epoch) return;
  constexpr uint32_t kB = HOST ? kTxBlockHost : kTxBlock;
  constexpr uint32_t kTabBytes = FCS ? kTxTabBytes : 0u;
  constexpr uint32_t kWaveBytes = kTxGroup * 8u * (1u + kRvHead);
  __shared__ __attribute__((aligned(16))) char lds[kTabBytes + (kB / 64) * kWaveBytes];
  if constexpr (FCS) {
    const uint32_t t = threadIdx.x;
    for (uint32_t vi = t; vi < 2048u; vi += kB) {
      const uint32_t v = image[vi];
      uint4* row = reinterpret_cast<uint4*>(lds + kRvT + ((vi & 255u) << 8) + ((vi >> 8) << 5));
      const uint4 v4 = {v, v, v, v};
      row[0] = v4;
      row[1] = v4;
    }
    for (uint32_t i = t; i < 32u * 128u; i += kB)
      reinterpret_cast<uint32_t*>(lds + kRvF)[32u * (i & 127u) + (i >> 7)] = image[kRvImgF + i];
    for (uint32_t i = t; i < 8u * 128u; i += kB)
      reinterpret_cast<uint32_t*>(lds + kRvB)[i] = image[kRvImgF + 32u * 128u + i];
    for (uint32_t i = t; i < 16u * 128u; i += kB) reinterpret_cast<uint32_t*>(lds + kTxP)[i] = image[kTxImgP + i];
    __syncthreads();
  }
  const uint32_t lane = threadIdx.x & 63u, wv = (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const RvLane z(lane);
  uint2* res = reinterpret_cast<uint2*>(lds + kTabBytes + kWaveBytes * wv);  // (R0, S) per frame
  uint2* head = res + kTxGroup;
  const uint2* zero = g_rv_zero;
  // (32-bit frame indices: the launcher splits larger batches; 64-bit ones cost
  // the kernel 30 registers' worth of scratch spills)
  // gsz <= kTxGroup frames per group, a multiple of 4 (launch_tx_finish)
  const uint32_t ngroups = (n + gsz - 1u) / gsz;
  for (uint32_t g = blockIdx.x * (kB / 64) + wv; g < ngroups; g += gridDim.x * (kB / 64)) {
    const uint32_t fk = g * gsz + lane;
    const bool live = lane < gsz && fk < n;
    const uint32_t fi = live ? fk : n - 1u;
    const uint64_t sk = start[fi];
    const uint32_t Ltk = live ? len[fi] : 0u;
    const uint32_t nrow = (uint32_t)(n - g * gsz < gsz ? n - g * gsz : gsz);
    const uint32_t pos = rv_rows<FCS, true, HOST, HOST ? kRvPf : kTxPf>(lds, res, head, z, bytes, sk, Ltk, nrow, 0u,
                                                                         capacity);
    __builtin_amdgcn_wave_barrier();

    // ---------------------------------------------------------------- B: one lane per frame
    const uint32_t L = Ltk;
    uint8_t* fr = bytes + sk;
    const uint32_t mis = (uint32_t)(reinterpret_cast<uintptr_t>(fr) & 7u);
    const uint2* base2 = reinterpret_cast<const uint2*>(fr - mis);
    const int32_t QE = (int32_t)((L + mis + 7u) >> 3);
    const uint32_t kk = lane < gsz ? pos : 0u;
    // the staged window bytes, read from LDS where used (held in registers, the
    // header words cost the kernel its occupancy: see kTxBlock); qwords 9 and 10
    // (IPv4 options past the staged bytes) from memory below
    const uint8_t* hbc = reinterpret_cast<const uint8_t*>(head + kRvHead * kk);
    const uint32_t* hw = reinterpret_cast<const uint32_t*>(head + kRvHead * kk);
    uint32_t dx[4] = {0, 0, 0, 0};
    auto dwd = [&](int d) -> uint32_t { return d < 2 * (int)kRvHead ? hw[d] : dx[d - 2 * (int)kRvHead]; };
    auto byt = [&](int o) -> uint32_t { return hbc[(uint32_t)o + mis]; };  // frame byte o (o + mis < 72)
    auto be16 = [&](int o) -> uint32_t { return (byt(o) << 8) | byt(o + 1); };
    auto dyn16 = [&](uint32_t o) -> uint32_t {  // (o + 2 <= L checked by the caller)
      const uint32_t a = o + mis;
      uint32_t b0, b1;
      if (a + 2u <= 8u * kRvHead) {
        const uint8_t* hb = reinterpret_cast<const uint8_t*>(head + kRvHead * kk);
        b0 = hb[a];
        b1 = hb[a + 1u];
      } else {
        const uint32_t* w = reinterpret_cast<const uint32_t*>(base2) + (a >> 2);
        const uint32_t lo = rv_ld32(w), hi = (a & 3u) == 3u ? rv_ld32(w + 1) : 0u;
        const uint32_t v2 = __builtin_amdgcn_alignbyte(hi, lo, a & 3u);
        b0 = v2 & 0xFFu;
        b1 = (v2 >> 8) & 0xFFu;
      }
      return (b0 << 8) | b1;
    };
    auto hsum = [&](auto D0, auto D1, int32_t a, int32_t b) -> uint32_t {
      uint32_t acc = 0;
#pragma unroll
      for (int d = decltype(D0)::value; d < decltype(D1)::value; ++d)
        acc = rv_dot2(dwd(d) & rv_range(4 * d - (int32_t)mis, a, b), acc);
      return acc;
    };
    using I3 = std::integral_constant<int, 3>;
    using I5 = std::integral_constant<int, 5>;
    using I11 = std::integral_constant<int, 11>;
    using I16 = std::integral_constant<int, 16>;
    using I22 = std::integral_constant<int, 22>;
    // a 16-bit big-endian value at an even frame offset, as it adds to the LE half-word sums
    auto cv = [&](uint32_t v) -> uint32_t { return (mis & 1u) ? v : (((v & 0xFFu) << 8) | (v >> 8)); };

    // ---- the checksum step (ingress_kernel.hip GEN, oracle.tx_checksum)
    uint32_t v = 0;
    uint32_t g_off[4] = {0, 0, 0, 0}, g_new[4] = {0, 0, 0, 0}, g_old[4] = {0, 0, 0, 0};
    bool hdr_sum = false, l4_sum = false, g_nz = false;
    int32_t pa = 0, pb = 0, la = 0;
    uint32_t lseed = 0, g_fix_h = 0, g_fix_t = 0;
    if constexpr (CK) {
      if (L < 14) {
        v = kErrTruncatedFrame;
      } else {
        const uint32_t et = be16(12);
        if (et == 0x0800) {
          const uint32_t ihl = byt(14) & 15u, hl = 4 * ihl;
          if (L < 34) v = kErrTruncatedFrame;
          else if (ihl < 5) v = kErrInvalidLengthField;
          else if (14 + hl > L) v = kErrTruncatedFrame;
          else if (L - 14 > 0xFFFFu) v = kErrInvalidLengthField;
          if (v == 0) {
            const uint32_t tl = L - 14, nn = tl - hl, proto = byt(23);
            const uint32_t need = proto == 6 ? 20u : (proto == 17 || proto == 1) ? 8u : 0u;
            if (nn < need) v = kErrTruncatedFrame;
            if (v == 0) {
              hdr_sum = true;
              g_off[0] = 16, g_new[0] = tl, g_old[0] = be16(16);  // SetTotalLength(n + hl)
              g_off[1] = 24, g_old[1] = be16(24);                 // SetCRC(CalculateHeaderCRC())
              g_fix_h = cv(tl) - cv(g_old[0]) - cv(g_old[1]);
              if (need) {
                l4_sum = true;
                la = 14 + hl;
                const uint32_t at = proto == 6 ? 16u : proto == 17 ? 6u : 2u;
                g_off[2] = la + at, g_old[2] = dyn16(la + at);
                g_fix_t = 0u - cv(g_old[2]);
                if (proto != 1) pa = 26, pb = 34, lseed = nn + proto;  // CRCWriteTCPPseudo / CRCWriteUDPPseudo(n)
                if (proto == 17) {
                  g_off[3] = la + 4, g_new[3] = nn, g_old[3] = dyn16(la + 4);  // SetLength(n)
                  g_fix_t += cv(nn) - cv(g_old[3]);
                  g_nz = true;
                }
              }
            }
          }
        } else if (et == 0x86DD) {
          const uint32_t nn = L - 54, proto = byt(20);
          if (L < 54) v = kErrTruncatedFrame;
          else if (nn > 0xFFFFu) v = kErrInvalidLengthField;
          const uint32_t need = proto == 6 ? 20u : (proto == 17 || proto == 58) ? 8u : 0u;
          if (v == 0 && nn < need) v = kErrTruncatedFrame;
          if (v == 0) {
            g_off[0] = 18, g_new[0] = nn, g_old[0] = be16(18);  // SetPayloadLength(n)
            if (need) {
              l4_sum = true;
              pa = 22, pb = 54, la = 54;  // CRCWritePseudo: AddUint32(n), AddUint32(proto)
              lseed = nn + proto;
              const uint32_t at = proto == 6 ? 16u : proto == 17 ? 6u : 2u;
              g_off[2] = 54 + at, g_old[2] = dyn16(54 + at);
              g_fix_t = 0u - cv(g_old[2]);
              if (proto == 17) {
                g_off[3] = 58, g_new[3] = nn, g_old[3] = be16(58);
                g_fix_t += cv(nn) - cv(g_old[3]);
                g_nz = true;
              }
            }
          }
        }
      }
      // IPv4 options past the staged bytes: qwords 9 and 10 from memory
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int32_t q = (int32_t)kRvHead + i;
        const bool need = l4_sum && la + (int32_t)mis > 8 * (int32_t)kRvHead && q < QE;
        const uint2 v2 = rv_ld(need ? base2 + q : zero);
        dx[2 * i] = v2.x;
        dx[2 * i + 1] = v2.y;
      }
      const uint2 rk = res[kk];
      auto conv = [&](uint32_t S) -> uint32_t {
        if (mis & 1u) return S;
        uint32_t fo = (S & 0xFFFFu) + (S >> 16);
        fo = (fo & 0xFFFFu) + (fo >> 16);
        return ((fo << 8) | (fo >> 8)) & 0xFFFFu;
      };
      if (hdr_sum) g_new[1] = rv_sum16(conv(hsum(I3{}, I11{}, 14, 34) + g_fix_h)) & 0xFFFFu;
      if (l4_sum) {
        const uint32_t tS = rk.y - hsum(I3{}, I22{}, 14, la) + hsum(I5{}, I16{}, pa, pb) + g_fix_t;
        const uint32_t tc = rv_sum16(conv(tS) + lseed) & 0xFFFFu;
        g_new[2] = g_nz && tc == 0 ? 0xFFFFu : tc;
      }
    }
    const bool written = CK && v == 0;

    // ---- the FCS over the frame with its new fields, padded to 60 bytes
    const uint32_t Lp = L < 60u ? 60u : L;
    const bool app = FCS && Lp + 4u <= capacity;
    uint32_t fcs = 0;
    if constexpr (FCS) {
      const uint32_t c = Lp < 128u ? Lp : 128u;
      uint32_t kf[4], xf[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint32_t d = written && g_off[i] != 0 ? (g_old[i] ^ g_new[i]) : 0u;
        xf[i] = ((d >> 8) & 0xFFu) | ((d & 0xFFu) << 8);  // the field's first byte low
        kf[i] = app && xf[i] ? c - g_off[i] : 0u;
      }
      const uint32_t D = tx_zk4(lds, kf, xf);
      const uint32_t dR = tx_zk(lds, app ? Lp - c : 0u, D);
      fcs = ~(res[kk].x ^ dR);
    }

    // ---- stores.  A byte that lies in a staged qword the frame's loads filled
    // (qword < min(kRvHead, QE): it holds what memory holds) is patched into
    // the staged copy, and the row pass below stores the patched qwords with
    // one coalesced write per frame; any other byte is stored directly
    // (the FCS of a frame past 72 bytes: one to three naturally aligned stores).
    const uint32_t qlim = (uint32_t)(QE < (int32_t)kRvHead ? QE : (int32_t)kRvHead);
    uint8_t* hb = reinterpret_cast<uint8_t*>(head + kRvHead * kk);
    uint32_t qlo = 0xFFu, qhi = 0;
    auto patch = [&](uint32_t o, uint32_t b) -> bool {
      const uint32_t a = o + mis;
      if ((a >> 3) >= qlim) return false;
      hb[a] = (uint8_t)b;
      qlo = (a >> 3) < qlo ? (a >> 3) : qlo;
      qhi = (a >> 3) > qhi ? (a >> 3) : qhi;
      return true;
    };
    if (live) {
      if (written) {
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (g_off[i] == 0) continue;
          const uint32_t o = g_off[i], hi8 = g_new[i] >> 8, lo8 = g_new[i] & 0xFFu;
          const bool in0 = patch(o, hi8), in1 = patch(o + 1u, lo8);
          if (!in0 && !in1) {
            tx_put16(fr + o, g_new[i]);
          } else {
            if (!in0) fr[o] = (uint8_t)hi8;
            if (!in1) fr[o + 1u] = (uint8_t)lo8;
          }
        }
      }
      if (app) {
        if (((L + mis) >> 3) >= qlim) {
          for (uint32_t o = L; o < Lp; ++o) fr[o] = 0;  // runts: zero padding to 60 bytes
          tx_put32(fr + Lp, fcs);
        } else {  // (short frames: padding and FCS partly in the staged qwords)
          for (uint32_t o = L; o < Lp + 4u; ++o) {
            const uint32_t b = o < Lp ? 0u : (fcs >> (8u * (o - Lp))) & 0xFFu;
            if (!patch(o, b)) fr[o] = (uint8_t)b;
          }
        }
      }
      if constexpr (FCS) len[fk] = app ? Lp + 4u : L;  // (the checksum step alone leaves the lengths: const for
                                                       // lnx_tx_checksum_batch, which may run this kernel)
      const uint32_t ap = FCS && !app ? 6u : 0u;
      if (st_ap == st_ck) {  // one status array: the checksum step's if non-zero, else the append's
        st_ck[fk] = (uint8_t)(v ? v : ap);
      } else {
        st_ck[fk] = (uint8_t)v;
        st_ap[fk] = (uint8_t)ap;
      }
    }
    // the frame's start (< 2^55) and the span of its patched staged qwords for the rows below
    // (bits 23..31 of the high word: 1 | qlo << 1 | qhi << 5, or 0 when there are none)
    if (lane < gsz)  // (every row pass below reads k < 4 ceil(nrow / 4) <= gsz: written this group)
      res[kk] = make_uint2((uint32_t)sk, (uint32_t)(sk >> 32) | ((live && qlo <= qhi ? 1u | qlo << 1 | qhi << 5 : 0u) << 23));
    __builtin_amdgcn_wave_barrier();
    // ---- the patched staged qwords [qlo, qhi] of each frame, one row per frame
    {
      const uint32_t p = lane & 15u, row = lane >> 4;
      // (readfirstlane: the trip count must stay wave-uniform, or hipcc makes
      // this an exec-narrowing loop with 64-bit loads inside; not in phase A,
      // where it costs 130 bytes of scratch spills per lane)
      const uint32_t nrw = (uint32_t)__builtin_amdgcn_readfirstlane((int)nrow);
      for (uint32_t j = 0; 4u * j < nrw; ++j) {
        const uint32_t k = 4u * j + row;
        const uint2 rk = res[k];
        const uint32_t sp = rk.y >> 23;
        uint8_t* frk = bytes + (((uint64_t)(rk.y & 0x7FFFFFu) << 32) | rk.x);
        uint2* bk = reinterpret_cast<uint2*>(frk - (reinterpret_cast<uintptr_t>(frk) & 7u));
        if ((sp & 1u) && p >= ((sp >> 1) & 15u) && p <= (sp >> 5)) {
          const uint2 q = head[kRvHead * k + p];
          *(__attribute__((address_space(1))) uint64_t*)(bk + p) = (uint64_t)q.x | ((uint64_t)q.y << 32);
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
}

// The group size for n frames over `waves` waves of at most gmax frames a
// group: the fewest rounds of groups the waves can take (ceil(n / gmax) groups
// over the waves), then the smallest group (a multiple of 4: the row passes)
// that still covers n in that many rounds -- so every wave's last round is as
// full as the others, where a fixed size left the last round 33 % (48) or
// 57 % (56) full on 1 M frames (0.331 / 0.322 ms against 0.310 for 52)
uint32_t balanced_group(uint64_t n, uint64_t waves, uint32_t gmax) {
  const uint64_t rounds = ((n + gmax - 1) / gmax + waves - 1) / waves;
  uint64_t g = (n + waves * rounds - 1) / (waves * rounds);
  g = (g + 3) & ~3ull;
  return (uint32_t)(g < 4 ? 4 : g > gmax ? gmax : g);
}

hipError_t launch_tx_finish(uint8_t* bytes, const uint64_t* start, uint32_t* len, uint64_t n, uint32_t capacity,
                            uint32_t flags, uint8_t* st_ck, uint8_t* st_ap, const uint32_t* image, int num_cus,
                            hipStream_t stream, bool host, const uint32_t* gate, uint32_t epoch) {
  const bool ck = flags & 1u, fcs = flags & 2u;
  // batches of up to 2^31 frames (the kernel's 32-bit frame indices)
  for (uint64_t f0 = 0; f0 < n; f0 += 1ull << 31) {
    const uint32_t m = (uint32_t)(n - f0 < (1ull << 31) ? n - f0 : 1ull << 31);
    const uint64_t blk = host ? kTxBlockHost : kTxBlock;
    uint64_t grid = ((uint64_t)m + (blk / 64) * kTxGroup - 1) / ((blk / 64) * kTxGroup);
    if (grid > (uint64_t)num_cus) grid = (uint64_t)num_cus;
    const uint32_t gsz = balanced_group(m, grid * (blk / 64), kTxGroup);
    uint8_t* sa = st_ap == st_ck ? st_ck + f0 : st_ap + f0;
#define LNX_TX(A, C, H)                                                                                                 \
  hipLaunchKernelGGL((tx_finish_kernel<A, C, H>), dim3((unsigned)grid), dim3((unsigned)blk), 0, stream, bytes, start + f0, \
                     len + f0, m, capacity, st_ck + f0, sa, image, gsz, gate, epoch)
    if (host) {
      if (fcs) {
        if (ck) LNX_TX(true, true, true); else LNX_TX(true, false, true);
      } else {
        if (ck) LNX_TX(false, true, true); else LNX_TX(false, false, true);
      }
    } else {
      if (fcs) {
        if (ck) LNX_TX(true, true, false); else LNX_TX(true, false, false);
      } else {
        if (ck) LNX_TX(false, true, false); else LNX_TX(false, false, false);
      }
    }
#undef LNX_TX
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

hipError_t launch_rx_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t flags, bool fcs,
                            uint8_t* ok, uint8_t* verdict, const uint32_t* seg_len, const RxFilter* filter,
                            const uint32_t* image, int num_cus, hipStream_t stream, bool host, const uint32_t* gate,
                            uint32_t epoch) {
  RxFilter filt{};
  if (filter) filt = *filter;
  if (n == 0) return hipSuccess;
  uint64_t grid = (n + (kRvBlock / 64) * kRvGroup - 1) / ((kRvBlock / 64) * kRvGroup);
  if (grid > (uint64_t)num_cus) grid = (uint64_t)num_cus;
  const uint32_t gsz = balanced_group(n, grid * (kRvBlock / 64), kRvGroup);
#define LNX_RV(C, F, H)                                                                                       \
  hipLaunchKernelGGL((rx_verify_kernel<C, F, H>), dim3((unsigned)grid), dim3(kRvBlock), 0, stream, bytes, off, n, \
                     flags, ok, verdict, seg_len, image, gsz, filt, gate, epoch)
  if (host) {
    if (fcs) {
      if (filt.on) LNX_RV(true, true, true); else LNX_RV(true, false, true);
    } else {
      if (filt.on) LNX_RV(false, true, true); else LNX_RV(false, false, true);
    }
  } else {
    if (fcs) {
      if (filt.on) LNX_RV(true, true, false); else LNX_RV(true, false, false);
    } else {
      if (filt.on) LNX_RV(false, true, false); else LNX_RV(false, false, false);
    }
  }
#undef LNX_RV
  return hipGetLastError();
}

}  // namespace lnx
