// Audit fixture (tests/test_kernel_audit.py): the round-1 r1g sum16 line-row
// kernel in the form that returned wrong sums on MI355X: the
// line loop bounded by each row's own count (divergent exits, exec-masked
// dwordx2 loads).  Rebuilt from commit 68eb888 with `k0 < nl` for the loop
// bound; not part of any library.
// sum16_kernel.hip — batched RFC 791/1071 internet checksum (lneto CRC791), gfx950.
//
// Reference: CRC791{sum}.PayloadSum16(buff) (lneto crc.go:52-59):
//   sum += BE16(buff[i:]) for even i  (uint32, wrap-around; sumWriteEven crc.go:23-28)
//   odd length: sum += last << 8
//   return ^fold(fold(sum))            (sum16, crc.go:17-21)
// Bit-exact reformulation used here: with E = sum of the bytes at EVEN offsets
// from the segment start and O = sum of the bytes at ODD offsets,
//   sum_final = seed + 256*E + O   (mod 2^32)
// — the odd trailing byte is an even-offset byte with weight 256, exactly the
// `<< 8` of crc.go:56.  Addition mod 2^32 is associative, so any lane/wave
// split of the bytes gives the identical uint32 before the folds.
//
// One 16-lane row per segment (four segments per wave); lane p reads aligned
// dwords p, p+16, ... in batches; bytes outside the segment are masked;
// v_dot4_u32_u8 forms the even/odd byte sums, DPP adds reduce the row.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lnx {

constexpr int kSumBlock = 256;
constexpr int kSumWaves = kSumBlock / 64;

__device__ __forceinline__ uint16_t fold_sum16(uint32_t sum) {
  sum = (sum & 0xffffu) + (sum >> 16);
  return (uint16_t)~(uint16_t)(sum + (sum >> 16));
}

constexpr int kSumRowLanes = 16;  // one segment per 16-lane row, four per wave
constexpr int kSumUnroll = 8;     // dwords per lane in flight per batch (512 B per row)

__device__ __forceinline__ uint32_t sum_keep_from(int32_t lo) {
  lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
  return (uint32_t)(0xFFFFFFFFull << (8 * lo));
}

__device__ __forceinline__ uint32_t row_add16(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return v;
}

// One 16-lane row per segment: lane p reads aligned dwords p, p+16, ... of the
// segment's aligned span, kSumUnroll at a time, masks the bytes outside the
// Line rows (round 1, r1g): the same row-per-segment split, but lane p loads
// 8 bytes (global_load_dwordx2 nt) at 8p + 128k of the segment's 128-byte
// aligned span, so every row instruction reads one whole line — the pattern
// whose non-temporal streaming rate is 6.4-6.5 TB/s against 6.0 for the
// 64-byte half lines above (DESIGN.md §3.1 "whole-line rows").  kLineUnroll
// lines per row in flight.
constexpr int kLineUnroll = 8;

__device__ __forceinline__ uint64_t keep8(int32_t d) {  // bytes [d, 8) of a qword, d clamped to 0..8
  const uint32_t q = 4u * (uint32_t)(d < 0 ? 0 : (d > 8 ? 8 : d));
  return (~0ull << q) << q;
}

template <bool NT>
__global__ void __launch_bounds__(kSumBlock)
sum16_lines_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                   const uint32_t* __restrict__ len, const uint32_t* __restrict__ seed, uint64_t nseg,
                   uint16_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u, p = lane & 15u, row = lane >> 4;
  const uint64_t nwaves = (uint64_t)gridDim.x * kSumWaves;
  for (uint64_t q = (uint64_t)blockIdx.x * kSumWaves + (threadIdx.x >> 6); q * 4 < nseg; q += nwaves) {
    const uint64_t i = q * 4 + row;
    const bool live = i < nseg;
    const uint64_t s = live ? off[i] : 0;
    const uint32_t L = live ? len[i] : 0u;
    const uint32_t sd = live && seed ? seed[i] : 0u;
    const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(bytes) + s) & 127u);
    const uint64_t* base = reinterpret_cast<const uint64_t*>(bytes + s - mis) + p;
    const uint32_t nl = L ? (mis + L + 127u) >> 7 : 0u;  // lines touching the segment
    const uint32_t wE = (mis & 1u) ? 0x01000100u : 0x00010001u;
    const uint32_t wO = (mis & 1u) ? 0x00010001u : 0x01000100u;
    uint32_t E = 0, O = 0;
    // One wave-uniform loop over the largest line count of the four rows.  A
    // loop bounded by each row's own count (divergent exits, a scalar line
    // counter, exec-masked loads) came out wrong for ~1 % of the segments of
    // workgroups 256 and up, differently each launch, on MI355X
    // (tools/debug/dbg_sum16.py); this form never did.
    uint32_t nlw = max(nl, (uint32_t)__shfl_xor((int)nl, 16));
    nlw = max(nlw, (uint32_t)__shfl_xor((int)nlw, 32));
    nlw = (uint32_t)__builtin_amdgcn_readfirstlane((int)nlw);
    for (uint32_t k0 = 0; k0 < nl; k0 += kLineUnroll) {
      uint64_t x[kLineUnroll];
#pragma unroll
      for (int u = 0; u < kLineUnroll; ++u)
        x[u] = k0 + u < nl ? (NT ? __builtin_nontemporal_load(base + 16u * (k0 + u)) : base[16u * (k0 + u)]) : 0ull;
#pragma unroll
      for (int u = 0; u < kLineUnroll; ++u) {
        const int32_t o0 = (int32_t)(128u * (k0 + u) + 8u * p) - (int32_t)mis;  // segment offset of byte 0
        const uint64_t y = x[u] & keep8(-o0) & ~keep8((int32_t)L - o0);
        E = __builtin_amdgcn_udot4((uint32_t)y, wE, E, false);
        O = __builtin_amdgcn_udot4((uint32_t)y, wO, O, false);
        E = __builtin_amdgcn_udot4((uint32_t)(y >> 32), wE, E, false);
        O = __builtin_amdgcn_udot4((uint32_t)(y >> 32), wO, O, false);
      }
    }
    E = row_add16(E);
    O = row_add16(O);
    if (live && p == 0) out[i] = fold_sum16(sd + 256u * E + O);
  }
}

template __global__ void sum16_lines_kernel<true>(const uint8_t*, const uint64_t*, const uint32_t*, const uint32_t*, uint64_t, uint16_t*);
}  // namespace lnx
