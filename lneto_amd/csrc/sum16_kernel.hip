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
#include <cstdlib>

namespace lnx {

constexpr int kSumBlock = 256;
constexpr int kSumWaves = kSumBlock / 64;

__device__ __forceinline__ uint16_t fold_sum16(uint32_t sum) {
  sum = (sum & 0xffffu) + (sum >> 16);
  return (uint16_t)~(uint16_t)(sum + (sum >> 16));
}

[[maybe_unused]] constexpr int kSumRowLanes = 16;  // one segment per 16-lane row, four per wave
[[maybe_unused]] constexpr int kSumUnroll = 8;     // dwords per lane in flight per batch (512 B per row)

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
// segment and accumulates E and O with v_dot4_u32_u8.
#ifdef LNX_RESEARCH  // the r1c half-line rows (var 1)
__global__ void __launch_bounds__(kSumBlock)
sum16_segments_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                      const uint32_t* __restrict__ len, const uint32_t* __restrict__ seed,
                      uint64_t nseg, uint16_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u, p = lane & 15u, row = lane >> 4;
  const uint64_t nwaves = (uint64_t)gridDim.x * kSumWaves;
  for (uint64_t q = (uint64_t)blockIdx.x * kSumWaves + (threadIdx.x >> 6); q * 4 < nseg; q += nwaves) {
    const uint64_t i = q * 4 + row;
    const bool live = i < nseg;
    const uint64_t s = live ? off[i] : 0;
    const uint32_t L = live ? len[i] : 0u;
    const uint32_t sd = live && seed ? seed[i] : 0u;
    const uint32_t mis = (uint32_t)((reinterpret_cast<uintptr_t>(bytes) + s) & 3u);
    const uint32_t* base = reinterpret_cast<const uint32_t*>(bytes + s - mis);
    const uint32_t nw = L ? (mis + L + 3) >> 2 : 0u;  // dwords touching the segment
    // bytes at even segment offsets sit at dword positions {0,2} when the
    // segment starts 2-aligned, {1,3} otherwise
    const uint32_t wE = (mis & 1u) ? 0x01000100u : 0x00010001u;
    const uint32_t wO = (mis & 1u) ? 0x00010001u : 0x01000100u;
    uint32_t E = 0, O = 0;
    for (uint32_t k0 = p; k0 < nw; k0 += kSumRowLanes * kSumUnroll) {
      uint32_t x[kSumUnroll];
#pragma unroll
      for (int u = 0; u < kSumUnroll; ++u) {
        const uint32_t k = k0 + u * kSumRowLanes;
        x[u] = k < nw ? base[k] : 0u;
      }
#pragma unroll
      for (int u = 0; u < kSumUnroll; ++u) {
        const int32_t o0 = (int32_t)(4 * (k0 + u * kSumRowLanes)) - (int32_t)mis;  // segment offset of byte 0
        const uint32_t y = x[u] & sum_keep_from(-o0) & ~sum_keep_from((int32_t)L - o0);
        E = __builtin_amdgcn_udot4(y, wE, E, false);
        O = __builtin_amdgcn_udot4(y, wO, O, false);
      }
    }
    E = row_add16(E);
    O = row_add16(O);
    if (live && p == 0) out[i] = fold_sum16(sd + 256u * E + O);
  }
}
#endif  // LNX_RESEARCH

// Line rows (round 1, r1g): the same row-per-segment split, but lane p loads
// 8 bytes (global_load_dwordx2 nt) at 8p + 128k of the segment's 128-byte
// aligned span, so every row instruction reads one whole line — the pattern
// whose non-temporal streaming rate is 6.4-6.5 TB/s against 6.0 for the
// 64-byte half lines above (DESIGN.md §3.1 "whole-line rows").  kLineUnroll
// lines per row in flight: 13 covers a 1500-B segment in one round trip
// (6.24 TB/s against 6.07 with 8 and 6.19 with 16, tools/prof/sum16_variants.py).
constexpr int kLineUnroll = 13;

__device__ __forceinline__ uint64_t keep8(int32_t d) {  // bytes [d, 8) of a qword, d clamped to 0..8
  const uint32_t q = 4u * (uint32_t)(d < 0 ? 0 : (d > 8 ? 8 : d));
  return (~0ull << q) << q;
}

// EDGE (with NT): the first line of each batch and its last two (where a
// 12- or 13-line segment ends) are loaded with the default cache policy, the
// rest non-temporally.  Back-to-back segments share a line; a wave's four rows
// ask for it twice within one batch, and with nt the second request found the
// line gone from L2 and fetched it from HBM again (the CRC kernel's lean rows
// showed the same, crc32_kernel.hip lines_body EP).

template <bool NT, int UNR = kLineUnroll, bool EDGE = true>
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
    for (uint32_t k0 = 0; k0 < nlw; k0 += UNR) {
      uint64_t x[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const bool nt = NT && !(EDGE && (u == 0 || u >= UNR - 2));
        x[u] = k0 + u < nl ? (nt ? __builtin_nontemporal_load(base + 16u * (k0 + u)) : base[16u * (k0 + u)]) : 0ull;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
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

// var 0: line rows, edge lines at the default policy (product); var 1: the half-line rows of
// sum16_segments_kernel; var 2: line rows, default cache policy; var 3 / 4: line rows with 8 / 16 lines in
// flight; var 5: line rows all nt (the r1h product)
hipError_t launch_sum16_segments(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                                  const uint32_t* seed, uint64_t n, uint16_t* out, int num_cus,
                                  hipStream_t stream, int var) {
  if (n == 0) return hipSuccess;
  const uint64_t seg_per_block = kSumWaves * 4;
  uint64_t grid = (n + seg_per_block - 1) / seg_per_block;
  // 256 workgroups per CU (one pass of 16 segments each at 1 M segments): 0.237-0.240 ms
  // against 0.259 for 32, 0.248 for 128 (profiles/r1h_grid_sweep.txt).
#ifdef LNX_RESEARCH
  // research library: LNX_PROF_SUM16_WG_PER_CU overrides it, var picks the A/B form
  static const uint64_t wg_per_cu = [] {
    const char* e = getenv("LNX_PROF_SUM16_WG_PER_CU");
    const int v = e ? atoi(e) : 0;
    return (uint64_t)(v > 0 ? v : 256);
  }();
  const uint64_t cap = (uint64_t)num_cus * wg_per_cu;
  if (grid > cap) grid = cap;
  if (var == 1)
    hipLaunchKernelGGL(sum16_segments_kernel, dim3((unsigned)grid), dim3(kSumBlock), 0, stream, bytes,
                       off, len, seed, n, out);
  else if (var == 3)
    hipLaunchKernelGGL((sum16_lines_kernel<true, 8>), dim3((unsigned)grid), dim3(kSumBlock), 0, stream, bytes,
                       off, len, seed, n, out);
  else if (var == 4)
    hipLaunchKernelGGL((sum16_lines_kernel<true, 16>), dim3((unsigned)grid), dim3(kSumBlock), 0, stream, bytes,
                       off, len, seed, n, out);
  else if (var == 2)
    hipLaunchKernelGGL(sum16_lines_kernel<false>, dim3((unsigned)grid), dim3(kSumBlock), 0, stream, bytes, off,
                       len, seed, n, out);
  else if (var == 5)
    hipLaunchKernelGGL((sum16_lines_kernel<true, kLineUnroll, false>), dim3((unsigned)grid), dim3(kSumBlock), 0,
                       stream, bytes, off, len, seed, n, out);
  else
#else
  (void)var;
  const uint64_t cap = (uint64_t)num_cus * 256;
  if (grid > cap) grid = cap;
#endif
    hipLaunchKernelGGL(sum16_lines_kernel<true>, dim3((unsigned)grid), dim3(kSumBlock), 0, stream, bytes, off,
                       len, seed, n, out);
  return hipGetLastError();
}

}  // namespace lnx
