// dispatch.hpp — which kernel folds each workgroup slice of an offsets batch
// (round 5).
//
// lnx_crc32_batch / lnx_fcs_verify_batch launch the rows kernel
// (crc32_kernel.hip) and then the staged kernel (stage_kernel.hip) over the
// SAME partition of the frame index range into slices.  Every workgroup of
// both launches classifies its own slice with slice_kind() — the same integer
// function of the same offsets, so the two launches agree without talking —
// and a workgroup whose slice belongs to the other kernel exits at once.  The
// library never reads device-resident offsets on the host, so the choice costs
// no sync; the second launch costs about 2 us when it has nothing to do
// (tools/ubench/dispatch_pair.hip, profiles/r5a_dispatch_pair.txt).
//
//  * kSliceRows: the frames are (nearly) all one length and the rows kernel
//    is faster at that length (the measured sweep, profiles/r5a_mean_sweep.jsonl:
//    fixed 1024 B and up, and 176-576 B);
//  * kSliceStage: any other mix (every mixed-length distribution measured ran
//    faster staged, 8-70 %);
//  * kSliceGiant: the slice's bytes do not fit 31-bit buffer offsets (frames
//    of gigabytes), or its frames average 1 MiB or more, or it spans 16 MiB or
//    more at 8 times the batch's mean frame length.  All workgroups of
//    the staged launch fold such slices together in byte pieces
//    (stage_kernel.hip giant_pieces).
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lnx {

constexpr uint32_t kSliceNone = 0, kSliceRows = 1, kSliceStage = 2, kSliceGiant = 3;
// policy: kPolicyAuto (the plain entries), kPolicyShort (LNX_BATCH_SHORT_FRAMES:
// every slice that fits goes to the staged kernel), kPolicyRows (the rows
// kernel owns every slice: segment mode, TX append, profiling variants)
constexpr uint32_t kPolicyAuto = 0, kPolicyShort = 1, kPolicyRows = 2;
// a slice whose span plus line alignment reaches this is giant (the staged
// kernel's blocks address bytes by 31-bit buffer offsets from a line-aligned
// base; the margin covers the 16-byte rounding of the range)
constexpr uint64_t kGiantSpan = (1ull << 31) - (1ull << 20);
// a slice whose frames average this many bytes or more is giant too: a few
// frames of many megabytes would each be one wave's serial stream otherwise
constexpr uint64_t kGiantMean = 1ull << 20;
// frames counted as one length: lengths of the 64 sampled frames within this
// many bytes of each other
constexpr uint32_t kUniformSpread = 8;

// a slice is giant as well when it spans kGiantBig bytes or more and its
// frames average kGiantSkew times the batch's mean or more: a few large frames
// among many short ones (a 1.9 GB frame among 65 536 Zipf frames is neither
// giant by span nor by mean, and one staged block, one wave, would stream it)
constexpr uint64_t kGiantBig = 16ull << 20;
constexpr uint64_t kGiantSkew = 8;

// Whether a slice of nf frames spanning `span` bytes from a base `adj` bytes
// into its 128-byte line is giant, in a batch whose frames average `gmean`
// bytes (both launches and every workgroup of the staged one evaluate this on
// the same offsets).
__host__ __device__ constexpr bool slice_is_giant(uint64_t span, uint64_t adj, uint64_t nf, uint64_t gmean) {
  return nf > 0 &&
         (span + adj >= kGiantSpan || span >= nf * kGiantMean || (span >= kGiantBig && span >= nf * kGiantSkew * gmean));
}

// The batch's mean frame length (off[n] - off[0]) / n, 0 when off[n] < off[0]
// (every workgroup of both launches: the same value).
__device__ __forceinline__ uint64_t batch_mean(const uint64_t* off, uint64_t n) {
  const uint64_t o0 = off[0], on = off[n];
  return on > o0 ? (on - o0) / n : 0;
}

// The partition both launches use: grid = min(#CU, ceil(n / 64)) workgroups,
// slice w = frames [w * per, min(n, (w + 1) * per)), per a multiple of 16
// (the rows kernel's 16 waves per workgroup).
struct SlicePlan {
  uint64_t grid, per;
};
inline SlicePlan slice_plan(uint64_t n, int num_cus) {
  uint64_t grid = (n + 63) / 64;
  if (grid > (uint64_t)num_cus) grid = (uint64_t)num_cus;
  if (grid == 0) grid = 1;
  const uint64_t fpw = (n + grid * 16 - 1) / (grid * 16);
  return {grid, fpw * 16};
}

// Rows or staged for a slice of equal-length frames of `mean` bytes.
__host__ __device__ constexpr bool rows_length(uint64_t mean) {
  return mean >= 960 || (mean >= 176 && mean < 576);
}

// Kind of slice [fb0, fb1) (wave-uniform: every lane returns the same value).
// Reads off[fb0], off[fb1] and the lengths of 64 frames evenly spaced over the
// slice.  A sampled end below its start (offsets out of order) sends the slice
// to the rows kernel, whose per-frame windows treat such a frame as empty.
__device__ __forceinline__ uint32_t slice_kind(const uint8_t* bytes, const uint64_t* __restrict__ off, uint64_t fb0,
                                               uint64_t fb1, uint32_t policy, uint64_t gmean) {
  if (fb1 <= fb0) return kSliceNone;
  const uint64_t o0 = off[fb0], o1 = off[fb1];
  const uint64_t span = o1 > o0 ? o1 - o0 : 0;
  const uint64_t adj = (reinterpret_cast<uintptr_t>(bytes) + o0) & 127u;
  if (slice_is_giant(span, adj, fb1 - fb0, gmean)) return kSliceGiant;
  if (policy == kPolicyShort) return kSliceStage;
  const uint64_t nf = fb1 - fb0;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t i = nf >= 64 ? (uint64_t)lane * (nf / 64) : (lane < nf ? lane : nf - 1);
  const uint64_t a = off[fb0 + i], b = off[fb0 + i + 1];
  const uint32_t len = b < a ? 0xFFFFFFFFu : (b - a > 0xFFFFFFF0ull ? 0xFFFFFFF0u : (uint32_t)(b - a));
  uint32_t mn = len, mx = len;
#pragma unroll
  for (int s = 1; s < 64; s <<= 1) {
    const uint32_t on = (uint32_t)__shfl_xor((int)mn, s), ox = (uint32_t)__shfl_xor((int)mx, s);
    mn = on < mn ? on : mn;
    mx = ox > mx ? ox : mx;
  }
  mn = (uint32_t)__builtin_amdgcn_readfirstlane((int)mn);
  mx = (uint32_t)__builtin_amdgcn_readfirstlane((int)mx);
  if (mx == 0xFFFFFFFFu) return kSliceRows;  // offsets out of order
  const uint64_t mean = span / nf;
  return (mx - mn <= kUniformSpread && rows_length(mean)) ? kSliceRows : kSliceStage;
}

}  // namespace lnx
