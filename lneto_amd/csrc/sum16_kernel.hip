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
// One wave per segment; lane l reads aligned dwords l, l+64, ...; bytes outside
// the segment are masked; v_dot4_u32_u8 forms the even/odd byte sums.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lnx {

constexpr int kSumBlock = 256;
constexpr int kSumWaves = kSumBlock / 64;

__device__ __forceinline__ uint32_t wave_add(uint32_t v) {
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);
  v += (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);
  return (uint32_t)(__builtin_amdgcn_readlane((int)v, 0) + __builtin_amdgcn_readlane((int)v, 16) +
                    __builtin_amdgcn_readlane((int)v, 32) + __builtin_amdgcn_readlane((int)v, 48));
}

__device__ __forceinline__ uint16_t fold_sum16(uint32_t sum) {
  sum = (sum & 0xffffu) + (sum >> 16);
  return (uint16_t)~(uint16_t)(sum + (sum >> 16));
}

__global__ void __launch_bounds__(kSumBlock)
sum16_segments_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                      const uint32_t* __restrict__ len, const uint32_t* __restrict__ seed,
                      uint64_t nseg, uint16_t* __restrict__ out) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave0 = (uint64_t)blockIdx.x * kSumWaves + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = (uint64_t)gridDim.x * kSumWaves;
  const uintptr_t base = reinterpret_cast<uintptr_t>(bytes);
  for (uint64_t i = wave0; i < nseg; i += nwaves) {
    const uint64_t s = off[i];
    const uint64_t e = s + len[i];
    const uint32_t mis = (uint32_t)((base + s) & 3u);
    const uint64_t a0 = s - mis;                     // first aligned dword of the segment
    const uint64_t nd = e > s ? (e - a0 + 3) >> 2 : 0;  // dwords touching [s, e)
    // Even-offset bytes sit at dword byte positions {0,2} when the segment
    // starts at an even address, {1,3} when it starts at an odd one.
    const uint32_t even_w = (mis & 1u) ? 0x01000100u : 0x00010001u;
    const uint32_t odd_w = (mis & 1u) ? 0x00010001u : 0x01000100u;
    uint32_t acc = 0;
    for (uint64_t k = lane; k < nd; k += 64) {
      const uint64_t pos = a0 + 4 * k;
      uint32_t w = *reinterpret_cast<const uint32_t*>(bytes + pos);
      const int32_t lo = pos < s ? (int32_t)(s - pos) : 0;
      const int32_t hi = (pos + 4 > e) ? (int32_t)(e - pos) : 4;
      w &= (uint32_t)((0xFFFFFFFFull << (8 * lo)) & ~(0xFFFFFFFFull << (8 * hi)));
      const uint32_t ev = __builtin_amdgcn_udot4(w, even_w, 0u, false);
      const uint32_t od = __builtin_amdgcn_udot4(w, odd_w, 0u, false);
      acc += (ev << 8) + od;
    }
    const uint32_t total = wave_add(acc) + (seed ? seed[i] : 0u);
    if (lane == 0) out[i] = fold_sum16(total);
  }
}

hipError_t launch_sum16_segments(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                                  const uint32_t* seed, uint64_t n, uint16_t* out, int num_cus,
                                  hipStream_t stream) {
  if (n == 0) return hipSuccess;
  uint64_t grid = (n + kSumWaves - 1) / kSumWaves;
  const uint64_t cap = (uint64_t)num_cus * 8;
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL(sum16_segments_kernel, dim3((unsigned)grid), dim3(kSumBlock), 0, stream, bytes,
                     off, len, seed, n, out);
  return hipGetLastError();
}

}  // namespace lnx
