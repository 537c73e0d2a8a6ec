// Does the memory pipeline pay for lanes that load nothing?  The narrow
// (4-lane) CRC rows issue every step's load for all 16 rows of a wave and
// give the rows past their item's end an out-of-range offset; on the Zipf mix
// that is about half the lane-loads.  Here 16 rows of 4 lanes
// each read 16 contiguous bytes per instruction at scattered positions (the
// narrow rows' shape), with only A of the 16 rows wanting data:
//   oob  : every lane issues; rows that want nothing use an out-of-range offset
//   exec : rows that want nothing are masked off (exec), the instruction issues
//          for the others
//   pack : the A active rows' loads packed into fewer full instructions (the
//          ideal: instructions x A/16)
// Not part of the product.  usage: exec_mask
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

constexpr uint32_t kOOB = 0x80000000u;
constexpr int kSteps = 64;  // row steps per wave (16 B each)

template <int MODE, int A>
__global__ void __launch_bounds__(1024) k(const uint8_t* base, uint32_t nbytes, uint32_t* out) {
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nbytes, 0x00020000);
  const uint32_t lane = threadIdx.x & 63, p = lane & 3, row = lane >> 2;
  const uint32_t gw = blockIdx.x * 16 + (threadIdx.x >> 6);
  uint32_t acc = 0;
  // rows sit 4 KiB + 16 B apart (different lines and channels), waves 64 KiB apart
  const uint32_t wbase = (gw * 65536u) % (nbytes - 65536u * 2);
  const bool want = row < (uint32_t)A;
  if constexpr (MODE == 2) {
    // pack: the same bytes, A/16 of the instructions with every row active
    constexpr int N = kSteps * A / 16;
#pragma unroll 8
    for (int s = 0; s < N; ++s) {
      const uint32_t rr = (uint32_t)(s * 16 + row) % A, ss = (uint32_t)(s * 16 + row) / A;
      const uint32_t o = wbase + rr * 4112u + ss * 16u + p * 4u;
      acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0);
    }
  } else {
#pragma unroll 8
    for (int s = 0; s < kSteps; ++s) {
      const uint32_t o = wbase + row * 4112u + s * 16u + p * 4u;
      if constexpr (MODE == 0) {
        acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, want ? o : kOOB, 0, 0);
      } else {
        if (want) acc ^= __builtin_amdgcn_raw_buffer_load_b32(r, o, 0, 0);
      }
    }
  }
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
float tm(F fn) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) fn();
  (void)hipDeviceSynchronize();
  std::vector<float> t;
  for (int k = 0; k < 9; ++k) {
    (void)hipEventRecord(a);
    for (int i = 0; i < 10; ++i) fn();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    t.push_back(ms / 10);
  }
  std::sort(t.begin(), t.end());
  return t[4];
}

int main() {
  const uint32_t nbytes = 1u << 30;
  uint8_t* buf;
  uint32_t* out;
  (void)hipMalloc(&buf, nbytes);
  (void)hipMalloc(&out, 64);
  (void)hipMemset(buf, 1, nbytes);
  const dim3 g(256 * 16), blk(1024);
  const double waves = 256.0 * 16 * 16;
#define RUN(A)                                                                                              \
  {                                                                                                         \
    const float t0 = tm([&] { k<0, A><<<g, blk>>>(buf, nbytes, out); });                                   \
    const float t1 = tm([&] { k<1, A><<<g, blk>>>(buf, nbytes, out); });                                   \
    const float t2 = tm([&] { k<2, A><<<g, blk>>>(buf, nbytes, out); });                                   \
    const double useful = waves * kSteps * A * 16.0;                                                        \
    printf("active rows %2d/16: oob %.4f ms (%.0f GB/s useful)  exec %.4f ms (%.0f)  pack %.4f ms (%.0f)\n", A, \
           t0, useful / t0 / 1e6, t1, useful / t1 / 1e6, t2, useful / t2 / 1e6);                          \
  }
  RUN(16);
  RUN(8);
  RUN(4);
  RUN(2);
  return 0;
}
