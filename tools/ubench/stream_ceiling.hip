// Chip-wide streaming-read ceiling on gfx950: which way of reading a
// once-touched 1.5 GB buffer (the 1 M x 1500 B batch) moves bytes fastest?
//   reg      global_load_dwordx4 into VGPRs, default cache policy
//   reg-nt   the same with the nontemporal hint
//   glds     LDS-DMA (global_load_lds_dwordx4) into a per-wave LDS ring, default policy
//   glds-nt  the same with aux = 2 (nt)
// Each variant at one 1024-thread workgroup per CU (what the CRC kernel's
// 160 KiB LDS image forces) and at several smaller shapes.  The checksum keeps
// the compiler from dropping loads.  Not part of the product.
// build: hipcc --offload-arch=gfx950 -O3 -o stream_ceiling stream_ceiling.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                                        \
  do {                                                                                               \
    hipError_t e_ = (x);                                                                             \
    if (e_ != hipSuccess) {                                                                          \
      fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__);         \
      exit(1);                                                                                       \
    }                                                                                                \
  } while (0)

// Each wave owns a contiguous span of the buffer (like a frame range) and
// sweeps it 1 KiB per wave-instruction, U instructions in flight.
template <int U, bool NT>
__global__ void __launch_bounds__(1024) reg_kernel(const uint4* __restrict__ p, uint64_t n16, uint64_t span16,
                                                   uint32_t* out) {
  const uint64_t wave = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const uint32_t lane = threadIdx.x & 63;
  uint64_t i = wave * span16, end = std::min<uint64_t>(i + span16, n16);
  uint32_t acc = 0;
  for (; i + U * 64 <= end; i += U * 64) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint4* q = p + i + u * 64 + lane;
      if constexpr (NT) {
        typedef uint32_t v4u __attribute__((ext_vector_type(4)));
        const v4u t = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(q));
        v[u] = uint4{t.x, t.y, t.z, t.w};
      } else {
        v[u] = *q;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  for (; i + lane < end; i += 64) acc ^= p[i + lane].x;
  if (acc == 0x12345678u) out[0] = acc;
}

// LDS-DMA: each wave has a ring of R 1 KiB slots in LDS and keeps R-1 in flight.
template <int R, int AUX, int WPB>
__global__ void __launch_bounds__(WPB * 64) glds_kernel(const uint4* __restrict__ p, uint64_t n16, uint64_t span16,
                                                        uint32_t* out) {
  __shared__ __attribute__((aligned(16))) uint32_t ring[WPB * R * 256];
  const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * WPB + wv;
  uint64_t i = wave * span16, end = std::min<uint64_t>(i + span16, n16);
  uint32_t* my = ring + wv * R * 256;
  uint32_t acc = 0;
  int slot = 0;
  for (; i + 64 <= end; i += 64) {
    __builtin_amdgcn_global_load_lds(p + i + lane, my + slot * 256, 16, 0, AUX);
    slot = slot + 1 == R ? 0 : slot + 1;
    // keep R-1 pieces in flight; touch one word of the oldest landed slot now and then
    __builtin_amdgcn_s_waitcnt(0x3f70 | (R - 1));  // vmcnt(R-1), expcnt/lgkmcnt max
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  acc ^= my[lane];
  if (acc == 0x12345678u) out[0] = acc;
}

struct Res {
  const char* name;
  double ms;
};

template <typename F>
double time_it(F&& launch, int reps = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 200; ++i) launch();  // clock ramp
  CK(hipDeviceSynchronize());
  std::vector<float> t;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    launch();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const uint64_t bytes = argc > 1 ? strtoull(argv[1], nullptr, 0) : 1572864000ull;
  const uint64_t n16 = bytes / 16;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  uint4* d;
  uint32_t* out;
  CK(hipMalloc(&d, n16 * 16));
  CK(hipMalloc(&out, 4));
  CK(hipMemset(d, 1, n16 * 16));
  printf("buffer %.3f GB, %d CUs\n", bytes / 1e9, cus);
  auto report = [&](const char* name, double ms) {
    printf("%-40s %8.4f ms  %7.1f GB/s\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  auto span_of = [&](uint64_t waves) { return ((n16 + waves - 1) / waves + 63) / 64 * 64; };
#define REG(U, NT, WG, TPB)                                                                              \
  do {                                                                                                   \
    const uint64_t waves = (uint64_t)(WG) * (TPB) / 64, sp = span_of(waves);                             \
    double ms = time_it([&] { hipLaunchKernelGGL((reg_kernel<U, NT>), dim3(WG), dim3(TPB), 0, 0, d, n16, sp, out); }); \
    char nm[96];                                                                                         \
    snprintf(nm, sizeof nm, "reg%s U=%d grid=%d x %d", NT ? "-nt" : "", U, (int)(WG), (int)(TPB));      \
    report(nm, ms);                                                                                      \
  } while (0)
#define GLDS(R, AUX, WPB, WG)                                                                            \
  do {                                                                                                   \
    const uint64_t waves = (uint64_t)(WG) * (WPB), sp = span_of(waves);                                  \
    double ms = time_it([&] { hipLaunchKernelGGL((glds_kernel<R, AUX, WPB>), dim3(WG), dim3((WPB) * 64), 0, 0, d, n16, sp, out); }); \
    char nm[96];                                                                                         \
    snprintf(nm, sizeof nm, "glds aux=%d R=%d grid=%d x %d waves", AUX, R, (int)(WG), WPB);            \
    report(nm, ms);                                                                                      \
  } while (0)
  REG(4, false, cus, 1024);
  REG(8, false, cus, 1024);
  REG(4, true, cus, 1024);
  REG(8, true, cus, 1024);
  REG(8, false, cus * 4, 256);
  REG(8, false, cus * 8, 256);
  REG(8, true, cus * 8, 256);
  GLDS(8, 0, 16, cus);
  GLDS(8, 2, 16, cus);
  GLDS(4, 0, 16, cus);
  GLDS(4, 2, 16, cus);
  GLDS(8, 0, 4, cus);
  GLDS(8, 2, 4, cus);
  GLDS(16, 2, 4, cus);
  GLDS(16, 0, 8, cus);
  GLDS(16, 2, 8, cus);
  GLDS(8, 2, 8, cus * 2);
  GLDS(8, 2, 4, cus * 4);
  CK(hipFree(d));
  return 0;
}
