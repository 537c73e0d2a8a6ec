// Microbenchmarks that decide the CRC-32 kernel's shape on gfx950:
//   1. streaming-read bandwidth by load width (dword / dwordx2 / dwordx4) and
//      by occupancy (many small workgroups vs one 1024-thread workgroup per CU
//      holding 160 KiB of LDS, which is what the CRC kernel needs);
//   2. LDS table-lookup rate for data-dependent indices: lane-private
//      replicated tables (bank = lane % 32) vs one shared table.
// Not part of the product; results are recorded in DESIGN.md.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

template <int W>
struct Vec;
template <> struct Vec<1> { typedef uint32_t T; };
template <> struct Vec<2> { typedef uint2 T; };
template <> struct Vec<4> { typedef uint4 T; };

__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }

// Grid-stride read with UNROLL independent loads in flight per thread.
template <int W, int UNROLL, bool BIGLDS>
__global__ void __launch_bounds__(1024) rd_kernel(const typename Vec<W>::T* __restrict__ p,
                                                  size_t n, uint32_t* out) {
  typedef typename Vec<W>::T T;
  __shared__ uint32_t pad[BIGLDS ? 40960 : 1];
  size_t tid = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  size_t i = tid;
  for (; i + (UNROLL - 1) * stride < n; i += UNROLL * stride) {
    T v[UNROLL];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) v[u] = p[i + u * stride];
#pragma unroll
    for (int u = 0; u < UNROLL; ++u) acc ^= fold(v[u]);
  }
  for (; i < n; i += stride) acc ^= fold(p[i]);
  if (BIGLDS) { pad[threadIdx.x] = acc; __syncthreads(); acc ^= pad[(threadIdx.x + 1) & 1023]; }
  if (acc == 0x12345678u) out[0] = acc;
}

// LDS lookup rate: chained data-dependent lookups; CHAINS independent chains per lane.
// PRIVATE: table replicated 32x so lane l only touches bank l%32.
template <bool PRIVATE, int CHAINS>
__global__ void __launch_bounds__(1024) lds_kernel(const uint32_t* __restrict__ tab, int iters,
                                                   uint32_t* out) {
  __shared__ uint32_t lds[32768];  // 128 KiB: 4 tables x 256 x 32 copies
  for (int i = threadIdx.x; i < 32768; i += blockDim.x) {
    // random-looking values everywhere (both layouts index into this array)
    uint32_t h = (uint32_t)i * 0x9e3779b1u; h ^= h >> 15; h *= 0x85ebca6bu; h ^= h >> 13;
    lds[i] = h ^ tab[i & 1023];
  }
  __syncthreads();
  uint32_t c = threadIdx.x & 31;
  uint32_t st[CHAINS];
#pragma unroll
  for (int k = 0; k < CHAINS; ++k) st[k] = (threadIdx.x * 2654435761u) ^ (k * 0x9e3779b9u) ^ blockIdx.x;
  const uint32_t base0 = c * 4, base1 = c * 4 + 65536;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < CHAINS; ++k) {
      uint32_t x = st[k];
      uint32_t a0, a1, a2, a3;
      if (PRIVATE) {
        // byte b of x -> bits 8..15 of the address; lane column in bits 2..6
        a0 = __builtin_amdgcn_perm(x, base0, 0x0c020400u);
        a1 = __builtin_amdgcn_perm(x, base0, 0x0c020500u);
        a2 = __builtin_amdgcn_perm(x, base1, 0x0c020600u);
        a3 = __builtin_amdgcn_perm(x, base1, 0x0c020700u);
        uint32_t v0 = *(const uint32_t*)((const char*)lds + a0);
        uint32_t v1 = *(const uint32_t*)((const char*)lds + a1 + 128);
        uint32_t v2 = *(const uint32_t*)((const char*)lds + a2);
        uint32_t v3 = *(const uint32_t*)((const char*)lds + a3 + 128);
        st[k] = v0 ^ v1 ^ v2 ^ v3 ^ it;
      } else {
        // shared compact table (4 x 256 dwords)
        uint32_t v0 = lds[(x & 0xff)];
        uint32_t v1 = lds[256 + ((x >> 8) & 0xff)];
        uint32_t v2 = lds[512 + ((x >> 16) & 0xff)];
        uint32_t v3 = lds[768 + (x >> 24)];
        st[k] = v0 ^ v1 ^ v2 ^ v3 ^ it;
      }
    }
  }
  uint32_t acc = 0;
#pragma unroll
  for (int k = 0; k < CHAINS; ++k) acc ^= st[k];
  if (acc == 0x12345678u) out[0] = acc;
}

template <typename F>
float time_ms(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f();
  CK(hipDeviceSynchronize());
  std::vector<float> ts;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(a));
    f();
    CK(hipEventRecord(b));
    CK(hipEventSynchronize(b));
    float ms; CK(hipEventElapsedTime(&ms, a, b)); ts.push_back(ms);
  }
  std::sort(ts.begin(), ts.end());
  return ts[ts.size() / 2];
}

int main() {
  int dev = 0; CK(hipSetDevice(dev));
  hipDeviceProp_t prop; CK(hipGetDeviceProperties(&prop, dev));
  int ncu = prop.multiProcessorCount;
  printf("device %s CUs=%d clock=%d kHz\n", prop.gcnArchName, ncu, prop.clockRate);
  const size_t bytes = (size_t)2 << 30;  // 2 GiB, far beyond the 256 MiB Infinity Cache
  void* buf; CK(hipMalloc(&buf, bytes));
  CK(hipMemset(buf, 0x5a, bytes));
  uint32_t* out; CK(hipMalloc(&out, 64));

#define RUN_RD(W, U, BIG, GRID, BLOCK) do { \
    size_t n = bytes / (4 * W); \
    float ms = time_ms([&] { rd_kernel<W, U, BIG><<<GRID, BLOCK>>>((const Vec<W>::T*)buf, n, out); }, 10); \
    printf("read W=%d unroll=%d biglds=%d grid=%d block=%d : %.3f ms  %.1f GB/s\n", W, U, (int)BIG, (int)(GRID), (int)(BLOCK), ms, bytes / ms / 1e6); \
  } while (0)

  RUN_RD(4, 4, false, ncu * 8, 256);
  RUN_RD(4, 8, false, ncu * 8, 256);
  RUN_RD(2, 8, false, ncu * 8, 256);
  RUN_RD(1, 8, false, ncu * 8, 256);
  RUN_RD(1, 16, false, ncu * 8, 256);
  RUN_RD(4, 4, true, ncu, 1024);
  RUN_RD(4, 8, true, ncu, 1024);
  RUN_RD(2, 8, true, ncu, 1024);
  RUN_RD(1, 8, true, ncu, 1024);
  RUN_RD(1, 16, true, ncu, 1024);
  RUN_RD(1, 8, true, ncu, 512);
  RUN_RD(1, 16, true, ncu, 512);

  std::vector<uint32_t> htab(1024);
  for (int i = 0; i < 1024; ++i) htab[i] = i * 0x9e3779b1u + 12345;
  uint32_t* dtab; CK(hipMalloc(&dtab, 4096));
  CK(hipMemcpy(dtab, htab.data(), 4096, hipMemcpyHostToDevice));
  const int iters = 4096;
#define RUN_LDS(P, C, BLOCK) do { \
    float ms = time_ms([&] { lds_kernel<P, C><<<ncu, BLOCK>>>(dtab, iters, out); }, 5); \
    double looks = (double)ncu * BLOCK * C * iters * 4; \
    printf("lds private=%d chains=%d block=%d : %.3f ms  %.2f Glookups/s  %.2f lookups/clk/CU @2.4GHz\n", (int)P, C, BLOCK, ms, looks / ms / 1e6, looks / (ms * 1e-3) / ncu / 2.4e9); \
  } while (0)
  RUN_LDS(true, 1, 1024);
  RUN_LDS(true, 2, 1024);
  RUN_LDS(true, 4, 1024);
  RUN_LDS(true, 2, 512);
  RUN_LDS(true, 4, 512);
  RUN_LDS(false, 1, 1024);
  RUN_LDS(false, 2, 1024);
  RUN_LDS(false, 4, 1024);
  CK(hipFree(buf));
  return 0;
}
