// Device-scope returning atomic add on a few counters: chip-wide throughput
// and latency, to size any work-stealing scheme for the CRC kernel (DESIGN.md
// §3.1 "work distribution").  G workgroups x W waves; lane 0 of every wave
// does K dependent fetch_adds on counter (block % NC), counters 4 KiB apart.
// Latency per atomic from s_memrealtime (100 MHz).  Not part of the product.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

__global__ void __launch_bounds__(1024) atom(uint64_t* ctr, int nc, int k, uint64_t* lat, int waves_per_block) {
  const int wave = threadIdx.x >> 6;
  if (wave >= waves_per_block) return;
  if ((threadIdx.x & 63) != 0) return;
  uint64_t* c = ctr + (size_t)(blockIdx.x % nc) * 512;
  uint64_t acc = 0, t = 0;
  for (int i = 0; i < k; ++i) {
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    acc += __hip_atomic_fetch_add(c, (uint64_t)1 + (acc & 0), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    t += __builtin_amdgcn_s_memrealtime() - t0;
  }
  lat[blockIdx.x * 16 + wave] = t | (acc & 0);
}

int main() {
  uint64_t *ctr, *lat;
  (void)hipMalloc(&ctr, 64 * 4096);
  (void)hipMalloc(&lat, 256 * 16 * 8);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  struct Cfg {
    int nc, k, wpb;
  };
  for (Cfg c : {Cfg{1, 4, 16}, Cfg{1, 16, 16}, Cfg{8, 4, 16}, Cfg{8, 16, 16}, Cfg{64, 16, 16}, Cfg{256, 16, 16},
                Cfg{1, 16, 1}, Cfg{8, 16, 1}, Cfg{1, 64, 1}, Cfg{8, 64, 1}}) {
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipMemset(ctr, 0, 64 * 4096);
      (void)hipMemset(lat, 0, 256 * 16 * 8);
      (void)hipEventRecord(a);
      hipLaunchKernelGGL(atom, dim3(256), dim3(1024), 0, 0, ctr, c.nc, c.k, lat, c.wpb);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      std::vector<uint64_t> l(256 * 16);
      (void)hipMemcpy(l.data(), lat, l.size() * 8, hipMemcpyDeviceToHost);
      std::vector<double> per;
      for (int i = 0; i < 256; ++i)
        for (int w = 0; w < c.wpb; ++w) per.push_back(l[i * 16 + w] * 10.0 / c.k);  // ns per atomic
      std::sort(per.begin(), per.end());
      const double total = 256.0 * c.wpb * c.k;
      if (rep == 2)
        printf("counters %3d  waves/WG %2d  atomics/wave %2d : %7.1f us total, %6.1f ns/atomic chip-wide, "
               "latency p50 %7.0f ns  p99 %7.0f ns\n",
               c.nc, c.wpb, c.k, ms * 1e3, ms * 1e6 / total, per[per.size() / 2], per[per.size() * 99 / 100]);
    }
  }
  return 0;
}
