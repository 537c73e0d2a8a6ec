// Does the page size behind pinned host memory change what a kernel reads over
// PCIe in place (the ring's zero-copy path)?  The same 1.5 GB
// of slots allocated three ways -- hipHostMalloc; mmap + MADV_HUGEPAGE +
// hipHostRegister; mmap + MADV_NOHUGEPAGE + hipHostRegister -- each read by the
// receive rows' pattern (256 B per slot, 16 lanes x 2 x 8 B) and by 16 lanes x
// 16 B, with the process's AnonHugePages after each allocation.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/host_pages.hip -o tools/ubench/host_pages
#include <hip/hip_runtime.h>
#include <sys/mman.h>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <string>

__global__ void rd(const uint8_t* __restrict__ slots, uint32_t n, uint32_t cap, int mode, uint32_t* sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t f = t >> 4, q = t & 15u;
  if (f >= n) return;
  uint32_t x;
  if (mode == 0) {
    const uint2 v = *reinterpret_cast<const uint2*>(slots + (size_t)f * cap + 8u * q);
    const uint2 w = *reinterpret_cast<const uint2*>(slots + (size_t)f * cap + 128u + 8u * q);
    x = v.x ^ v.y ^ w.x ^ w.y;
  } else {
    const uint4 v = *reinterpret_cast<const uint4*>(slots + (size_t)f * cap + 16u * q);
    x = v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) sink[0] = t;
}

static long anon_huge_kb() {
  std::ifstream f("/proc/self/smaps_rollup");
  std::string k;
  long v;
  while (f >> k) {
    if (k == "AnonHugePages:") {
      f >> v;
      return v;
    }
  }
  return -1;
}

int main() {
  const uint32_t n = 1u << 20, cap = 1536;
  const size_t bytes = (size_t)n * cap;
  uint32_t* sink = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&sink), 4) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  {
    std::ifstream t("/sys/kernel/mm/transparent_hugepage/enabled");
    std::string s;
    std::getline(t, s);
    printf("{\"thp_enabled\": \"%s\"}\n", s.c_str());
  }
  const char* names[] = {"hipHostMalloc", "mmap+MADV_HUGEPAGE+hipHostRegister", "mmap+MADV_NOHUGEPAGE+hipHostRegister"};
  for (int how = 0; how < 3; ++how) {
    uint8_t* h = nullptr;
    const long before = anon_huge_kb();
    if (how == 0) {
      if (hipHostMalloc(reinterpret_cast<void**>(&h), bytes, hipHostMallocDefault) != hipSuccess) return 2;
    } else {
      void* m = mmap(nullptr, bytes + (2u << 20), PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (m == MAP_FAILED) return 3;
      h = reinterpret_cast<uint8_t*>(((uintptr_t)m + (2u << 20) - 1) & ~(uintptr_t)((2u << 20) - 1));
      madvise(h, bytes, how == 1 ? MADV_HUGEPAGE : MADV_NOHUGEPAGE);
      memset(h, 1, bytes);
      if (hipHostRegister(h, bytes, hipHostRegisterMapped) != hipSuccess) return 4;
    }
    memset(h, 0, bytes);
    const long after = anon_huge_kb();
    uint8_t* d = nullptr;
    if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) return 5;
    for (int mode = 0; mode < 2; ++mode) {
      float best = 1e9f;
      for (int rep = 0; rep < 6; ++rep) {
        hipEventRecord(a, 0);
        hipLaunchKernelGGL(rd, dim3(n * 16 / 256), dim3(256), 0, 0, d, n, cap, mode, sink);
        hipEventRecord(b, 0);
        hipEventSynchronize(b);
        float ms = 0;
        hipEventElapsedTime(&ms, a, b);
        if (rep > 0 && ms < best) best = ms;
      }
      printf("{\"alloc\": \"%s\", \"anon_huge_mb\": %ld, \"mode\": %d, \"ms\": %.3f, \"GB_per_s\": %.1f}\n", names[how],
             (after - before) / 1024, mode, best, n * 256.0 / best / 1e6);
      fflush(stdout);
    }
    if (how == 0) hipHostFree(h);
    else hipHostUnregister(h);
  }
  hipFree(sink);
  return 0;
}
