// What a kernel pays to patch frames in place in pinned host memory (the
// zero-copy egress path): 1 M slots of 1536 B, each patched by
//   mode 0: one 4-byte store (an FCS)
//   mode 1: four 2-byte stores at offsets 16, 24, 38, 40 (IPv4 length and
//           checksum, UDP length and checksum) plus a 4-byte FCS store
//   mode 2: one 16-byte store
//   mode 3: 64 contiguous bytes per slot by 4 adjacent lanes (16 B each)
//   mode 4: read 256 B per slot (16 lanes x 16 B), no store (the read side)
// by one lane per slot (modes 0-2) or as stated, with hipEvent timing.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/host_write.hip -o tools/ubench/host_write
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>

__global__ void patch(uint8_t* __restrict__ slots, uint32_t n, uint32_t cap, int mode, uint32_t* sink) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (mode <= 2) {
    if (t >= n) return;
    uint8_t* s = slots + (size_t)t * cap;
    if (mode == 0) {
      *reinterpret_cast<uint32_t*>(s + 1500) = t;
    } else if (mode == 1) {
      *reinterpret_cast<uint16_t*>(s + 16) = (uint16_t)t;
      *reinterpret_cast<uint16_t*>(s + 24) = (uint16_t)(t + 1);
      *reinterpret_cast<uint16_t*>(s + 38) = (uint16_t)(t + 2);
      *reinterpret_cast<uint16_t*>(s + 40) = (uint16_t)(t + 3);
      *reinterpret_cast<uint32_t*>(s + 1500) = t;
    } else {
      *reinterpret_cast<uint4*>(s + 16) = make_uint4(t, t + 1, t + 2, t + 3);
    }
  } else if (mode == 3) {
    const uint32_t f = t >> 2, q = t & 3u;
    if (f >= n) return;
    *reinterpret_cast<uint4*>(slots + (size_t)f * cap + 16u * q) = make_uint4(t, t + 1, t + 2, t + 3);
  } else {
    const uint32_t f = t >> 4, q = t & 15u;
    if (f >= n) return;
    const uint4 v = *reinterpret_cast<const uint4*>(slots + (size_t)f * cap + 16u * q);
    if ((v.x ^ v.y ^ v.z ^ v.w) == 0x12345678u) sink[0] = t;
  }
}

int main() {
  const uint32_t n = 1u << 20, cap = 1536;
  uint8_t* h = nullptr;
  uint32_t* sink = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&h), (size_t)n * cap, hipHostMallocDefault) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&sink), 4) != hipSuccess) {
    fprintf(stderr, "alloc failed\n");
    return 1;
  }
  memset(h, 0, (size_t)n * cap);
  uint8_t* d = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) return 1;
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const char* names[] = {"4 B store", "4 x 2 B + 4 B stores", "16 B store", "64 B by 4 lanes", "256 B read by 16 lanes"};
  const uint32_t lanes[] = {1, 1, 1, 4, 16};
  for (int mode = 0; mode < 5; ++mode) {
    const uint32_t threads = n * lanes[mode];
    const uint32_t grid = (threads + 255) / 256;
    float best = 1e9f;
    for (int rep = 0; rep < 6; ++rep) {
      hipEventRecord(a, 0);
      hipLaunchKernelGGL(patch, dim3(grid), dim3(256), 0, 0, d, n, cap, mode, sink);
      hipEventRecord(b, 0);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      if (rep > 0 && ms < best) best = ms;
    }
    printf("{\"mode\": %d, \"what\": \"%s\", \"slots\": %u, \"ms\": %.3f, \"Mslots_per_s\": %.1f}\n", mode, names[mode], n,
           best, n / best / 1e3);
    fflush(stdout);
  }
  if (h[1500] != 0 && *reinterpret_cast<uint32_t*>(h + 1536 + 1500) != 1u) printf("{\"check\": \"unexpected\"}\n");
  hipHostFree(h);
  hipFree(sink);
  return 0;
}
