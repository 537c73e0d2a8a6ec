// What a kernel pays to patch frames in place in HBM (the transmit kernels:
// tx_checksum's fields, fcs_append's FCS, tx_finish's row stores; DESIGN.md
// §4): 1 M slots of 1536 B in device memory, each written by
//   mode 0: one 4-byte store at offset 1496 (an FCS), one lane per slot
//   mode 1: 32 bytes at offset 16 by 4 lanes x 8 B (tx_finish's patched qwords 2..5)
//   mode 2: the whole 64-byte block at offset 0 by 8 lanes x 8 B
//   mode 3: the whole 128-byte line at offset 0 by 16 lanes x 8 B
//   mode 4: 4 B at 1496 and 32 B at 16 (both of a tx_finish frame)
//   mode 5: the 64-byte blocks at 0 and 1472 (the fields' and the FCS's, whole)
// then the same slots are read whole by a streaming kernel (the next step's
// loads), so write-backs that the next reads wait for are counted too.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/dev_write.hip -o tools/ubench/dev_write
#include <hip/hip_runtime.h>
#include <cstdio>

__global__ void wr(uint8_t* __restrict__ slots, uint32_t n, uint32_t cap, int mode) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (mode == 0) {
    if (t >= n) return;
    *reinterpret_cast<uint32_t*>(slots + (size_t)t * cap + 1496) = t;
  } else if (mode == 1) {
    const uint32_t f = t >> 2, q = t & 3u;
    if (f >= n) return;
    *reinterpret_cast<uint2*>(slots + (size_t)f * cap + 16 + 8 * q) = make_uint2(t, f);
  } else if (mode == 2) {
    const uint32_t f = t >> 3, q = t & 7u;
    if (f >= n) return;
    *reinterpret_cast<uint2*>(slots + (size_t)f * cap + 8 * q) = make_uint2(t, f);
  } else if (mode == 3) {
    const uint32_t f = t >> 4, q = t & 15u;
    if (f >= n) return;
    *reinterpret_cast<uint2*>(slots + (size_t)f * cap + 8 * q) = make_uint2(t, f);
  } else if (mode == 4) {
    const uint32_t f = t >> 2, q = t & 3u;
    if (f >= n) return;
    *reinterpret_cast<uint2*>(slots + (size_t)f * cap + 16 + 8 * q) = make_uint2(t, f);
    if (q == 0) *reinterpret_cast<uint32_t*>(slots + (size_t)f * cap + 1496) = t;
  } else {
    const uint32_t f = t >> 3, q = t & 7u;
    if (f >= n) return;
    *reinterpret_cast<uint2*>(slots + (size_t)f * cap + 8 * q) = make_uint2(t, f);
    *reinterpret_cast<uint2*>(slots + (size_t)f * cap + 1472 + 8 * q) = make_uint2(t, f);
  }
}

__global__ void rd(const uint4* __restrict__ p, size_t n16, uint32_t* sink) {
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4* q = reinterpret_cast<const u32x4*>(p);
  uint32_t x = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n16; i += (size_t)gridDim.x * blockDim.x) {
    const u32x4 v = __builtin_nontemporal_load(q + i);
    x ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (x == 0x12345678u) sink[0] = x;
}

int main() {
  const uint32_t n = 1u << 20, cap = 1536;
  uint8_t* d = nullptr;
  uint32_t* sink = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&d), (size_t)n * cap) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&sink), 4) != hipSuccess)
    return 1;
  (void)hipMemset(d, 0, (size_t)n * cap);
  hipEvent_t a, b, c;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  (void)hipEventCreate(&c);
  const char* names[] = {"4 B at 1496", "32 B at 16 (4 lanes)", "64 B block at 0 (8 lanes)", "128 B line at 0 (16 lanes)",
                         "32 B at 16 + 4 B at 1496", "64 B blocks at 0 and 1472"};
  const uint32_t lanes[] = {1, 4, 8, 16, 4, 8};
  const size_t n16 = (size_t)n * cap / 16;
  for (int mode = -1; mode < 6; ++mode) {
    float bw = 1e9f, br = 1e9f;
    for (int rep = 0; rep < 8; ++rep) {
      (void)hipEventRecord(a, 0);
      if (mode >= 0)
        hipLaunchKernelGGL(wr, dim3((n * lanes[mode] + 255) / 256), dim3(256), 0, 0, d, n, cap, mode);
      (void)hipEventRecord(b, 0);
      hipLaunchKernelGGL(rd, dim3(4096), dim3(256), 0, 0, reinterpret_cast<const uint4*>(d), n16, sink);
      (void)hipEventRecord(c, 0);
      (void)hipEventSynchronize(c);
      float m1 = 0, m2 = 0;
      (void)hipEventElapsedTime(&m1, a, b);
      (void)hipEventElapsedTime(&m2, b, c);
      if (rep > 1) {
        if (m1 < bw) bw = m1;
        if (m2 < br) br = m2;
      }
    }
    printf("{\"mode\": %d, \"what\": \"%s\", \"write_ms\": %.4f, \"read_after_ms\": %.4f, \"sum_ms\": %.4f}\n", mode,
           mode >= 0 ? names[mode] : "none (read only)", mode >= 0 ? bw : 0.0f, br, (mode >= 0 ? bw : 0.0f) + br);
    fflush(stdout);
  }
  (void)hipFree(d);
  (void)hipFree(sink);
  return 0;
}
