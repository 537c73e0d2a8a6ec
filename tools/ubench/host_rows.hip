// The receive rows' read pattern over pinned host memory (the ring's zero-copy
// ingress), without the CRC: 1 M slots of 1536 B, each wave takes
// 48 consecutive slots, four at a time (one 16-lane row each, lane p loading
// qwords p, p + 16, ... of the slot), `ahead` passes loaded before the first
// is consumed (whole_lines: every 128-B line the frame touches is loaded
// whole, not just its qwords).  Slot lengths from a file (uint32 each; the Zipf mix of
// bench.py) or 256 B; a lane whose qword lies past its slot's length loads a
// zero qword in device memory instead (as rx_verify_kernel does).  Batches of
// `batch` slots, one launch each, on 1 or 3 streams.
//   hipcc --offload-arch=gfx950 -O3 tools/ubench/host_rows.hip -o tools/ubench/host_rows
//   host_rows [lengths.u32]
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstring>
#include <vector>

__device__ uint2 g_zero[2];

template <int AHEAD, bool WHOLE>
__global__ void __launch_bounds__(1024) rows(const uint8_t* __restrict__ slots, const uint32_t* __restrict__ len,
                                             uint32_t n, uint32_t cap, uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63u, p = lane & 15u, row = lane >> 4;
  const uint32_t w = blockIdx.x * 16u + (threadIdx.x >> 6);
  const uint32_t f0 = w * 48u;
  uint32_t acc = 0;
  for (uint32_t j = 0; j < 12u; j += AHEAD) {
    uint2 v[AHEAD][12];
#pragma unroll
    for (int a = 0; a < AHEAD; ++a) {
      const uint32_t f = f0 + 4u * (j + a) + row;
      const bool live = f < n && j + a < 12u;
      const uint32_t q8 = live ? (len[f] + 7u) >> 3 : 0u;
      const uint32_t qe = WHOLE ? (q8 + 15u) & ~15u : q8;  // WHOLE: every line the frame touches, whole
      const uint2* b = reinterpret_cast<const uint2*>(slots + (size_t)(live ? f : 0u) * cap);
#pragma unroll
      for (int u = 0; u < 12; ++u) {
        const uint32_t q = p + 16u * u;
        const uint2* ad = q < qe ? b + q : g_zero;
        const uint64_t x = *(const __attribute__((address_space(1))) uint64_t*)ad;
        v[a][u] = make_uint2((uint32_t)x, (uint32_t)(x >> 32));
      }
    }
#pragma unroll
    for (int a = 0; a < AHEAD; ++a)
#pragma unroll
      for (int u = 0; u < 12; ++u) acc ^= v[a][u].x ^ v[a][u].y;
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// gather: slot i's first len[i] bytes (rounded up to 16) copied to the same
// place in a device buffer, LANES lanes per slot x 16 B, looping for longer frames
template <int LANES>
__global__ void __launch_bounds__(256) gather(const uint8_t* __restrict__ slots, const uint32_t* __restrict__ len,
                                              uint32_t n, uint32_t cap, uint8_t* __restrict__ dst) {
  const uint32_t t = blockIdx.x * 256u + threadIdx.x;
  const uint32_t f = t / LANES, c = t % LANES;
  if (f >= n) return;
  const uint32_t l = len[f];
  const size_t b = (size_t)f * cap;
  for (uint32_t o = 16u * c; o < l; o += 16u * LANES) {
    const uint4 v = *reinterpret_cast<const uint4*>(slots + b + o);
    *reinterpret_cast<uint4*>(dst + b + o) = v;
  }
}

int main(int argc, char** argv) {
  const uint32_t n = 1u << 20, cap = 1536;
  std::vector<uint32_t> hl(n, 256u);
  const char* what = "256 B";
  if (argc > 1) {
    FILE* f = fopen(argv[1], "rb");
    if (!f || fread(hl.data(), 4, n, f) != n) return 1;
    fclose(f);
    what = "Zipf lengths";
  }
  uint64_t useful = 0, lines64 = 0;
  for (uint32_t l : hl) useful += l, lines64 += (l + 63) / 64 * 64;
  uint8_t* h = nullptr;
  uint32_t *dl = nullptr, *sink = nullptr;
  if (hipHostMalloc(reinterpret_cast<void**>(&h), (size_t)n * cap, hipHostMallocDefault) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&dl), n * 4) != hipSuccess ||
      hipMalloc(reinterpret_cast<void**>(&sink), 4) != hipSuccess)
    return 2;
  memset(h, 1, (size_t)n * cap);
  (void)hipMemcpy(dl, hl.data(), n * 4, hipMemcpyHostToDevice);
  uint8_t* d = nullptr;
  if (hipHostGetDevicePointer(reinterpret_cast<void**>(&d), h, 0) != hipSuccess) return 3;
  hipStream_t st[3];
  for (auto& s : st) (void)hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (uint32_t batch : {65536u, 1048576u}) {
   for (bool whole : {false, true}) {
    for (int ns : {3}) {
      for (int ahead : {1, 3}) {
        float best = 1e9f;
        for (int rep = 0; rep < 5; ++rep) {
          (void)hipDeviceSynchronize();
          (void)hipEventRecord(a, 0);
          for (uint32_t b0 = 0, k = 0; b0 < n; b0 += batch, ++k) {
            const uint32_t nb = n - b0 < batch ? n - b0 : batch;
            const uint32_t waves = (nb + 47) / 48, grid = (waves + 15) / 16;
            hipStream_t s = st[k % ns];
            if (ahead == 1 && !whole)
              hipLaunchKernelGGL((rows<1, false>), dim3(grid), dim3(1024), 0, s, d + (size_t)b0 * cap, dl + b0, nb, cap, sink);
            else if (ahead == 1)
              hipLaunchKernelGGL((rows<1, true>), dim3(grid), dim3(1024), 0, s, d + (size_t)b0 * cap, dl + b0, nb, cap, sink);
            else if (!whole)
              hipLaunchKernelGGL((rows<3, false>), dim3(grid), dim3(1024), 0, s, d + (size_t)b0 * cap, dl + b0, nb, cap, sink);
            else
              hipLaunchKernelGGL((rows<3, true>), dim3(grid), dim3(1024), 0, s, d + (size_t)b0 * cap, dl + b0, nb, cap, sink);
          }
          (void)hipDeviceSynchronize();
          (void)hipEventRecord(b, 0);
          (void)hipEventSynchronize(b);
          float ms = 0;
          (void)hipEventElapsedTime(&ms, a, b);
          if (rep > 0 && ms < best) best = ms;
        }
        printf("{\"lengths\": \"%s\", \"batch\": %u, \"whole_lines\": %d, \"streams\": %d, \"ahead\": %d, \"ms\": %.3f, "
               "\"useful_GB_per_s\": %.1f, \"lines64_GB_per_s\": %.1f}\n",
               what, batch, (int)whole, ns, ahead, best, useful / best / 1e6, lines64 / best / 1e6);
        fflush(stdout);
      }
    }
   }
  }
  uint8_t* dd = nullptr;
  if (hipMalloc(reinterpret_cast<void**>(&dd), (size_t)n * cap) != hipSuccess) return 4;
  for (uint32_t batch : {65536u, 1048576u}) {
    for (int lanes : {4, 8, 16}) {
      float best = 1e9f;
      for (int rep = 0; rep < 5; ++rep) {
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a, 0);
        for (uint32_t b0 = 0, k = 0; b0 < n; b0 += batch, ++k) {
          const uint32_t nb = n - b0 < batch ? n - b0 : batch;
          const uint32_t grid = (nb * lanes + 255) / 256;
          hipStream_t s = st[k % 3];
          const uint8_t* src = d + (size_t)b0 * cap;
          if (lanes == 4) hipLaunchKernelGGL(gather<4>, dim3(grid), dim3(256), 0, s, src, dl + b0, nb, cap, dd + (size_t)b0 * cap);
          if (lanes == 8) hipLaunchKernelGGL(gather<8>, dim3(grid), dim3(256), 0, s, src, dl + b0, nb, cap, dd + (size_t)b0 * cap);
          if (lanes == 16) hipLaunchKernelGGL(gather<16>, dim3(grid), dim3(256), 0, s, src, dl + b0, nb, cap, dd + (size_t)b0 * cap);
        }
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, a, b);
        if (rep > 0 && ms < best) best = ms;
      }
      printf("{\"gather\": true, \"lengths\": \"%s\", \"batch\": %u, \"lanes_per_slot\": %d, \"ms\": %.3f, "
             "\"useful_GB_per_s\": %.1f}\n", what, batch, lanes, best, useful / best / 1e6);
      fflush(stdout);
    }
  }
  (void)hipFree(dd);
  (void)hipHostFree(h);
  (void)hipFree(dl);
  (void)hipFree(sink);
  return 0;
}
