// Does the order in which a workgroup's waves walk its frames matter to HBM?
// 4 rows x 16 lanes per wave, dword loads, each row one whole frame of FB
// bytes (24 steps in flight), as crc32_rows_kernel does for 1500-B frames.
//   mode 0: wave w owns a contiguous run of frames (ubench pattern.hip)
//   mode 1: the workgroup's slice is cut into chunks of CH frames dealt to its
//           waves round-robin (the kernel's dynamic chunks, statically)
//   mode 2: like 1, chunks claimed dynamically from an LDS counter
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

// LD 0: global loads of the frame's own bytes from its start; LD 1: a window of
// 24 steps ending at the frame end rounded up to 4 (lead-in = previous frame's
// bytes, as crc32_rows_kernel reads); LD 2: LD 1 through inline-asm raw buffer
// loads from one voffset + immediates (the kernel's instruction form).
#define L6(k) "buffer_load_dword %" #k ", %24, %25, 0 offen offset:" #k "*64\n\t"
template <int MODE, int CH, int LD = 0, int EX = 0>
__global__ void __launch_bounds__(1024) walk(const uint8_t* __restrict__ base, uint64_t nframes, uint32_t fb,
                                             uint32_t* out) {
  __shared__ uint32_t pad[40950];
  __shared__ uint32_t ctr;
  if (threadIdx.x == 0) ctr = 0;
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63, p = lane & 15, row = lane >> 4;
  const uint32_t w = threadIdx.x >> 6;
  const uint64_t per_block = (nframes + gridDim.x - 1) / gridDim.x;
  const uint64_t b0 = blockIdx.x * per_block, b1 = std::min<uint64_t>(b0 + per_block, nframes);
  uint32_t acc = 0, held = 0, nheld = 0;
  const __amdgpu_buffer_rsrc_t rsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)(nframes * fb), 0x00020000);
  // EX bits (LD 2 only): 1 = two offset loads per batch (lanes 0..7, 8-byte
  // stride, like the kernel's bounds window), 2 = one 4-byte store per row per
  // batch, 4 = a 160 KiB LDS fill from global memory at start
  if (EX & 4) {
    const uint4* src = reinterpret_cast<const uint4*>(base);
    uint4* l4 = reinterpret_cast<uint4*>(pad);
    for (int i = threadIdx.x; i < 40950 / 4; i += 1024) l4[i] = src[i];
    __syncthreads();
  }
  const __amdgpu_buffer_rsrc_t osr =
      __builtin_amdgcn_make_buffer_rsrc(out, (short)0, (int)(nframes * 4), 0x00020000);
  const __amdgpu_buffer_rsrc_t orsrc =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)(nframes * 8 + 8), 0x00020000);
  auto frame4 = [&](uint64_t f) {
    uint32_t v[24];
    if (LD == 0) {
      const uint8_t* fr = base + f * fb;
#pragma unroll
      for (int u = 0; u < 24; ++u) {
        const uint32_t oo = u * 64 + p * 4;
        v[u] = (f < b1 && oo + 4 <= fb) ? *(const uint32_t*)(fr + oo) : 0u;
      }
    } else if (LD == 1) {
      const int64_t e4 = (int64_t)(((f + 1) * fb + 3) & ~3ull);
      const int64_t w0 = e4 - 24 * 64 + 4 * p;
#pragma unroll
      for (int u = 0; u < 24; ++u) {
        const int64_t a = w0 + 64 * u;
        v[u] = (f < b1 && a >= 0) ? *(const uint32_t*)(base + a) : 0u;
      }
    } else {
      const int64_t e4 = (int64_t)(((f + 1) * fb + 3) & ~3ull);
      const uint32_t vo = f < b1 ? (uint32_t)(e4 - 24 * 64 + 4 * p) : 0x80000000u;
      asm volatile("s_nop 4\n\t" L6(0) L6(1) L6(2) L6(3) L6(4) L6(5) L6(6) L6(7) L6(8) L6(9) L6(10) L6(11)
                   L6(12) L6(13) L6(14) L6(15) L6(16) L6(17) L6(18) L6(19) L6(20) L6(21) L6(22) L6(23)
                   "s_waitcnt vmcnt(0)"
                   : "=v"(v[0]), "=v"(v[1]), "=v"(v[2]), "=v"(v[3]), "=v"(v[4]), "=v"(v[5]), "=v"(v[6]), "=v"(v[7]),
                     "=v"(v[8]), "=v"(v[9]), "=v"(v[10]), "=v"(v[11]), "=v"(v[12]), "=v"(v[13]), "=v"(v[14]),
                     "=v"(v[15]), "=v"(v[16]), "=v"(v[17]), "=v"(v[18]), "=v"(v[19]), "=v"(v[20]), "=v"(v[21]),
                     "=v"(v[22]), "=v"(v[23])
                   : "v"(vo), "s"(rsrc));
      if (EX & 1) {
        uint32_t a, b;
        const uint32_t oo = lane < 8 ? (uint32_t)(f * 8 + lane * 8) : 0x80000000u;
        asm volatile("s_nop 4\n\tbuffer_load_dword %0, %2, %3, 0 offen\n\tbuffer_load_dword %1, %2, %3, 0 offen offset:8\n\ts_waitcnt vmcnt(0)"
                     : "=v"(a), "=v"(b) : "v"(oo), "s"(orsrc));
        v[0] ^= a ^ b;
      }
    }
#pragma unroll
    for (int u = 0; u < 24; ++u) acc ^= v[u];
    if (EX & 2) {
      const uint32_t so = (p == 0 && f < b1) ? (uint32_t)(f * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(acc, osr, so, 0, 0);
    }
    if (EX & 8) {  // one 64-lane dword store (256 B contiguous) every 64 frames
      if (((f - row) & 63) == 0) {
        const uint32_t so = f + 64 <= b1 ? (uint32_t)(f * 4 + lane * 4) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b32(acc, osr, so, 0, 0);
      }
    }
    if (EX & 32) {  // keep the result; written once at the end (below)
      held = held * 31u + acc;
      ++nheld;
    }
    if (EX & 16) {  // per-batch store, non-temporal
      const uint32_t so = (p == 0 && f < b1) ? (uint32_t)(f * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(acc, osr, so, 0, 2);
    }
  };
  if (MODE == 0) {
    const uint64_t pw = (b1 - b0 + 15) / 16;
    const uint64_t f0 = b0 + w * pw, f1 = std::min<uint64_t>(f0 + pw, b1);
    for (uint64_t f = f0; f < f1; f += 4) frame4(f + row < f1 ? f + row : b1);
  } else if (MODE == 1) {
    for (uint64_t c = b0 + (uint64_t)w * CH; c < b1; c += 16 * CH)
      for (uint32_t k = 0; k < CH; k += 4) frame4(c + k + row);
  } else {
    for (;;) {
      uint32_t c = 0;
      if (lane == 0) c = atomicAdd(&ctr, CH);
      c = __builtin_amdgcn_readfirstlane(c);
      if (b0 + c >= b1) break;
      for (uint32_t k = 0; k < CH; k += 4) frame4(b0 + c + k + row);
    }
  }
  if (EX & 32) {  // the same byte count as per-batch stores, in one burst at the end
    const uint64_t gw = (uint64_t)blockIdx.x * 16 + w;
    const uint64_t per_wave = nframes / (gridDim.x * 16);
    for (uint32_t k = 0; k < per_wave; k += 64) {
      const uint32_t so = (gw * per_wave + k + lane) < nframes ? (uint32_t)((gw * per_wave + k + lane) * 4) : 0x80000000u;
      __builtin_amdgcn_raw_buffer_store_b32(held + k, osr, so, 0, 0);
    }
  }
  pad[threadIdx.x] = acc;
  __syncthreads();
  if (pad[(threadIdx.x + 1) & 1023] == 0x12345678u) out[0] = acc;
}

template <typename F>
float tm(F fn) {
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  for (int i = 0; i < 20; ++i) fn();
  (void)hipDeviceSynchronize();
  std::vector<float> t;
  for (int r = 0; r < 9; ++r) { (void)hipEventRecord(a); fn(); (void)hipEventRecord(b); (void)hipEventSynchronize(b);
    float ms; (void)hipEventElapsedTime(&ms, a, b); t.push_back(ms); }
  std::sort(t.begin(), t.end()); return t[4];
}

int main(int argc, char** argv) {
  const uint32_t fb = argc > 1 ? (uint32_t)atoi(argv[1]) : 1536;
  const uint64_t nframes = 1 << 20;
  uint8_t* buf; uint32_t* out;
  (void)hipMalloc(&buf, nframes * fb + 4096); (void)hipMalloc(&out, nframes * 4 + 64);
  (void)hipMemset(buf, 3, nframes * fb);
#define RUN(M, C, LD, EX) { float ms = tm([&] { walk<M, C, LD, EX><<<256, 1024>>>(buf, nframes, fb, out); }); \
  printf("fb=%u mode=%d CH=%3d LD=%d EX=%d : %.4f ms %.1f GB/s\n", fb, M, C, LD, EX, ms, nframes * fb / ms / 1e6); }
  for (int rep = 0; rep < 2; ++rep) {
    RUN(2, 4, 2, 0); RUN(2, 4, 2, 2); RUN(2, 4, 2, 32); RUN(2, 4, 2, 0); RUN(2, 4, 2, 2); RUN(2, 4, 2, 32);
  }
  return 0;
}
