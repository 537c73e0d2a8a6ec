// Read ceiling of STREAMING rows on the Zipf mix (BASELINE configs[3]: lengths
// 64..1500 B, P(L) ~ 1/(L - 63), packed back to back, arbitrary alignment).
// Unlike pattern4.hip (rows take interleaved frames), each row of 8 lanes x 16 B
// (one whole 128-byte line per row step) owns a CONTIGUOUS, byte-balanced run
// of frames:
//   MODE 1  per-frame windows: each frame from its own 128-aligned start, so the
//           line two frames share is loaded twice, by the same row, one step
//           apart;
//   MODE 2  one stream per row over the run's lines (each line loaded once);
//           the row still reads every frame's end offset as it passes it.
//   MODE 0  pattern4's interleaved frames with per-frame windows (reference).
// Loads only, D row steps in flight.  (The buffer is > 2 GiB: idle lanes use
// offset 0xFFFFF000, past the 4.13 GB range.)  Not part of the product.
// usage: pattern5 [nframes]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
template <int W> struct Vt;
template <> struct Vt<4> { typedef uint32_t T; };
template <> struct Vt<8> { typedef u32x2 T; };
template <> struct Vt<16> { typedef u32x4 T; };
template <int W>
__device__ __forceinline__ typename Vt<W>::T ldv2(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  if constexpr (W == 4) return __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0);
  if constexpr (W == 8) return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0);
  if constexpr (W == 16) return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
}
__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(u32x2 v) { return v[0] ^ v[1]; }
__device__ __forceinline__ uint32_t fold(u32x4 v) { return v[0] ^ v[1] ^ v[2] ^ v[3]; }

template <int P>
__device__ __forceinline__ u32x4 ldv(__amdgpu_buffer_rsrc_t r, uint32_t off) {
  return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, P);
}

template <int D, int MODE, int P>
__global__ void __launch_bounds__(1024) pat5(const uint8_t* __restrict__ base, uint32_t nbytes,
                                             const uint32_t* __restrict__ off, const uint32_t* __restrict__ rowf,
                                             uint32_t* out) {
  __shared__ uint32_t pad[40960];  // one workgroup per CU, as the CRC kernel
  const uint32_t lane = threadIdx.x & 63, p = lane & 7, row = lane >> 3;
  const uint32_t gw = blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint32_t rid = gw * 8 + row;
  uint32_t f, f1, stride;
  if (MODE == 0) {  // interleaved: row r of the wave takes frames f0 + r, f0 + r + 8, ...
    f = rowf[gw * 8] + row, f1 = rowf[gw * 8 + 8], stride = 8;
  } else {
    f = rowf[rid], f1 = rowf[rid + 1], stride = 1;
  }
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nbytes, 0x00020000);
  uint32_t a = 0xFFFFF000u, e = 0, fe = 0;
  if (f < f1) {
    a = off[f] & ~127u;
    e = off[f + 1];
    fe = MODE >= 2 ? off[f1] : e;
  }
  if (MODE == 5) {  // contiguous wave range, row r starts at line r
    const uint32_t w0 = rowf[gw * 8], w1 = rowf[gw * 8 + 8];
    f = w0, f1 = w1;
    a = w0 < w1 ? (off[w0] & ~127u) + 128 * row : 0xFFFFF000u;
    fe = off[w1];
  }
  auto next = [&]() -> uint32_t {
    const uint32_t o = a + p * 16;
    a += 128;
    if (MODE == 3) {
      if (a >= fe) a = 0xFFFFF000u, f = f1;
    } else if (MODE == 5) {
      a += 896;  // the wave's 8 rows take 8 consecutive lines of the wave's range
      if (a >= fe) a = 0xFFFFF000u, f = f1;
    } else if (MODE == 2) {
      while (f < f1 && e <= a) {  // pass every frame end in this line: one offset read each
        f += 1;
        e = f < f1 ? off[f + 1] : 0xFFFFFFFFu;
      }
      if (a >= fe) a = 0xFFFFF000u, f = f1;
    } else if (a >= e && f < f1) {
      f += stride;
      if (f < f1) {
        a = off[f] & ~127u;
        e = off[f + 1];
      } else {
        a = 0xFFFFF000u;
      }
    }
    return o;
  };
  u32x4 v[D];
#pragma unroll
  for (int u = 0; u < D; ++u) v[u] = ldv<P>(r, next());
  uint32_t acc = 0;
  for (;;) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
      v[u] = ldv<P>(r, next());
    }
    if (!__builtin_amdgcn_ballot_w64(f < f1)) break;
  }
#pragma unroll
  for (int u = 0; u < D; ++u) acc ^= v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
  pad[threadIdx.x] = acc + e;
  __syncthreads();
  if (pad[(threadIdx.x + 1) & 1023] == 0x12345678u) out[0] = acc;
}


// 4-lane rows, 16 rows per wave, each row streams its own byte-balanced run;
// per row step (one line) each lane loads two 16-byte pieces:
//   HALF = 1: [L + 16p, +16) and [L + 64 + 16p, +16) (each instruction: a half line per row)
//   HALF = 0: [L + 32p, +32) as two dwordx4 (each instruction: 16-byte pieces 32 bytes apart)
template <int D, int HALF, int P>
__global__ void __launch_bounds__(1024) pat6(const uint8_t* __restrict__ base, uint32_t nbytes,
                                             const uint32_t* __restrict__ off, const uint32_t* __restrict__ rowf,
                                             uint32_t* out) {
  __shared__ uint32_t pad[40960];
  const uint32_t lane = threadIdx.x & 63, p = lane & 3, row = lane >> 2;
  const uint32_t gw = blockIdx.x * 16 + (threadIdx.x >> 6);
  // rowf has 8 entries per wave: split each 8-row run in two halves by frames
  const uint32_t r8 = gw * 8 + (row >> 1);
  const uint32_t fa = rowf[r8], fb = rowf[r8 + 1];
  const uint32_t fm = fa + (fb - fa) / 2;
  const uint32_t f = (row & 1) ? fm : fa, f1 = (row & 1) ? fb : fm;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nbytes, 0x00020000);
  uint32_t a = 0xFFFFF000u, fe = 0;
  if (f < f1) a = off[f] & ~127u, fe = off[f1];
  const uint32_t o0 = HALF ? p * 16 : p * 32, o1 = HALF ? 64 + p * 16 : p * 32 + 16;
  u32x4 v[D][2];
  auto issue = [&](int u) {
    v[u][0] = ldv<P>(r, a + o0);
    v[u][1] = ldv<P>(r, a + o1);
    if (a != 0xFFFFF000u) {
      a += 128;
      if (a >= fe) a = 0xFFFFF000u;
    }
  };
#pragma unroll
  for (int u = 0; u < D; ++u) issue(u);
  uint32_t acc = 0;
  for (;;) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      acc ^= v[u][0][0] ^ v[u][0][1] ^ v[u][0][2] ^ v[u][0][3] ^ v[u][1][0] ^ v[u][1][1] ^ v[u][1][2] ^ v[u][1][3];
      issue(u);
    }
    if (!__builtin_amdgcn_ballot_w64(a != 0xFFFFF000u)) break;
  }
#pragma unroll
  for (int u = 0; u < D; ++u) acc ^= v[u][0][0] ^ v[u][1][3];
  pad[threadIdx.x] = acc;
  __syncthreads();
  if (pad[(threadIdx.x + 1) & 1023] == 0x12345678u) out[0] = acc;
}


// Per-frame windows (each frame from its own aligned start, as the product's
// rows) with the frame offsets prefetched 8 frames ahead in a register ring
// (no dependent offset load on the critical path).  RL lanes x W bytes per row
// step; CONTIG = 1: row r takes frames f0 + rK .. (contiguous, the shared line
// comes back to the same row one step later); CONTIG = 0: row r takes frames
// f0 + r, f0 + r + ROWS, ... (the product's interleave).
template <int W, int RL, int D, int A, int CONTIG>
__global__ void __launch_bounds__(1024) pat7(const uint8_t* __restrict__ base, uint32_t nbytes,
                                             const uint32_t* __restrict__ off, const uint32_t* __restrict__ rowf,
                                             uint32_t* out) {
  __shared__ uint32_t pad[40960];
  constexpr uint32_t ROWS = 64 / RL, RB = RL * W;
  const uint32_t lane = threadIdx.x & 63, p = lane % RL, row = lane / RL;
  const uint32_t gw = blockIdx.x * 16 + (threadIdx.x >> 6);
  const uint32_t w0 = rowf[gw * 8], w1 = rowf[gw * 8 + 8];
  const uint32_t nfw = w1 - w0;
  uint32_t f, f1, st;
  if (CONTIG) {
    f = w0 + (uint32_t)((uint64_t)nfw * row / ROWS), f1 = w0 + (uint32_t)((uint64_t)nfw * (row + 1) / ROWS), st = 1;
  } else {
    f = w0 + row, f1 = w1, st = ROWS;
  }
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, (int)nbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t ro = __builtin_amdgcn_make_buffer_rsrc((void*)off, (short)0, (int)0x7FFFFFF0, 0x00020000);
  // offset ring: starts and ends of the next 8 frames
  uint32_t ra[8], re[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t fi = f + i * st;
    ra[i] = fi < f1 ? off[fi] : 0xFFFFF000u;
    re[i] = fi < f1 ? off[fi + 1] : 0;
  }
  uint32_t a = ra[0] & ~(uint32_t)(A - 1), e = re[0];
  bool live = f < f1;
  if (!live) a = 0xFFFFF000u;
  auto next = [&]() -> uint32_t {
    const uint32_t o = a + p * W;
    if (live) {
      a += RB;
      if (a >= e) {
        f += st;
#pragma unroll
        for (int i = 0; i < 7; ++i) ra[i] = ra[i + 1], re[i] = re[i + 1];
        const uint32_t fn = f + 7 * st;
        ra[7] = __builtin_amdgcn_raw_buffer_load_b32(ro, fn < f1 ? fn * 4 : 0xFFFFF000u, 0, 0);
        re[7] = __builtin_amdgcn_raw_buffer_load_b32(ro, fn < f1 ? fn * 4 + 4 : 0xFFFFF000u, 0, 0);
        live = f < f1;
        a = live ? (ra[0] & ~(uint32_t)(A - 1)) : 0xFFFFF000u;
        e = re[0];
      }
    }
    return o;
  };
  typename Vt<W>::T v[D];
#pragma unroll
  for (int u = 0; u < D; ++u) v[u] = ldv2<W>(r, next());
  uint32_t acc = 0;
  for (;;) {
#pragma unroll
    for (int u = 0; u < D; ++u) {
      acc ^= fold(v[u]);
      v[u] = ldv2<W>(r, next());
    }
    if (!__builtin_amdgcn_ballot_w64(live)) break;
  }
#pragma unroll
  for (int u = 0; u < D; ++u) acc ^= fold(v[u]);
  pad[threadIdx.x] = acc;
  __syncthreads();
  if (pad[(threadIdx.x + 1) & 1023] == 0x12345678u) out[0] = acc;
}

template <typename F>
float tm(F fn) {
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int i = 0; i < 30; ++i) fn();
  (void)hipDeviceSynchronize();
  std::vector<float> t;
  for (int k = 0; k < 9; ++k) {
    (void)hipEventRecord(a);
    fn();
    (void)hipEventRecord(b);
    (void)hipEventSynchronize(b);
    float ms;
    (void)hipEventElapsedTime(&ms, a, b);
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[4];
}

int main(int argc, char** argv) {
  const uint32_t nframes = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 24);
  std::vector<double> cdf(1437);
  double acc = 0;
  for (int i = 0; i < 1437; ++i) cdf[i] = (acc += 1.0 / (i + 1));
  std::mt19937_64 g(20261015);
  std::uniform_real_distribution<double> u(0, acc);
  std::vector<uint32_t> off(nframes + 1, 0);
  for (uint32_t i = 0; i < nframes; ++i) {
    const uint32_t L = 64 + (uint32_t)(std::lower_bound(cdf.begin(), cdf.end(), u(g)) - cdf.begin());
    off[i + 1] = off[i] + L;
  }
  const uint32_t nbytes = off[nframes];
  const uint32_t waves = 256 * 16, rows = waves * 8;
  // Byte-balanced rows: row k takes the frames whose end lies in (k*S, (k+1)*S].
  std::vector<uint32_t> rowf(rows + 1);
  for (uint32_t k = 0; k <= rows; ++k) {
    const uint64_t b = (uint64_t)nbytes * k / rows;
    rowf[k] = (uint32_t)(std::lower_bound(off.begin() + 1, off.end(), (uint32_t)b) - (off.begin() + 1));
    if (k == rows) rowf[k] = nframes;
  }
  uint8_t* buf;
  uint32_t *doff, *drow, *out;
  (void)hipMalloc(&buf, (size_t)nbytes + 4096);
  (void)hipMalloc(&doff, off.size() * 4);
  (void)hipMalloc(&drow, rowf.size() * 4);
  (void)hipMalloc(&out, 64);
  (void)hipMemset(buf, 3, (size_t)nbytes + 4096);
  (void)hipMemcpy(doff, off.data(), off.size() * 4, hipMemcpyHostToDevice);
  (void)hipMemcpy(drow, rowf.data(), rowf.size() * 4, hipMemcpyHostToDevice);
  printf("zipf frames %u, %u bytes (mean %.1f), lines %.1f M\n", nframes, nbytes, (double)nbytes / nframes,
         nbytes / 128.0 / 1e6);
#define RUN(D, M, P)                                                                                        \
  {                                                                                                         \
    float ms = tm([&] { pat5<D, M, P><<<256, 1024>>>(buf, nbytes + 4096, doff, drow, out); });             \
    printf("mode=%d D=%2d pol=%d : %.4f ms %.1f GB/s of frame bytes\n", M, D, P, ms, nbytes / ms / 1e6); \
  }
#define RUN6(D, H, P)                                                                                      \
  {                                                                                                         \
    float ms = tm([&] { pat6<D, H, P><<<256, 1024>>>(buf, nbytes + 4096, doff, drow, out); });            \
    printf("4-lane rows half=%d D=%2d pol=%d : %.4f ms %.1f GB/s of frame bytes\n", H, D, P, ms, nbytes / ms / 1e6); \
  }
#define RUN7(W, RL, D, A, C)                                                                              \
  {                                                                                                         \
    float ms = tm([&] { pat7<W, RL, D, A, C><<<256, 1024>>>(buf, nbytes + 4096, doff, drow, out); });     \
    printf("per-frame windows W=%2d RL=%2d D=%d align=%3d contig=%d : %.4f ms %.1f GB/s\n", W, RL, D, A, C, ms, nbytes / ms / 1e6); \
  }
  RUN7(4, 4, 16, 4, 0);
  RUN7(4, 4, 16, 4, 1);
  RUN7(16, 4, 8, 16, 0);
  RUN7(16, 4, 8, 16, 1);
  RUN7(16, 8, 8, 128, 0);
  RUN7(16, 8, 8, 128, 1);
  RUN7(8, 16, 8, 128, 1);
  RUN6(4, 1, 0);
  RUN6(4, 1, 2);
  RUN6(4, 0, 0);
  RUN6(4, 0, 2);
  RUN6(2, 1, 0);
  RUN(8, 3, 0);
  RUN(4, 3, 0);
  RUN(8, 5, 0);
  RUN(8, 3, 2);
  RUN(8, 5, 2);
  RUN(8, 0, 0);
  RUN(4, 1, 0);
  RUN(8, 1, 0);
  RUN(4, 2, 0);
  RUN(8, 2, 0);
  RUN(12, 2, 0);
  RUN(8, 2, 2);
  return 0;
}
