// Do byte-misaligned buffer_load_dword streams run at full rate on gfx950, and
// what do they return?  Each wave streams a contiguous region with lane l
// reading the dword at byte offset SHIFT + 4l + 256k (k = 0, 1, ...), exactly
// the row pattern of the CRC kernel for a frame whose end is SHIFT mod 4.
// Checks (1) the bytes against the host copy, (2) the range-check behaviour of
// a dword straddling the end of the descriptor's range, (3) bandwidth per SHIFT.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <cstring>
#include <vector>
#include <algorithm>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  fprintf(stderr, "HIP error %s at %s:%d\n", hipGetErrorString(e_), __FILE__, __LINE__); exit(1);} } while (0)

__device__ __forceinline__ uint32_t ldb(uint32_t voff, __amdgpu_buffer_rsrc_t r) {
  uint32_t v;
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=v"(v) : "v"(voff), "s"(r));
  return v;
}

// Streaming: each wave owns `per_wave` bytes; 8 loads in flight.
__global__ void __launch_bounds__(1024) stream(const uint8_t* base, uint64_t per_wave, uint32_t shift,
                                               uint32_t* out) {
  __shared__ uint32_t pad[40960];
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t gw = blockIdx.x * 16ull + (uint32_t)__builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base + gw * per_wave), (short)0, (int)per_wave, 0x00020000);
  asm volatile("s_nop 4" ::: "memory");
  uint32_t acc = 0;
  for (uint32_t o = shift + lane * 4; o < per_wave; o += 256 * 8) {
    uint32_t v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = ldb(o + 256 * k, r);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < 8; ++k) acc ^= v[k];
  }
  pad[threadIdx.x] = acc;
  __syncthreads();
  out[gw * 64 + lane] = acc ^ pad[(threadIdx.x + 64) & 1023];
}

// Correctness: one wave, returns the dword at every offset 0..n-1 (range n_rec).
__global__ void probe(const uint8_t* base, uint32_t n, uint32_t n_rec, uint32_t* out) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)n_rec, 0x00020000);
  asm volatile("s_nop 4" ::: "memory");
  for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
    uint32_t v = ldb(i, r);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    out[i] = v;
  }
}

// Range check with an immediate offset: which of vgpr / vgpr+imm is checked?
template <int IMM>
__device__ __forceinline__ uint32_t ldi(uint32_t voff, __amdgpu_buffer_rsrc_t r) {
  uint32_t v;
  asm volatile("buffer_load_dword %0, %1, %2, 0 offen offset:%3" : "=v"(v) : "v"(voff), "s"(r), "i"(IMM));
  return v;
}
__global__ void probe_imm(const uint8_t* base, uint32_t n_rec, uint32_t* out) {
  const __amdgpu_buffer_rsrc_t r =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(base), (short)0, (int)n_rec, 0x00020000);
  asm volatile("s_nop 4" ::: "memory");
  if (threadIdx.x == 0) {
    uint32_t v[8];
    v[0] = ldi<0>(n_rec - 8, r);
    v[1] = ldi<4>(n_rec - 8, r);
    v[2] = ldi<8>(n_rec - 8, r);
    v[3] = ldi<16>(n_rec - 8, r);
    v[4] = ldi<64>(n_rec - 8, r);
    v[5] = ldi<8>(0xFFFFFFFCu, r);
    v[6] = ldi<64>(0xFFFFFFC0u, r);
    v[7] = ldi<0>(n_rec, r);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    for (int i = 0; i < 8; ++i) out[i] = v[i];
  }
}

int main() {
  // (1) + (2): correctness and range check
  const uint32_t n = 4096, n_rec = 4001;  // deliberately not a multiple of 4
  std::vector<uint8_t> h(n + 8);
  for (uint32_t i = 0; i < h.size(); ++i) h[i] = (uint8_t)(i * 131 + 7);
  uint8_t* d; uint32_t* o;
  CK(hipMalloc(&d, h.size())); CK(hipMalloc(&o, n * 4));
  CK(hipMemcpy(d, h.data(), h.size(), hipMemcpyHostToDevice));
  probe<<<1, 256>>>(d, n, n_rec, o);
  CK(hipDeviceSynchronize());
  std::vector<uint32_t> got(n);
  CK(hipMemcpy(got.data(), o, n * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  for (uint32_t i = 0; i + 4 <= n_rec; ++i) {
    uint32_t want; memcpy(&want, &h[i], 4);
    if (got[i] != want && bad++ < 5) printf("mismatch at %u: got %08x want %08x\n", i, got[i], want);
  }
  printf("unaligned in-range dwords: %s\n", bad ? "WRONG" : "exact");
  for (uint32_t i = n_rec - 5; i < n_rec + 2; ++i) {
    uint32_t want = 0;
    for (uint32_t b = 0; b < 4; ++b) if (i + b < n_rec) want |= (uint32_t)h[i + b] << (8 * b);
    printf("straddle off %u (n_rec %u): got %08x  bytes-in-range %08x\n", i, n_rec, got[i], want);
  }
  {
    const uint32_t nr = 2000;
    probe_imm<<<1, 64>>>(d, nr, o);
    CK(hipDeviceSynchronize());
    uint32_t g[8];
    CK(hipMemcpy(g, o, 32, hipMemcpyDeviceToHost));
    const char* what[8] = {"v=nr-8 imm=0", "v=nr-8 imm=4", "v=nr-8 imm=8 (past end)", "v=nr-8 imm=16 (past end)",
                           "v=nr-8 imm=64 (past end)", "v=-4 imm=8 (=4, in range)", "v=-64 imm=64 (=0, in range)",
                           "v=nr imm=0 (past end)"};
    uint32_t addr[8] = {nr - 8, nr - 4, nr, nr + 8, nr + 56, 4, 0, nr};
    for (int i = 0; i < 8; ++i) {
      uint32_t mem; memcpy(&mem, &h[addr[i]], 4);
      printf("imm probe %-30s got %08x  memory %08x\n", what[i], g[i], mem);
    }
  }
  CK(hipFree(d)); CK(hipFree(o));

  // (3) bandwidth
  const uint64_t waves = 256 * 16, per_wave = 384 * 1024, total = waves * per_wave;  // 1.5 GiB
  uint8_t* big; uint32_t* out;
  CK(hipMalloc(&big, total + 256)); CK(hipMalloc(&out, waves * 64 * 4));
  CK(hipMemset(big, 1, total + 256));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  for (int rep = 0; rep < 2; ++rep)
    for (uint32_t shift = 0; shift < 4; ++shift) {
      stream<<<256, 1024>>>(big, per_wave, shift, out);
      CK(hipDeviceSynchronize());
      std::vector<float> t;
      for (int r = 0; r < 7; ++r) {
        CK(hipEventRecord(a)); stream<<<256, 1024>>>(big, per_wave, shift, out); CK(hipEventRecord(b));
        CK(hipEventSynchronize(b)); float ms; CK(hipEventElapsedTime(&ms, a, b)); t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      printf("stream shift=%u: %.3f ms  %.1f GB/s\n", shift, t[3], total / t[3] / 1e6);
    }
  return 0;
}
