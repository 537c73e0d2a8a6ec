// What in-place result stores cost a streaming read (the TX append and
// checksum-generate shapes): 1 M slots of 1536 B are read
// whole with dwordx4 loads (8 in flight per lane), and per slot one 4-byte
// result is stored
//   0: nowhere (reads only)
//   1: in place at byte 1496 of the slot (the FCS position of a 1496-B frame)
//   2: in place, non-temporal
//   3: into a compact array (4 B per slot)
//   4: in place as four byte stores
//   5: in place at byte 24 (the IPv4 header checksum of a frame at slot start)
//   6: in place, the whole 16-byte piece holding byte 1496 rewritten (the
//      loaded bytes with the result dword replaced)
//   7: in place, the whole 32-byte sector [1472, 1504) rewritten
//   8: in place, the whole 64-byte sector [1472, 1536) rewritten
//   9: in place, the whole 128-byte line [1408, 1536) rewritten
//  10: in place at byte 1496, held in a register and stored after the
//      thread's last read (writes deferred to the end of each thread's work)
//  11: a separate launch storing the 4-byte results in place (the reads-only
//      kernel's cost is mode 0; mode 3 + mode 11 = a compact array, then a scatter)
// Not part of the product.  usage: scatter_write [nslots]
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
constexpr uint32_t kSlot = 1536, kChunks = kSlot / 16, D = 8;

template <int MODE>
__global__ void __launch_bounds__(1024) rd(const u32x4* __restrict__ src, uint8_t* data, uint32_t* compact,
                                           uint32_t nchunks) {
  const uint32_t nt = gridDim.x * blockDim.x;
  uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t acc = 0, held_slot = 0xFFFFFFFFu, held = 0;
  if constexpr (MODE == 11) {  // scatter only: slot i's result from the compact array
    for (uint32_t s = i; s < nchunks / kChunks; s += nt)
      *reinterpret_cast<uint32_t*>(data + (size_t)s * kSlot + 1496) = compact[s];
    return;
  }
  for (; i + (D - 1) * nt < nchunks; i += D * nt) {
    u32x4 v[D];
#pragma unroll
    for (uint32_t u = 0; u < D; ++u) v[u] = __builtin_nontemporal_load(src + i + u * nt);
#pragma unroll
    for (uint32_t u = 0; u < D; ++u) {
      const uint32_t x = v[u][0] ^ v[u][1] ^ v[u][2] ^ v[u][3];
      acc = __builtin_amdgcn_alignbit(acc, acc, 7) ^ x;
      const uint32_t c = i + u * nt, slot = c / kChunks, k = c - slot * kChunks;
      if constexpr (MODE == 1 || MODE == 2 || MODE == 4) {
        if (k == 1496 / 16) {
          uint8_t* q = data + (size_t)slot * kSlot + 1496;
          if constexpr (MODE == 1) *reinterpret_cast<uint32_t*>(q) = acc;
          if constexpr (MODE == 2) __builtin_nontemporal_store(acc, reinterpret_cast<uint32_t*>(q));
          if constexpr (MODE == 4) q[0] = acc, q[1] = acc >> 8, q[2] = acc >> 16, q[3] = acc >> 24;
        }
      } else if constexpr (MODE == 3) {
        if (k == 1496 / 16) compact[slot] = acc;
      } else if constexpr (MODE == 10) {
        if (k == 1496 / 16) {
          if (held_slot != 0xFFFFFFFFu) *reinterpret_cast<uint32_t*>(data + (size_t)held_slot * kSlot + 1496) = held;
          held_slot = slot, held = acc;
        }
      } else if constexpr (MODE == 5) {
        if (k == 1) *reinterpret_cast<uint32_t*>(data + (size_t)slot * kSlot + 24) = acc;
      } else if constexpr (MODE >= 6) {
        // pieces k0 .. 95 of the slot are rewritten whole; piece 93 carries the result
        constexpr uint32_t k0 = MODE == 6 ? 93 : MODE == 7 ? 92 : MODE == 8 ? 92 : 88;
        constexpr uint32_t k1 = MODE == 6 ? 94 : MODE == 7 ? 94 : 96;
        if (k >= k0 && k < k1) {
          u32x4 o = v[u];
          if (k == 93) o[2] = acc;  // bytes 1496..1499
          reinterpret_cast<u32x4*>(data)[c] = o;
        }
      }
    }
  }
  if constexpr (MODE == 10) {
    if (held_slot != 0xFFFFFFFFu) *reinterpret_cast<uint32_t*>(data + (size_t)held_slot * kSlot + 1496) = held;
  }
  if (acc == 0x9E3779B9u) compact[0] = acc;  // keeps the reads live in mode 0
}

int main(int argc, char** argv) {
  const uint32_t nslots = argc > 1 ? (uint32_t)atoi(argv[1]) : (1u << 20);
  const size_t nbytes = (size_t)nslots * kSlot;
  const uint32_t nchunks = (uint32_t)(nbytes / 16);
  uint8_t* buf;
  uint32_t* compact;
  (void)hipMalloc(&buf, nbytes);
  (void)hipMalloc(&compact, (size_t)nslots * 4);
  (void)hipMemset(buf, 5, nbytes);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  auto launch = [&](int m) {
    const dim3 g(256 * 8), blk(1024);
    switch (m) {
      case 0: rd<0><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 1: rd<1><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 2: rd<2><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 3: rd<3><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 4: rd<4><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 5: rd<5><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 6: rd<6><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 7: rd<7><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 8: rd<8><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 9: rd<9><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 10: rd<10><<<g, blk>>>((const u32x4*)buf, buf, compact, nchunks); break;
      case 11: rd<11><<<dim3(1024), dim3(1024)>>>((const u32x4*)buf, buf, compact, nchunks); break;
    }
  };
  for (int k = 0; k < 200; ++k) launch(0);
  (void)hipDeviceSynchronize();
  std::vector<std::vector<float>> t(12);
  for (int r = 0; r < 9; ++r)
    for (int m = 0; m < 12; ++m) {
      (void)hipEventRecord(a);
      for (int k = 0; k < 10; ++k) launch(m);
      (void)hipEventRecord(b);
      (void)hipEventSynchronize(b);
      float ms;
      (void)hipEventElapsedTime(&ms, a, b);
      t[m].push_back(ms / 10);
    }
  const char* what[12] = {"reads only", "in place, dword at 1496", "in place, non-temporal dword",
                          "compact array (4 B per slot)", "in place, four byte stores", "in place, dword at 24",
                          "in place, 16-B piece rewritten", "in place, 32-B sector rewritten",
                          "in place, 64-B sector rewritten", "in place, 128-B line rewritten",
                          "in place, held to the end", "scatter launch alone"};
  printf("%u slots x %u B (%.3f GB), grid 2048 x 1024, dwordx4 nt loads, %u in flight\n", nslots, kSlot, nbytes / 1e9,
         D);
  for (int m = 0; m < 12; ++m) {
    std::sort(t[m].begin(), t[m].end());
    const float ms = t[m][4];
    printf("mode %d %-30s: %.4f ms  %.1f GB/s (slot bytes)  %+.1f %%\n", m, what[m], ms, nbytes / ms / 1e6,
           100.0 * (ms / t[0][4] - 1));
  }
  return 0;
}
