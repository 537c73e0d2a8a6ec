// Audit fixture (tests/test_kernel_audit.py): a DPP read of a VGPR that lanes
// >= n never wrote (stale) and the same with the register zeroed first (fine).
#include <hip/hip_runtime.h>
__global__ void stale(unsigned* o, unsigned n) {
  unsigned x;
  if (threadIdx.x < n) x = o[threadIdx.x] * 3u;  // written under a narrowed exec only
  o[threadIdx.x + 64] = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xF, 0xF, false);
}
__global__ void fine(unsigned* o, unsigned n) {
  unsigned x = 0;
  if (threadIdx.x < n) x = o[threadIdx.x] * 3u;
  o[threadIdx.x + 64] = (unsigned)__builtin_amdgcn_mov_dpp((int)x, 0x111, 0xF, 0xF, false);
}
