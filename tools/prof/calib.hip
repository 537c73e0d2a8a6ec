// FETCH_SIZE calibration for rocprofv3 on gfx950 (MI355X_MICROARCH.md §HBM:
// FETCH_SIZE is uncalibrated for access widths other than 16 B/lane).
// Reads a known number of bytes with the CRC kernel's access width
// (one dword per lane, 256 contiguous bytes per wave instruction) and with
// 16 B/lane, so that FETCH_SIZE can be converted to bytes for that pattern.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <typename T>
__global__ void __launch_bounds__(256) rd(const T* __restrict__ p, size_t n, uint32_t* out) {
  size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x, st = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  for (; i < n; i += st) {
    T v = p[i];
    if constexpr (sizeof(T) == 4) acc ^= v; else acc ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const size_t bytes = (size_t)2 << 30;
  void* buf; uint32_t* out;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
  (void)hipMemset(buf, 1, bytes);
  for (int r = 0; r < 3; ++r) {
    rd<uint32_t><<<2048, 256>>>((const uint32_t*)buf, bytes / 4, out);
    rd<uint4><<<2048, 256>>>((const uint4*)buf, bytes / 16, out);
  }
  (void)hipDeviceSynchronize();
  printf("calib: read %zu bytes per dispatch (rd<uint32_t> dword/lane, rd<uint4> 16B/lane)\n", bytes);
  return 0;
}
