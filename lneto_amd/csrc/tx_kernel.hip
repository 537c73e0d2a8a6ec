// tx_kernel.hip — batched TX FCS append, gfx950.
//
// Reference: the tail of StackEthernet.Encapsulate (internet/stack-ethernet.go:
// 200-214): zero-pad the frame to 60 bytes, then with the CRC32Update hook set
// write LE32(CRC32Update(0, frame)) after it and grow the frame by 4.  The
// batch form runs three launches on the stream:
//   tx_pad_kernel       zero padding to 60 bytes, d_len <- padded length
//   crc32_rows_kernel   segment mode over (d_start, d_len) -> CRCs (scratch)
//   tx_fcs_kernel       LE32 FCS after the padded frame, d_len += 4
// A frame whose padded length + 4 exceeds `capacity` is left untouched with
// status 6 (lneto.ErrShortBuffer, errors.go:13; the per-frame form of
// Encapsulate's io.ErrShortBuffer check on the destination size,
// internet/stack-ethernet.go:170-179).  The onSend hook
// that the reference runs between padding and FCS has no batch equivalent.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lnx {

constexpr uint32_t kMinFrame = 60;
constexpr uint8_t kErrShortBuffer = 6;

__global__ void __launch_bounds__(256)
tx_pad_kernel(uint8_t* __restrict__ bytes, const uint64_t* __restrict__ start, uint32_t* __restrict__ len,
              uint64_t n, uint32_t capacity, uint8_t* __restrict__ status) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t l = len[i];
    const uint32_t pl = l < kMinFrame ? kMinFrame : l;
    if ((uint64_t)pl + 4 > capacity) {
      status[i] = kErrShortBuffer;
      continue;
    }
    status[i] = 0;
    uint8_t* f = bytes + start[i];
    for (uint32_t k = l; k < pl; ++k) f[k] = 0;
    len[i] = pl;
  }
}

__global__ void __launch_bounds__(256)
tx_fcs_kernel(uint8_t* __restrict__ bytes, const uint64_t* __restrict__ start, uint32_t* __restrict__ len,
              uint64_t n, const uint32_t* __restrict__ crc, const uint8_t* __restrict__ status) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (status[i] != 0) continue;
    const uint32_t pl = len[i], c = crc[i];
    uint8_t* f = bytes + start[i] + pl;
    f[0] = (uint8_t)c, f[1] = (uint8_t)(c >> 8), f[2] = (uint8_t)(c >> 16), f[3] = (uint8_t)(c >> 24);
    len[i] = pl + 4;
  }
}

hipError_t launch_crc32_segments(const uint8_t* bytes, const uint64_t* start, const uint32_t* len, uint64_t n,
                                 void* out, const void* images, int num_cus, hipStream_t stream);

hipError_t launch_fcs_append(uint8_t* bytes, const uint64_t* start, uint32_t* len, uint64_t n, uint32_t capacity,
                             uint8_t* status, uint32_t* crc_scratch, const void* images, int num_cus,
                             hipStream_t stream) {
  if (n == 0) return hipSuccess;
  uint64_t grid = (n + 255) / 256;
  if (grid > (uint64_t)num_cus * 8) grid = (uint64_t)num_cus * 8;
  hipLaunchKernelGGL(tx_pad_kernel, dim3((unsigned)grid), dim3(256), 0, stream, bytes, start, len, n, capacity,
                     status);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  e = launch_crc32_segments(bytes, start, len, n, crc_scratch, images, num_cus, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(tx_fcs_kernel, dim3((unsigned)grid), dim3(256), 0, stream, bytes, start, len, n, crc_scratch,
                     status);
  return hipGetLastError();
}

}  // namespace lnx
