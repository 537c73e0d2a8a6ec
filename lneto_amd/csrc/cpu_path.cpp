// cpu_path.cpp — per-frame host functions with exact Go semantics.
//
// These are the single-frame drop-ins (ethernet.CRC32 / CRC32Search /
// crc32.Update, lneto.CRC791 methods).  They never touch the GPU: a kernel
// launch costs microseconds, a 60-byte FCS tens of nanoseconds.
// They are not a fallback of the batch path — the batch entry points have no
// CPU route and fail with an error code when no HIP device is usable.
//
// CRC-32 here is slicing-by-16 over tables derived from the same register
// algebra as the GPU tables (gf2.hpp).
#include <cstdint>
#include <cstring>
#include "../../include/lneto_amd.h"
#include "gf2.hpp"

namespace {

struct Slice16 {
  uint32_t t[16][256];
  Slice16() {
    for (uint32_t b = 0; b < 256; ++b) {
      uint32_t r = b;
      for (int i = 0; i < 8; ++i) r = lnx::zbit(r);
      t[0][b] = r;
    }
    for (int k = 1; k < 16; ++k)
      for (uint32_t b = 0; b < 256; ++b) t[k][b] = (t[k - 1][b] >> 8) ^ t[0][t[k - 1][b] & 0xffu];
  }
};
const Slice16 kTab;

inline uint32_t load_le32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;  // x86-64 and the GPU are little-endian
}

// Register update without init/xorout: r over bytes p[0..n).
uint32_t reg_update(uint32_t r, const uint8_t* p, size_t n) {
  const auto& t = kTab.t;
  while (n >= 16) {
    const uint32_t a = load_le32(p) ^ r, b = load_le32(p + 4), c = load_le32(p + 8), d = load_le32(p + 12);
    r = t[15][a & 0xff] ^ t[14][(a >> 8) & 0xff] ^ t[13][(a >> 16) & 0xff] ^ t[12][a >> 24] ^
        t[11][b & 0xff] ^ t[10][(b >> 8) & 0xff] ^ t[9][(b >> 16) & 0xff] ^ t[8][b >> 24] ^
        t[7][c & 0xff] ^ t[6][(c >> 8) & 0xff] ^ t[5][(c >> 16) & 0xff] ^ t[4][c >> 24] ^
        t[3][d & 0xff] ^ t[2][(d >> 8) & 0xff] ^ t[1][(d >> 16) & 0xff] ^ t[0][d >> 24];
    p += 16;
    n -= 16;
  }
  while (n--) r = (r >> 8) ^ t[0][(r ^ *p++) & 0xffu];
  return r;
}

}  // namespace

extern "C" {

uint32_t lnx_crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
  if (n == 0) return crc;
  return ~reg_update(~crc, p, n);
}

uint32_t lnx_crc32(const uint8_t* p, size_t n) { return lnx_crc32_update(0, p, n); }

int64_t lnx_crc32_search(const uint8_t* p, size_t n, int64_t min_off) {
  // ethernet/crc.go:28-47: clamp, length guard, incremental per-byte extension.
  if (min_off < 0) min_off = 0;
  if ((int64_t)n < min_off + 4) return -1;
  uint32_t crc = lnx_crc32(p, (size_t)min_off);
  for (int64_t off = min_off; off <= (int64_t)n - 4; ++off) {
    if (crc == load_le32(p + off)) return off;
    crc = lnx_crc32_update(crc, p + off, 1);
  }
  return -1;
}

uint32_t lnx_sum_write_even(uint32_t sum, const uint8_t* p, size_t n) {
  for (size_t i = 0; i + 1 < n; i += 2) sum += (uint32_t)((p[i] << 8) | p[i + 1]);
  return sum;
}

uint16_t lnx_sum16(uint32_t sum) {
  sum = (sum & 0xffffu) + (sum >> 16);
  return (uint16_t)~(uint16_t)(sum + (sum >> 16));
}

uint16_t lnx_sum16_payload(uint32_t sum, const uint8_t* p, size_t n) {
  const size_t odd = n & 1u;
  sum = lnx_sum_write_even(sum, p, n - odd);
  if (odd) sum += (uint32_t)p[n - 1] << 8;
  return lnx_sum16(sum);
}

uint16_t lnx_never_zero_sum(uint16_t s) { return s == 0 ? 0xffff : s; }

}  // extern "C"
