// gf2.hpp — CRC-32/IEEE register algebra used to build the kernels' tables.
//
// The CRC register here is the reflected 32-bit register of CRC-32/ISO-HDLC
// (poly 0x04C11DB7 reflected = 0xEDB88320), the algorithm Go's hash/crc32
// implements for crc32.IEEETable (the table lneto builds at ethernet/crc.go:13).
//
// Z_k denotes "advance the register over k zero bytes".  It is GF(2)-linear and
// invertible (P has a non-zero constant term), so Z_k is defined for negative k
// too.  Processing a 32-bit little-endian word w at a register r is Z_4(r ^ w);
// every table in this library is a byte/nibble decomposition of some Z_k.
#pragma once
#include <cstdint>

namespace lnx {

constexpr uint32_t kPolyReflected = 0xEDB88320u;

// One zero bit forward: r' = r*x mod P in the reflected representation.
constexpr uint32_t zbit(uint32_t r) { return (r >> 1) ^ ((r & 1u) ? kPolyReflected : 0u); }

// One zero bit backward (inverse of zbit).  Bit 31 of zbit(r) equals r&1
// because the reflected poly has bit 31 set and r>>1 has bit 31 clear.
constexpr uint32_t unzbit(uint32_t r) {
  const uint32_t b = r >> 31;
  const uint32_t t = b ? (r ^ kPolyReflected) : r;
  return (t << 1) | b;
}

// Z_k for a small |k| (bit-serial; used only to build tables).
constexpr uint32_t zshift_bytes(uint32_t r, int64_t k) {
  if (k >= 0) {
    for (int64_t i = 0; i < 8 * k; ++i) r = zbit(r);
  } else {
    for (int64_t i = 0; i < -8 * k; ++i) r = unzbit(r);
  }
  return r;
}

// a*b mod P for two reflected polynomials (zlib's multmodp idea).
constexpr uint32_t multmodp(uint32_t a, uint32_t b) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = zbit(b);
  }
  return p;
}

// x^(8k) mod P for any k >= 0 (square-and-multiply); x^0 is 0x80000000.
inline uint32_t x8kmodp(uint64_t k) {
  uint32_t result = 0x80000000u;
  uint32_t sq = zshift_bytes(0x80000000u, 1);  // x^8
  while (k) {
    if (k & 1) result = multmodp(sq, result);
    sq = multmodp(sq, sq);
    k >>= 1;
  }
  return result;
}

// Z_k(r) for any k >= 0 in O(log k).
inline uint32_t zshift_bytes_fast(uint32_t r, uint64_t k) { return multmodp(x8kmodp(k), r); }

}  // namespace lnx
