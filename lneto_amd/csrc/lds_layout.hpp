// lds_layout.hpp — byte layout of the 160 KiB LDS image of the CRC-32 kernel.
//
// One 1024-thread workgroup per CU holds the whole image.  Every table is
// "lane-private": lane l only ever reads LDS bank (l % 32), so the 64 lanes of
// a ds_read_b32 (serviced as two 32-lane groups) never conflict whatever the
// data-dependent index is.  Measured on MI355X: ~21-24 lookups/clk/CU this way
// vs ~9.9 for one shared table with random indices.
//
// U region [0, 128 KiB): the stride map U = Z_256 (advance the CRC register
// over 256 bytes) split into four byte tables U_m[e] = Z_256(e << 8m):
//     byte address = (m>>1)<<16 | e<<8 | (m&1)<<7 | c<<2        (c = lane%32)
// so the address of U_m[byte k of x] is v_perm(x, base_m, sel_k) — one VALU op:
// byte 1 of the address is the data byte, bytes 0 and 2 come from a per-lane
// base.  m&1 is folded into the ds_read immediate offset (+128).
//
// F region [128 KiB, 160 KiB): per-lane final alignment F_l = Z_{-4l} (lane l's
// register ends 4l bytes past the frame end) as eight 16-entry nibble tables:
//     byte address = 128K | h<<14 | i<<11 | v<<7 | c<<2    (h = l/32, nibble i, value v)
// F_l(r) = XOR_i F_l,i[(r >> 4i) & 15].  The content differs per lane; lanes l
// and l+32 share a bank column and are separated by h.
#pragma once
#include <cstdint>

namespace lnx {

constexpr uint32_t kWindowBytes = 256;   // bytes one wave consumes per step (64 lanes x 4 B)
constexpr uint32_t kLdsBytes = 163840;   // 160 KiB
constexpr uint32_t kLdsDwords = kLdsBytes / 4;
constexpr uint32_t kFBase = 131072;      // start of the F region

constexpr uint32_t u_addr(uint32_t m, uint32_t e, uint32_t c) {
  return ((m >> 1) << 16) | (e << 8) | ((m & 1) << 7) | (c << 2);
}
constexpr uint32_t f_addr(uint32_t lane, uint32_t nib, uint32_t v) {
  return kFBase | ((lane >> 5) << 14) | (nib << 11) | (v << 7) | ((lane & 31) << 2);
}

}  // namespace lnx
