// lds_layout.hpp — geometry of the CRC-32 kernel and byte layout of its LDS image.
//
// Geometry: a wave is four 16-lane "rows"; each row folds one frame.  Lane p of
// a row (p = lane % 16) consumes the 4-byte word at window offset 4p + 64j, so
// a row advances 64 bytes per step and a wave 256 bytes per dword load.
//
// One 1024-thread workgroup per CU holds the image.  Every table is
// "lane-private": lane l only ever reads LDS bank (l % 32), so a ds_read_b32
// (serviced as two 32-lane groups) never conflicts whatever the data-dependent
// index is.  Measured on MI355X: ~21-24 lookups/clk/CU this way vs ~9.9 for a
// shared table with random indices.
//
// U region [0, 128 KiB): the row stride map U = Z_64 (advance the CRC register
// over 64 bytes) as four byte tables U_m[e] = Z_64(e << 8m):
//     byte address = (m>>1)<<16 | e<<8 | (m&1)<<7 | c<<2        (c = lane%32)
// so the address of U_m[byte k of x] is v_perm(x, base_m, sel_k) — one VALU op:
// byte 1 of the address is the data byte, bytes 0 and 2 come from a per-lane
// base; m&1 is folded into the ds_read immediate offset (+128).
//
// F region [128 KiB, 144 KiB): per-lane final alignment F_p = Z_{-4p} (lane p's
// register ends 4p bytes past the frame end) as eight 16-entry nibble tables:
//     byte address = 128K | i<<11 | v<<7 | c<<2          (nibble i, value v)
// F_p(r) = XOR_i F_p,i[(r >> 4i) & 15]; column c holds the tables of p = c%16,
// which serves lanes c and c+32 alike.  [144 KiB, 160 KiB) is unused.
#pragma once
#include <cstdint>

namespace lnx {

constexpr uint32_t kRowLanes = 16;                 // lanes folding one frame
constexpr uint32_t kStepBytes = kRowLanes * 4;     // bytes a row consumes per step
constexpr uint32_t kLdsBytes = 163840;             // 160 KiB (whole CU)
constexpr uint32_t kLdsDwords = kLdsBytes / 4;
constexpr uint32_t kFBase = 131072;                // start of the F region

constexpr uint32_t u_addr(uint32_t m, uint32_t e, uint32_t c) {
  return ((m >> 1) << 16) | (e << 8) | ((m & 1) << 7) | (c << 2);
}
constexpr uint32_t f_addr(uint32_t c, uint32_t nib, uint32_t v) {
  return kFBase | (nib << 11) | (v << 7) | (c << 2);
}

}  // namespace lnx
