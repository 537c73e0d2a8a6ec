// lds_layout.hpp — geometry of the CRC-32 kernel and byte layout of its LDS images.
//
// Geometry: a wave is 64/RL "rows" of RL lanes; each row folds one frame.  Lane
// p of a row (p = lane % RL) consumes the 4-byte word at window offset
// 4p + SB*j, SB = 4*RL, so a row advances SB bytes per step.  Two row widths
// exist: RL = 16 (4 frames per wave, 64-byte steps) for long
// frames and RL = 4 (16 frames per wave, 16-byte steps) for short ones.  Each
// has its own 160 KiB image; a workgroup loads the one its frames call for.
//
// One 1024-thread workgroup per CU holds the image.  Every table is
// "lane-private": lane l only ever reads LDS bank (l % 32), so a ds_read_b32
// (serviced as two 32-lane groups) never conflicts whatever the data-dependent
// index is.  Measured on MI355X: ~21-24 lookups/clk/CU this way vs ~9.9 for a
// shared table with random indices.
//
// U region [0, 128 KiB): the row stride map U = Z_SB (advance the CRC register
// over SB bytes) as four byte tables U_m[e] = Z_SB(e << 8m):
//     byte address = (m>>1)<<16 | e<<8 | (m&1)<<7 | c<<2        (c = lane%32)
// so the address of U_m[byte k of x] is v_perm(x, base_m, sel_k) — one VALU op:
// byte 1 of the address is the data byte, bytes 0 and 2 come from a per-lane
// base; m&1 is folded into the ds_read immediate offset (+128).
//
// F region [128 KiB, 144 KiB): per-lane final alignment F_p = Z_{-4p} (lane p's
// register ends 4p bytes past the window end) as eight 16-entry nibble tables,
// interleaved in pairs like the U tables (nibbles 2k and 2k+1 share 256-byte
// rows):
//     byte address = 128K | (i>>1)<<12 | v<<8 | (i&1)<<7 | c<<2   (nibble i, value v)
// F_p(r) = XOR_i F_p,i[(r >> 4i) & 15]; column c holds the tables of
// p = c % RL, which serves lanes c and c+32 alike.  With y = r & 0x0F0F0F0F and
// z = (r >> 4) & 0x0F0F0F0F, nibble 2k is byte k of y and nibble 2k+1 byte k
// of z, so every address is one v_perm of y or z with the lane's base (byte 1
// = the nibble, byte 2 = 0x02 from 128K) plus an immediate (k<<12 | (i&1)<<7).
//
// T region [144 KiB, 156 KiB): the window ends at the frame end rounded up to
// 4 bytes, t = 0..3 bytes past it, so the row's register needs Z_{-t} too.  The
// row's lanes share that work by nibble: entry (h, t, v) of column c, t = 1..3,
// is Z_{-t}(v << 4q_h) with q_0 = (c % RL) & 7 and q_1 = q_0 + 4 (h = 1 is used
// by RL = 4 only, where each lane covers two nibbles); t = 0 is the identity
// and needs no table:
//     byte address = 144K | (48h + 16(t-1) + v)<<7 | c<<2
//
// [156 KiB, 160 KiB): zero in the image; the workgroup's frame-chunk counter
// lives at kCtrBase (DESIGN.md §3.1 "work distribution").
#pragma once
#include <cstdint>

namespace lnx {

constexpr uint32_t kLdsBytes = 163840;             // 160 KiB (whole CU)
constexpr uint32_t kLdsDwords = kLdsBytes / 4;
constexpr uint32_t kFBase = 131072;                // start of the F region
constexpr uint32_t kTBase = 147456;                // start of the T region
constexpr uint32_t kCtrBase = 159744;              // frame-chunk counter (one dword)
constexpr int kImageCount = 6;  // images: [0] RL = 16, [1] RL = 4, [2] RL = 32, [3] stream, [4] stream64, [5] lanes
// the streaming rows' image (stream_rows.hpp): U = Z_4, F column n = Z_{-4n},
// then the Z_116 / Z_c / Z_{128-4k} / Z_1 tables at these byte addresses
constexpr uint32_t kSZ116 = 147456;  // Z_{SB-12} byte tables (Z_116 / Z_52): entry (m, e) at 1024m + 4e
constexpr uint32_t kSTc = 151552;    // Z_c, c = 0..3, nibble p of the row: dword ((c*8 + p)*16 + v)
constexpr uint32_t kSG = 153600;     // Z_{128-4k}, k = 0..4, nibble p: dword ((k*8 + p)*16 + v)
constexpr uint32_t kSK = 156160;     // Z_{128-j}(0xFFFFFFFF), j = 0..15
constexpr uint32_t kST1 = 156224;    // Z_1 byte table (slow-path byte steps)
// the lane streams' image (stream_lanes.hpp): U = Z_4, then Z_c byte tables
// (c = 1..3: dword (c-1)*1024 + 256m + e), Z_{64-4k} nibble tables (k = 0..15:
// dword 128k + 16i + v) and the constants Z_{64-j}(0xFFFFFFFF), j = 0..63
constexpr uint32_t kLZc = 131072;
constexpr uint32_t kLZd = kLZc + 12288;
constexpr uint32_t kLK = kLZd + 8192;

constexpr uint32_t u_addr(uint32_t m, uint32_t e, uint32_t c) {
  return ((m >> 1) << 16) | (e << 8) | ((m & 1) << 7) | (c << 2);
}
constexpr uint32_t f_addr(uint32_t c, uint32_t nib, uint32_t v) {
  return kFBase | ((nib >> 1) << 12) | (v << 8) | ((nib & 1) << 7) | (c << 2);
}
constexpr uint32_t t_addr(uint32_t c, uint32_t h, uint32_t t, uint32_t v) {  // t = 1..3
  return kTBase + ((48u * h + 16u * (t - 1) + v) << 7) + (c << 2);
}
static_assert(t_addr(31, 1, 3, 15) < kCtrBase, "T region overlaps the counter");
// (8 and 9: the streaming rows' images with 128- and 64-byte row steps; 10: the lane streams')
constexpr int image_index(int rl) {
  return rl == 16 ? 0 : rl == 4 ? 1 : rl == 8 ? 3 : rl == 9 ? 4 : rl == 10 ? 5 : 2;
}

// Compact image in HBM (what a workgroup reads at start): the 1024 distinct U
// values U_m[e] at dword 256m + e, then the [kFBase, kLdsBytes) tail of the
// LDS image verbatim (F, T, the zero counter).  The kernel writes each U value
// into its 32 bank replicas itself, so a workgroup reads 36 KiB instead of
// 160 KiB before its first frame load.
constexpr uint32_t kCompactUDwords = 1024;
constexpr uint32_t kCompactDwords = kCompactUDwords + (kLdsBytes - kFBase) / 4;

}  // namespace lnx
