// rows_emulator.cpp — CPU emulation of one row of crc32_rows_kernel, lane by
// lane, reading the real LDS images that liblneto_amd builds (api.cpp
// build_lds_image) at the byte addresses the kernel uses.  Checks the window
// geometry (aligned window end, lead-in mask, init fold and its spill, junk
// removal, F_p, row XOR, Z_{-t} fix) against a plain table CRC-32 for every
// length 0..N at every start alignment and in every row of the wave, for all
// three row widths (32-lane rows: line-aligned window, junk lanes skipping the
// last step, register rotation before F; lean line rows: two words per lane,
// F columns chosen per virtual lane instead of a rotation).  No GPU: this pins
// the algebra and the table contents on the CPU.
// Built and run by tests/test_abi.py.
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
#include "../../lneto_amd/csrc/lds_layout.hpp"

namespace lnx {
std::vector<uint32_t> build_lds_image(uint32_t rl);
}
using namespace lnx;

static uint32_t crc_tab[256];
static uint32_t ref_crc(const uint8_t* p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; ++i) c = crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
  return ~c;
}

struct Emu {
  int RL;
  std::vector<uint32_t> img;
  uint32_t rd(uint32_t byte_addr) const { return img[byte_addr / 4]; }
  uint32_t U(uint32_t x, uint32_t c) const {  // u_step: byte m of x -> U_m
    uint32_t r = 0;
    for (uint32_t m = 0; m < 4; ++m) r ^= rd(u_addr(m, (x >> (8 * m)) & 0xFF, c));
    return r;
  }
  uint32_t F(uint32_t r, uint32_t c) const {
    uint32_t a = 0;
    for (uint32_t i = 0; i < 8; ++i) a ^= rd(f_addr(c, i, (r >> (4 * i)) & 15));
    return a;
  }
  // word at rel position pos of the wave's range [0, size): out-of-range reads 0
  static uint32_t word(const std::vector<uint8_t>& buf, int64_t pos) {
    if (pos < 0 || pos + 4 > (int64_t)buf.size()) return 0;
    uint32_t w;
    memcpy(&w, &buf[pos], 4);
    return w;
  }
  static uint32_t keep_from(int32_t lo) {
    lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
    return (uint32_t)(0xFFFFFFFFull << (8 * lo));
  }
  // 32-lane rows (crc32_kernel.hip rows_body, RL = 32): the window runs from
  // the 128-byte line holding the frame start to the end of the line holding
  // its last byte, so every step reads one whole line.  t = 4a + b window bytes
  // follow the frame end: lanes p >= 32 - a hold only those in the last step
  // and skip it, lane 31 - a (when b > 0) takes the U-image of its b junk bytes
  // out, and the registers are rotated by a lanes so that lane q's own F_q
  // lands every one of them on the frame end less b bytes; Z_{-b} finishes.
  uint32_t crc32w(const std::vector<uint8_t>& buf, uint32_t rs, uint32_t re) const {
    const uint32_t SB = 128;
    const uint32_t n = re > rs ? re - rs : 0;
    const uint32_t ea = (re + SB - 1) & ~(SB - 1), t = ea - re, a = t >> 2, b = t & 3;
    const uint32_t J = n ? (n + t + SB - 1) / SB : 0;
    const int64_t ws = (int64_t)ea - (int64_t)J * SB;
    const uint32_t lead = J * SB - n - t;
    std::vector<uint32_t> lanes(32);
    for (uint32_t p = 0; p < 32; ++p) {
      const uint32_t m4 = n < 4 ? n : 4;
      const int32_t d0 = (int32_t)lead - (int32_t)(4 * p);
      const uint32_t keep = keep_from(d0), initm = keep & ~keep_from(d0 + (int32_t)m4);
      const int32_t x1 = (int32_t)(lead + m4) - (int32_t)SB;
      const uint32_t m1 = (x1 > 0 && p == 0) ? (uint32_t)((1ull << (8 * x1)) - 1) : 0;
      const uint32_t Jp = (J && p >= 32 - a) ? J - 1 : J;
      uint32_t reg = 0;
      for (uint32_t j = 0; j < Jp; ++j) {
        uint32_t x = word(buf, ws + 4 * p + (int64_t)SB * j);
        if (j == 0) x = (x & keep) ^ initm;
        if (j == 1) x ^= m1;
        reg = U(reg ^ x, p);
      }
      if (J && b && p == 31 - a) {
        const uint32_t junk = word(buf, (int64_t)ea - SB + 4 * p) & ~(uint32_t)(0xFFFFFFFFull >> (8 * b));
        reg ^= U(junk, p);
      }
      lanes[p] = reg;
    }
    uint32_t R = 0;
    for (uint32_t q = 0; q < 32; ++q) R ^= F(lanes[(q - a) & 31], q);  // rotation, F_q, row_xor
    uint32_t T = 0;
    for (uint32_t p = 0; p < 8; ++p) {
      const uint32_t nib = (R >> (4 * p)) & 15;
      T ^= b ? rd(t_addr(p, 0, b, nib)) : nib << (4 * p);
    }
    R = n ? T : 0;
    if (n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * n));
    return ~R;
  }
  // Lean line rows (crc32_kernel.hip lines_body): 16 lanes, lane p loads the
  // 8 bytes at 8p + 128j (virtual lanes v = 2p, 2p + 1), window = the lines
  // holding the frame, junk lanes v >= 32 - a skip the last step, virtual lane
  // 31 - a takes its b junk bytes' U-image out, and with no rotation virtual
  // lane v's register takes F_q, q = (v + a) mod 32, from column q of the
  // RL = 32 image; then Z_{-b} as t_fix<16> shares it over the row's lanes.
  uint32_t crc32lean(const std::vector<uint8_t>& buf, uint32_t rs, uint32_t re, uint32_t row) const {
    const uint32_t n = re > rs ? re - rs : 0;
    const uint32_t wend = (re + 127) & ~127u, ws = rs & ~127u, t = wend - re, a = t >> 2, b = t & 3;
    const uint32_t J = n ? (wend - ws) >> 7 : 0, lead = rs - ws, m4 = n < 4 ? n : 4;
    auto keep8 = [](int32_t d) -> uint64_t {
      const uint32_t q = 4u * (uint32_t)(d < 0 ? 0 : (d > 8 ? 8 : d));
      return (~0ull << q) << q;
    };
    uint32_t R = 0;
    for (uint32_t p = 0; p < 16; ++p) {
      const uint32_t col = (row * 16 + p) % 32;
      const int32_t d0 = (int32_t)lead - (int32_t)(8 * p);
      const uint64_t keep = keep8(d0), initm = keep & ~keep8(d0 + (int32_t)m4);
      const int32_t x1 = (int32_t)(lead + m4) - 128;
      const uint32_t m1 = (x1 > 0 && p == 0) ? (uint32_t)((1ull << (8 * x1)) - 1) : 0;
      for (uint32_t h = 0; h < 2; ++h) {
        const uint32_t v = 2 * p + h;
        const uint32_t nsl = J ? J - (v >= 32 - a ? 1 : 0) : 0;
        uint32_t reg = 0;
        for (uint32_t j = 0; j < nsl; ++j) {
          uint64_t q;
          memcpy(&q, &buf[ws + 8 * p + 128 * j], 8);
          if (j == 0) q = (q & keep) ^ initm;
          uint32_t x = (uint32_t)(q >> (32 * h));
          if (j == 1 && v == 0) x ^= m1;
          reg = U(reg ^ x, col);
        }
        if (J && b && v == 31 - a) {
          const uint32_t junk = word(buf, (int64_t)ws + 128 * (J - 1) + 4 * v) & ~(uint32_t)(0xFFFFFFFFull >> (8 * b));
          reg ^= U(junk, col);
        }
        R ^= F(reg, (v + a) & 31);
      }
    }
    uint32_t T = 0;
    for (uint32_t p = 0; p < 8; ++p) {
      const uint32_t c = (row * 16 + p) % 32, nib = (R >> (4 * (p & 7))) & 15;
      T ^= b ? rd(t_addr(c, 0, b, nib)) : nib << (4 * (p & 7));
    }
    R = n ? T : 0;
    if (n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * n));
    return ~R;
  }
  // CRC of frame [rs, re) of buf as row `row` of a wave would compute it.
  uint32_t crc(const std::vector<uint8_t>& buf, uint32_t rs, uint32_t re, uint32_t row) const {
    const uint32_t SB = 4 * RL;
    const uint32_t n = re > rs ? re - rs : 0;
    const uint32_t ea = (re + 3) & ~3u, t = ea - re;
    const uint32_t J = n ? (n + t + SB - 1) / SB : 0;
    const int64_t ws = (int64_t)ea - (int64_t)J * SB;
    const uint32_t lead = J * SB - n - t;
    std::vector<uint32_t> lanes(RL);
    for (uint32_t p = 0; p < (uint32_t)RL; ++p) {
      const uint32_t c = (row * RL + p) % 32;
      const uint32_t m4 = n < 4 ? n : 4;
      const int32_t d0 = (int32_t)lead - (int32_t)(4 * p);
      const uint32_t keep = keep_from(d0), initm = keep & ~keep_from(d0 + (int32_t)m4);
      const int32_t x1 = (int32_t)(lead + m4) - (int32_t)SB;
      const uint32_t m1 = (x1 > 0 && p == 0) ? (uint32_t)((1ull << (8 * x1)) - 1) : 0;
      uint32_t reg = 0;
      for (uint32_t j = 0; j < J; ++j) {
        uint32_t x = word(buf, ws + 4 * p + (int64_t)SB * j);
        if (j == 0) x = (x & keep) ^ initm;
        if (j == 1) x ^= m1;
        reg = U(reg ^ x, c);
      }
      if (J && t && p == (uint32_t)RL - 1) {
        const uint32_t junk = word(buf, (int64_t)ea - 4) & ~(uint32_t)(0xFFFFFFFFull >> (8 * t));
        reg ^= U(junk, c);
      }
      lanes[p] = F(reg, c);
    }
    uint32_t R = 0;
    for (uint32_t v : lanes) R ^= v;  // row_xor
    // t_fix: lane-shared nibble lookups, XOR-reduced as the DPP steps do
    uint32_t T = 0;
    auto tl = [&](uint32_t c, uint32_t h, uint32_t q) {  // t = 0: identity, no table
      const uint32_t nib = (R >> (4 * q)) & 15;
      return t ? rd(t_addr(c, h, t, nib)) : nib << (4 * q);
    };
    if (RL == 16) {
      for (uint32_t p = 0; p < 8; ++p) {  // lanes 0-3 and 4-7 of the reduction of lane 0
        const uint32_t c = (row * RL + p) % 32;
        T ^= tl(c, 0, p & 7);
      }
    } else {
      for (uint32_t p = 0; p < 4; ++p) {
        const uint32_t c = (row * RL + p) % 32;
        T ^= tl(c, 0, p) ^ tl(c, 1, p + 4);
      }
    }
    R = n ? T : 0;
    if (n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * n));
    return ~R;
  }
};

int main() {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c >> 1) ^ ((c & 1) ? 0xEDB88320u : 0);
    crc_tab[i] = c;
  }
  std::vector<uint8_t> buf(8192);
  uint64_t s = 0x6C6E65746FULL;
  for (auto& b : buf) {
    s = s * 6364136223846793005ULL + 1442695040888963407ULL;
    b = (uint8_t)(s >> 56);
  }
  int bad = 0, checked = 0;
  for (int rl : {32, 16, 4}) {
    Emu e{rl, build_lds_image((uint32_t)rl)};
    const uint32_t nr = 64 / rl;
    for (uint32_t n = 0; n <= 1100; ++n) {
      for (uint32_t start : {0u, 1u, 2u, 3u, 61u, 124u, 125u, 127u, 128u, 130u, 4093u}) {
        if (start + n > buf.size()) continue;
        const uint32_t row = (n + start) % nr;
        const uint32_t got = rl == 32 ? e.crc32w(buf, start, start + n) : e.crc(buf, start, start + n, row);
        const uint32_t want = ref_crc(&buf[start], n);
        ++checked;
        if (got != want && bad++ < 10)
          printf("RL=%d n=%u start=%u row=%u: got %08x want %08x\n", rl, n, start, row, got, want);
      }
    }
  }
  {  // lean line rows: the RL = 32 image, rows 0..3 of a wave
    Emu e{32, build_lds_image(32u)};
    for (uint32_t n = 0; n <= 1700; ++n) {
      for (uint32_t start : {128u, 129u, 130u, 131u, 189u, 252u, 253u, 255u, 256u, 258u, 4221u}) {
        if (start + n + 256 > buf.size()) continue;
        const uint32_t row = (n + start) % 4;
        const uint32_t got = e.crc32lean(buf, start, start + n, row);
        const uint32_t want = ref_crc(&buf[start], n);
        ++checked;
        if (got != want && bad++ < 10) printf("lean n=%u start=%u row=%u: got %08x want %08x\n", n, start, row, got, want);
      }
    }
  }
  printf("rows emulator: %d of %d frames wrong\n", bad, checked);
  return bad ? 1 : 0;
}
