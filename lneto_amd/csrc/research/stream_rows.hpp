// stream_rows.hpp — streaming rows for short frames, included
// by crc32_kernel.hip after its helpers.  The host-side restatement of this
// schedule, checked against zlib, is tests/stream_algebra.py.
//
// The narrow rows fetch every frame's lines on their own: a line two frames
// share is requested by both rows, and a 16-byte row piece touches a line
// eight times; on the Zipf mix (configs[3], mean 246 B) that is 56 M L2
// requests for 32 M lines and the load side alone takes 1.0 ms.  A streaming
// row instead walks a contiguous run of frames one whole 128-byte line per
// step (8 lanes x buffer_load_dwordx4), so each line is requested once: the
// loads alone stream the mix at 0.59 ms (tools/ubench/pattern5.hip).
//
// Lane p of a row holds bytes [L + 16p, L + 16p + 16) of line L and ONE
// register r, its share of the running CRC state of the row's byte stream:
//     y0 = r ^ w0, y1 = Z4(y0) ^ w1, y2 = Z4(y1) ^ w2, y3 = Z4(y2) ^ w3,
//     ra = Z116(y3)        (Z4: the lane-private U image; Z116: shared tables)
// A frame boundary x in the line (an "event") combines the lanes into the
// stream's state there: lanes before x's lane use ra, lanes after it r, x's
// own lane the chain value y_k of x's dword with the c = x & 3 bytes before x
// kept; each value through F column n (Z_{-4n}), the row's XOR, then Z_c.  The
// event's frame CRC is ~S; the next frame starts by injecting ~S at x (into
// x's lane's ra, shifted forward to its position), which sets the stream's
// state at x to 0xFFFFFFFF, the CRC init: no per-frame length operator, no
// lead-in or tail masks, and the junk before a row's first frame cancels.
//
// Work: the workgroup's slice of frames is split evenly over its 128 rows
// (16 waves x 8 rows); each row's frame boundaries come from an 8-offset
// block per row held across its lanes, with the next block requested one
// ring slot ahead.  Every step issues exactly three VMEM instructions (the
// line, the offset block request, the held results' store; out-of-range
// offsets when a row has nothing to move), so the ring's vmcnt is static.
#pragma once
// (included inside namespace lnx)

// stream image tail: lds_layout.hpp kSZ116 .. kST1
static_assert(kST1 + 1024 <= kCtrBase, "stream tables overlap the counter");

__device__ __forceinline__ uint32_t z116(const char* lds, uint32_t y) {
  const uint32_t a0 = kSZ116 + ((y & 0xFFu) << 2);
  const uint32_t a1 = kSZ116 + 1024u + (__builtin_amdgcn_ubfe(y, 8, 8) << 2);
  const uint32_t a2 = kSZ116 + 2048u + (__builtin_amdgcn_ubfe(y, 16, 8) << 2);
  const uint32_t a3 = kSZ116 + 3072u + ((y >> 24) << 2);
  return __builtin_amdgcn_bitop3_b32(lds_rd(lds, a0), lds_rd(lds, a1), lds_rd(lds, a2), 0x96) ^ lds_rd(lds, a3);
}
// XOR over the 8 lanes of a row (quads, then the two quads by half-mirror)
__device__ __forceinline__ uint32_t row8_xor(uint32_t v) {
  v = dpp_xor<kQuadX1>(v);
  v = dpp_xor<kQuadX2>(v);
  return dpp_xor<0x141>(v);  // row_half_mirror: lane i <-> 7 - i within each 8
}
// Z_1 byte step (x: register, one zero byte)
__device__ __forceinline__ uint32_t z1(const char* lds, uint32_t x) {
  return lds_rd(lds, kST1 + ((x & 0xFFu) << 2)) ^ (x >> 8);
}

// XOR over the RLS lanes of a row
template <int RLS>
__device__ __forceinline__ uint32_t rowx(uint32_t v) {
  if constexpr (RLS == 8) return row8_xor(v);
  v = dpp_xor<kQuadX1>(v);
  return dpp_xor<kQuadX2>(v);
}

// RLS: lanes per row (8: one 128-byte line per row step, the stream image;
// 4: a 64-byte half line, the stream64 image).  With 4-lane rows a frame of
// at least 64 bytes ends at most once per row step, so a step takes one
// boundary pass where 8-lane rows take up to two.
template <CrcMode MODE, int VAR, int RLS = 8, int D = 4>
__device__ __forceinline__ void stream_body(const char* lds, const Lanes& L, const WaveCtx& cx) {
  static_assert(MODE != CrcMode::kAppend, "offsets mode only");
  static_assert(RLS == 8 || RLS == 4, "row width");
  constexpr uint32_t SB = 16u * RLS;                  // bytes per row step
  constexpr uint32_t kRowLog = RLS == 8 ? 7 : 8;      // log2(rows per workgroup)
  constexpr int OPL = 8 / RLS;                        // offsets per lane in an 8-event block
  const uint32_t p = L.p;  // lane of the row
  const uint32_t bu0 = L.bu0, bu1 = L.bu1;
  const uint32_t nfb = cx.nfb, o0_lo = cx.o0_lo, adj = cx.adj;
  const __amdgpu_buffer_rsrc_t data_rsrc = cx.data_rsrc, off_rsrc = cx.off_rsrc, out_rsrc = cx.out_rsrc;
  auto rel = [&](uint32_t x_lo) -> uint32_t { return x_lo - o0_lo + adj; };

  // ---- the row's frames: [fr0, fr0 + m) of the range, events 0..m at off[fr0 + k]
  const uint32_t jrow = threadIdx.x / RLS;
  const uint32_t fr0 = (uint32_t)(((uint64_t)jrow * nfb) >> kRowLog),
                 fr1 = (uint32_t)(((uint64_t)(jrow + 1) * nfb) >> kRowLog);
  const uint32_t m = fr1 - fr0;
  // first two offset blocks and the last event, synchronously
  auto ld_off = [&](uint32_t k) -> uint32_t {  // low dword of off[fr0 + k], k <= m; junk otherwise
    return __builtin_amdgcn_raw_buffer_load_b32(off_rsrc, k <= m ? (fr0 + k) * 8u : kOOB, 0, 0);
  };
  // lane p holds events kb + p + RLS*i of the block in A[i] (the next block in B)
  uint32_t A[OPL], B[OPL];
#pragma unroll
  for (int i = 0; i < OPL; ++i) A[i] = rel(ld_off(p + RLS * i)), B[i] = rel(ld_off(8 + p + RLS * i));
  const uint32_t xm = rel(__builtin_amdgcn_raw_buffer_load_b32(off_rsrc, fr1 * 8u, 0, 0));
  uint32_t kb = 0;             // event index of A's lane 0
  bool hasB = m >= 8;          // B holds events kb + 8 ..
  bool reqd = false;           // B's block requested, arriving in ob[reqs]
  uint32_t reqs = 0;
  const uint32_t rowbase = (threadIdx.x & 63u) & ~(RLS - 1u);
  auto pick = [&](uint32_t j) -> uint32_t {  // event kb + j, j < 16: from A (j < 8) or B
    uint32_t v = j < 8u ? A[0] : B[0];
    if constexpr (OPL == 2) v = ((j >> 2) & 1u) ? (j < 8u ? A[1] : B[1]) : v;
    return (uint32_t)__builtin_amdgcn_ds_bpermute((int)((rowbase + (j & (RLS - 1u))) << 2), (int)v);
  };
  uint32_t k = 0;                         // next event
  uint32_t x = pick(0);                   // its position
  uint32_t Lr = x & ~(SB - 1u);           // the row's current line (row step)
  const uint32_t Lend = xm & ~(SB - 1u);  // its last one
  uint32_t xs = x;                        // the previous event (verify: frame length)
  uint32_t r = 0;                         // the lane's chain register
  uint32_t P = 0, xprev = 0, pprev = 0xFFu;  // same-piece events (frames < 16 B)
  uint32_t hv = 0, hf = 0, hc = 0;        // held results: lane p < hc holds one
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- ring: D steps of (line, offset block) in flight, three VMEM per step.
  // R = D + 1 register sets: step t's loads go into set t mod R and the load
  // for step t + D into the set step t - 1 used, which is dead by then — a
  // set still holding this step's line would make hipcc copy it to another
  // register above the ring's wait (tools/prof/audit_ring.py).
  constexpr int R = D + 1;
  u32x4 w[R];
  uint32_t ob[R][OPL];
  auto issue = [&](int s, uint32_t line, bool req, uint32_t kreq) {
    const uint32_t vl = line <= Lend ? line + 16u * p : kOOB;
    const uint32_t vo = req && kreq + p <= m ? (fr0 + kreq + p) * 8u : kOOB;
    asm volatile("s_nop 4\n\tbuffer_load_dwordx4 %0, %2, %4, 0 offen\n\tbuffer_load_dword %1, %3, %5, 0 offen"
                 : "=&v"(w[s]), "=&v"(ob[s][0])
                 : "v"(vl), "v"(vo), "s"(data_rsrc), "s"(off_rsrc));
    if constexpr (OPL == 2) {
      const uint32_t vo1 = req && kreq + p + RLS <= m ? (fr0 + kreq + p + RLS) * 8u : kOOB;
      asm volatile("buffer_load_dword %0, %1, %2, 0 offen" : "=&v"(ob[s][1]) : "v"(vo1), "s"(off_rsrc));
    }
  };
  auto store_held = [&]() {
    const uint32_t a = p < hc ? (MODE == CrcMode::kCrc ? hf * 4u : hf) : kOOB;
    if constexpr (MODE == CrcMode::kCrc)
      asm volatile("buffer_store_dword %0, %1, %2, 0 offen" ::"v"(hv), "v"(a), "s"(out_rsrc) : "memory");
    else
      asm volatile("buffer_store_byte %0, %1, %2, 0 offen" ::"v"(hv), "v"(a), "s"(out_rsrc) : "memory");
    hc = 0;
  };
#pragma unroll
  for (int s = 0; s < D; ++s) {
    issue(s, Lr + SB * s, false, 0);
    asm volatile("buffer_store_dword %0, %1, %2, 0 offen" ::"v"(0u), "v"(kOOB), "s"(out_rsrc) : "memory");
  }

  auto pending = [&]() -> bool { return k <= m && x < Lr + SB; };
  // one event per row: the row's next frame boundary, if it lies in this line
  auto event = [&](const u32x4& wv, uint32_t y0, uint32_t y1, uint32_t y2, uint32_t y3, uint32_t& ra) {
    {
      const bool ev = pending();
      const uint32_t rl = x - Lr;  // 0..SB-1 where ev
      const uint32_t pe = (rl >> 4) & (RLS - 1u), ke = (rl >> 2) & 3u, c = rl & 3u;
      // the lane's value and F column
      const uint32_t yk = ke == 0 ? y0 : ke == 1 ? y1 : ke == 2 ? y2 : y3;
      const uint32_t wk = ke == 0 ? wv[0] : ke == 1 ? wv[1] : ke == 2 ? wv[2] : wv[3];
      const uint32_t hm = (uint32_t)(0xFFFFFFFFull << (8 * c));
      const uint32_t E = yk ^ (wk & hm);
      const uint32_t v = p == pe ? E : (p < pe ? ra : r);
      const uint32_t n = p == pe ? 0u : 4u * ((p - pe) & (RLS - 1u)) - ke;
      uint32_t O = f_step(lds, v, kFBase | (n << 2));
      O = rowx<RLS>(O);
      // S = Z_c(O) and the injection's Z_{SB-4k}(O): nibble p (and p + 4 on
      // 4-lane rows) of O on lane p
      auto nibs = [&](uint32_t base, uint32_t sel, uint32_t y) -> uint32_t {
        uint32_t t = lds_rd(lds, base + (((sel * 8u + p) * 16u + ((y >> (4 * p)) & 15u)) << 2));
        if constexpr (RLS == 4)
          t ^= lds_rd(lds, base + (((sel * 8u + p + 4u) * 16u + ((y >> (4 * p + 16)) & 15u)) << 2));
        return t;
      };
      uint32_t S = rowx<RLS>(nibs(kSTc, c, O));
      uint32_t G = rowx<RLS>(nibs(kSG, ke, O)) ^ lds_rd(lds, kSK + ((rl & 15u) << 2));
      const bool same = pe == pprev;
      if (wave_any(ev && same)) {  // slow path: an earlier event of this row in the same lane piece
        if (ev && same) {          // (row-uniform: the row's 8 lanes together)
          uint32_t q = P;          // the piece's injections, moved from xprev to x
          for (uint32_t i = 0; i < x - xprev; ++i) q = z1(lds, q);
          S ^= q;
          // G = Z_{SB - (rl & 15)}(~S) = Z_{SB - 4(ke + [c > 0])}(Z_{(4 - c) & 3}(~S))
          uint32_t u = ~S;
          for (uint32_t i = 0; i < ((4u - c) & 3u); ++i) u = z1(lds, u);
          const uint32_t kk = ke + (c != 0u ? 1u : 0u);
          G = rowx<RLS>(nibs(kSG, kk, u));
          P = q;
        }
      }
      if (ev) {
        const uint32_t crc = ~S;
        if (k >= 1) {  // frame fr0 + k - 1 ends at x
          if (p == hc) hv = MODE == CrcMode::kCrc ? crc : ((x - xs >= 4u && crc == 0x2144DF1Cu) ? 1u : 0u), hf = fr0 + k - 1;
          hc += 1;
        }
        if (p == pe) ra ^= G;                 // the next frame starts at x
        P = (same ? P : 0u) ^ crc;            // injections of this piece, at x
        xprev = x, pprev = pe, xs = x;
        k += 1;
      }
      // next event: from A / B (full exec for the bpermute)
      const bool adv = ev && k - kb >= 8u && k <= m;  // A used up
      if (wave_any(adv && !hasB)) {  // slow path: the next block is not here yet: load it now
        // (a request in flight is dropped: its set is not read on this path, so
        // hipcc keeps no copy of an outstanding ring register here)
        uint32_t nb[OPL];
#pragma unroll
        for (int i = 0; i < OPL; ++i) nb[i] = rel(ld_off(kb + 8u + p + RLS * i));
        if (adv && !hasB) {
#pragma unroll
          for (int i = 0; i < OPL; ++i) B[i] = nb[i];
          reqd = false, hasB = true;
        }
      }
      if (adv) {
#pragma unroll
        for (int i = 0; i < OPL; ++i) A[i] = B[i];
        kb += 8u, hasB = false;
      }
      const uint32_t xn = pick(k - kb);
      if (ev) x = xn;
      if (wave_any(hc >= 2u && pending())) store_held();  // a third result in this line: flush (extra VMEM)
    }
  };
  // Frames of >= 64 bytes end at most twice in a 128-byte row step and once
  // in a 64-byte one: those passes are unrolled, so the common path has no
  // loop (whose phi copies cost ~16 VALU an iteration); more (shorter frames) loop.
  auto event_loop = [&](const u32x4& wv, uint32_t y0, uint32_t y1, uint32_t y2, uint32_t y3, uint32_t& ra) {
    pprev = 0xFFu;
    if (wave_any(pending())) {
      event(wv, y0, y1, y2, y3, ra);
      if constexpr (RLS == 8) {
        if (wave_any(pending())) {
          event(wv, y0, y1, y2, y3, ra);
          while (wave_any(pending())) event(wv, y0, y1, y2, y3, ra);
        }
      } else {
        while (wave_any(pending())) event(wv, y0, y1, y2, y3, ra);
      }
    }
  };

  bool live = true;
  while (live) {
#pragma unroll
    for (int s = 0; s < R; ++s) {
      // set s holds line Lr
      // loads younger than set s's: the store of its step, then D - 1 steps of
      // (line, OPL offsets, store)
      asm volatile("s_waitcnt vmcnt(%0)" ::"i"(1 + (2 + OPL) * (D - 1)));
      asm volatile("" : "+v"(w[s]), "+v"(ob[s][0]));
      if constexpr (OPL == 2) asm volatile("" : "+v"(ob[s][1]));
      const u32x4 wv = w[s];
      {
        const bool arr = reqd && reqs == (uint32_t)s;
        uint32_t bo[OPL];
#pragma unroll
        for (int i = 0; i < OPL; ++i) bo[i] = rel(ob[s][i]);
        if (arr) {
#pragma unroll
          for (int i = 0; i < OPL; ++i) B[i] = bo[i];
          hasB = true, reqd = false;
        }
      }
      // next request: B free, a block after it exists
      const bool req = !hasB && !reqd && kb + 8u <= m;
      const uint32_t kreq = kb + 8u;
      const int sn = (s + D) % R;  // the set step t - 1 used
      issue(sn, Lr + SB * D, req, kreq);
      if (req) reqd = true, reqs = (uint32_t)sn;
      // the fold
      uint32_t ra;
      if constexpr (VAR == 152) {  // profiling: loads only
        ra = r ^ wv[0] ^ wv[1] ^ wv[2] ^ wv[3];
      } else {
        uint32_t y0 = r ^ wv[0];
        uint32_t y1 = u_step_xor(lds, y0, wv[1], bu0, bu1);
        uint32_t y2 = u_step_xor(lds, y1, wv[2], bu0, bu1);
        uint32_t y3 = u_step_xor(lds, y2, wv[3], bu0, bu1);
        ra = z116(lds, y3);
        if constexpr (VAR != 151) event_loop(wv, y0, y1, y2, y3, ra);  // 151 (profiling): loads + chain only
      }
      r = ra;
      Lr += SB;
      if (Lr > Lend) k = m + 1u;  // past the row's last line (a bound every wave reaches)
      store_held();
      live = wave_any(k <= m);
      if (!live) break;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (VAR == 151 || VAR == 152) {  // keep the fold live
    if (r == 0x9E3779B9u) store_held();
  }
}

