// stream_lanes.hpp — lane streams for short frames, included
// by crc32_kernel.hip after stream_rows.hpp.  The host-side restatement of
// this schedule, checked against zlib, is tests/stream_algebra.py lane_stream.
//
// The streaming rows (stream_rows.hpp) read the Zipf mix's lines once, but
// each frame boundary combines a row's lanes into the stream's state: a
// wave-wide pass of ~145 VALU with rotated F columns whose LDS reads conflict.
// Here ONE lane folds a contiguous run of frames serially, so its register IS
// the running CRC state and a boundary needs no cross-lane work at all:
//
//   loads: a quad (4 lanes) owns 4 runs; per superstep it reads 64 contiguous
//     bytes of each (4 buffer_load_dwordx4, each a half line), then a 4x4
//     transpose of 16-byte blocks by DPP quad swaps gives every lane its own
//     run's 64 bytes;
//   fold: per 64-byte superstep at P, y0 = r ^ w0, y_i = Z4(y_{i-1}) ^ w_i,
//     r' = Z4(y15) (Z4: the lane-private U image, conflict-free), keeping
//     y_k, w_k of the dword k of the lane's next boundary;
//   boundary x in [P, P + 64) (cb = x - P, k = cb >> 2, c = cb & 3):
//     e = y_k ^ (w_k & ~lomask(c)), the chain's state at x is S = Z_c(e): the
//     frame ending at x has CRC ~S; the frame starting at x resets the state
//     to ~0, i.e. r' ^= Z_{64-cb}(S ^ ~0) = Z_{64-4k}(e) ^ Z_{64-cb}(~0)
//     (Z_c: shared byte tables, Z_{64-4k}: shared nibble tables; only the
//     lanes with a boundary read them).  A frame of >= 64 bytes starts at
//     most once in a superstep, so the wave runs one boundary pass per 4 KiB.
//
// Work: the workgroup's slice is split over its 1024 lanes by BYTES (each
// lane's first frame is the first whose start reaches j/1024 of the slice:
// a binary search over the offsets), so the runs are byte-balanced.  A lane's
// frame boundaries come from 4-offset blocks (two buffer_load_dwordx4 of
// uint64 offsets), the next block requested through the ring.  Every
// superstep issues exactly seven ring VMEM instructions (four data loads, two
// offset loads, the held result's store; out-of-range when idle), so the
// ring's vmcnt is static; a second frame end in one superstep (frames under
// 64 bytes) stores at once, which only makes the wait stricter.  (Storing
// each result at once cost 0.3 ms on the Zipf mix: every store younger than a
// set's loads makes its vmcnt wait retire the NEXT superstep's loads too.)
#pragma once
// (included inside namespace lnx)

// lane-stream image tail: lds_layout.hpp kLZc, kLZd, kLK
static_assert(kLK + 256u <= kCtrBase, "lane-stream tables overlap the counter");

template <int CTRL>
__device__ __forceinline__ uint32_t dpp_mov(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
// one level of the quad transpose: lanes with `hi` swap their a for the
// partner's b (the partner across lane bit CTRL selects)
template <int CTRL>
__device__ __forceinline__ void quad_swap(u32x4& a, u32x4& b, bool hi) {
#pragma unroll
  for (int d = 0; d < 4; ++d) {
    const uint32_t rcv = dpp_mov<CTRL>(hi ? a[d] : b[d]);
    if (hi)
      a[d] = rcv;
    else
      b[d] = rcv;
  }
}

template <CrcMode MODE, int VAR, int D = 2>
__device__ __forceinline__ void lanes_body(const char* lds, const Lanes& L, const WaveCtx& cx) {
  static_assert(MODE != CrcMode::kAppend, "offsets mode only");
  const uint32_t lane = L.lane, qi = lane & 3u;
  const uint32_t bu0 = L.bu0, bu1 = L.bu1;
  const uint32_t nfb = cx.nfb, o0_lo = cx.o0_lo, adj = cx.adj;
  const __amdgpu_buffer_rsrc_t data_rsrc = cx.data_rsrc, off_rsrc = cx.off_rsrc, out_rsrc = cx.out_rsrc;
  auto rel = [&](uint32_t x_lo) -> uint32_t { return x_lo - o0_lo + adj; };
  auto ld_rel = [&](uint32_t f) -> uint32_t {  // rel(off[f]) of the range, f <= nfb; junk otherwise
    return rel(__builtin_amdgcn_raw_buffer_load_b32(off_rsrc, f <= nfb ? f * 8u : kOOB, 0, 0));
  };

  // ---- the lane's run: frames [fa, fa + m), events 0..m at off[fa + k]
  uint32_t fa, fz;
  {
    const uint32_t tot = ld_rel(nfb) - adj;
    const uint32_t j = threadIdx.x;
    const uint32_t t0 = adj + (uint32_t)(((uint64_t)j * tot) >> 10), t1 = adj + (uint32_t)(((uint64_t)(j + 1) * tot) >> 10);
    // first f in [0, nfb] with rel(off[f]) >= t (off[nfb] = the end reaches every t)
    uint32_t lo0 = 0, hi0 = nfb, lo1 = 0, hi1 = nfb;
    while (wave_any(lo0 < hi0 || lo1 < hi1)) {
      const uint32_t m0 = (lo0 + hi0) >> 1, m1 = (lo1 + hi1) >> 1;
      const uint32_t v0 = ld_rel(m0), v1 = ld_rel(m1);
      if (lo0 < hi0) {
        if (v0 >= t0) hi0 = m0; else lo0 = m0 + 1u;
      }
      if (lo1 < hi1) {
        if (v1 >= t1) hi1 = m1; else lo1 = m1 + 1u;
      }
    }
    fa = j == 0 ? 0u : lo0;
    fz = j == kBlockThreads - 1 ? nfb : lo1;
  }
  const uint32_t m = fz - fa;
  uint32_t A[4], B[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) A[i] = ld_rel(fa + i <= fz ? fa + i : kOOB), B[i] = ld_rel(fa + 4 + i <= fz ? fa + 4 + i : kOOB);
  const uint32_t xlast = ld_rel(fz);
  uint32_t k = m == 0 ? 1u : 0u;  // next event (an empty run has none)
  uint32_t kb = 0;                // event index of A[0]
  bool hasB = m >= 4, reqd = false;
  uint32_t reqs = 0;
  uint32_t x = k <= m ? A[0] : 0xFFFFFFFFu;  // next event's position
  uint32_t xs = x;                           // the previous event (verify: frame length)
  uint32_t P = k <= m ? x & ~63u : kOOB;     // the lane's superstep (64 bytes)
  const uint32_t Pend = k <= m ? xlast & ~63u : 0u;
  uint32_t r = 0;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");

  // ---- ring: D supersteps of (4 data loads, 2 offset loads) in flight.  Set s
  // is read (and transposed) first, then refilled for the superstep D ahead.
  u32x4 w[D][4];
  u32x4 ob[D][2];
  constexpr bool HALF = VAR == 165 && D == 2;  // offset requests on even sets only (4 fewer VMEM per 2 supersteps)
  auto issue = [&](int s, uint32_t Pn, bool req, uint32_t kreq) {
    const uint32_t vp = Pn <= Pend ? Pn : kOOB;  // this lane's run, D supersteps ahead
    const uint32_t a0 = dpp_mov<0x00>(vp) + 16u * qi, a1 = dpp_mov<0x55>(vp) + 16u * qi,
                   a2 = dpp_mov<0xAA>(vp) + 16u * qi, a3 = dpp_mov<0xFF>(vp) + 16u * qi;
    const uint32_t f0 = fa + kreq, f2 = fa + kreq + 2u;
    const uint32_t vo0 = req && f0 <= nfb ? f0 * 8u : kOOB, vo1 = req && f2 <= nfb ? f2 * 8u : kOOB;
    if (HALF && (s & 1)) {  // VAR 165: offsets only on even sets
      asm volatile(
          "s_nop 4\n\t"
          "buffer_load_dwordx4 %0, %4, %8, 0 offen" LNX_LD_POL "\n\t"
          "buffer_load_dwordx4 %1, %5, %8, 0 offen" LNX_LD_POL "\n\t"
          "buffer_load_dwordx4 %2, %6, %8, 0 offen" LNX_LD_POL "\n\t"
          "buffer_load_dwordx4 %3, %7, %8, 0 offen" LNX_LD_POL
          : "=&v"(w[s][0]), "=&v"(w[s][1]), "=&v"(w[s][2]), "=&v"(w[s][3])
          : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "s"(data_rsrc));
      return;
    }
    asm volatile(
        "s_nop 4\n\t"
        "buffer_load_dwordx4 %0, %6, %12, 0 offen" LNX_LD_POL "\n\t"
        "buffer_load_dwordx4 %1, %7, %12, 0 offen" LNX_LD_POL "\n\t"
        "buffer_load_dwordx4 %2, %8, %12, 0 offen" LNX_LD_POL "\n\t"
        "buffer_load_dwordx4 %3, %9, %12, 0 offen" LNX_LD_POL "\n\t"
        "buffer_load_dwordx4 %4, %10, %13, 0 offen\n\t"
        "buffer_load_dwordx4 %5, %11, %13, 0 offen"
        : "=&v"(w[s][0]), "=&v"(w[s][1]), "=&v"(w[s][2]), "=&v"(w[s][3]), "=&v"(ob[s][0]), "=&v"(ob[s][1])
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(vo0), "v"(vo1), "s"(data_rsrc), "s"(off_rsrc));
  };
  // the held result (one store per superstep: a frame of >= 64 bytes ends at
  // most once in 64 bytes)
  uint32_t hv = 0, hf = 0;
  bool hold = false;
  auto store_held = [&]() {
    const uint32_t a = hold ? (MODE == CrcMode::kCrc ? hf * 4u : hf) : kOOB;
    if constexpr (MODE == CrcMode::kCrc)
      asm volatile("buffer_store_dword %0, %1, %2, 0 offen" ::"v"(hv), "v"(a), "s"(out_rsrc) : "memory");
    else
      asm volatile("buffer_store_byte %0, %1, %2, 0 offen" ::"v"(hv), "v"(a), "s"(out_rsrc) : "memory");
    hold = false;
  };
#pragma unroll
  for (int s = 0; s < D; ++s) {
    issue(s, P + 64u * s, false, 0);
    asm volatile("buffer_store_dword %0, %1, %2, 0 offen" ::"v"(0u), "v"(kOOB), "s"(out_rsrc) : "memory");
  }

  // Z_1 byte step through the Z_1 byte table (slow path)
  auto z1 = [&](uint32_t v) -> uint32_t { return lds_rd(lds, kLZc + ((v & 0xFFu) << 2)) ^ (v >> 8); };
  // slow path (a later boundary of this lane in the same superstep, frames
  // under 64 bytes): e at dword kev, the chain rerun from r0 with every step
  // predicated
  auto e_at = [&](uint32_t r0, const u32x4* Xs, uint32_t kev, uint32_t hm) -> uint32_t {
    uint32_t st = r0, e = 0;
#pragma unroll
    for (uint32_t d = 0; d < 16u; ++d) {
      const uint32_t wd = Xs[d >> 2][d & 3u];
      const uint32_t y = st ^ wd;
      if (d == kev) e = y ^ (wd & hm);
      st = u_step(lds, y, bu0, bu1);
    }
    return e;
  };
  // ---- VAR 164: the reset as a select inside the fold.  A
  // frame starting at byte c of dword k makes the chain value there
  // y = (~w_k & hm) ^ K_c (hm = ~0 << 8c, K_c = Z_{-c}(the top c bytes of ~0)),
  // so Z4(y) is the new frame's state after the dword; only the ending
  // frame's Z_c(e) is a lookup, off the fold's critical path.
  constexpr auto unz = [](uint32_t v, int n) constexpr {
    for (int i = 0; i < n; ++i) {
      const uint32_t b = v >> 31, t = b ? v ^ 0xEDB88320u : v;
      v = (t << 1) | b;
    }
    return v;
  };
  constexpr uint32_t kK1 = unz(0xFF000000u, 8), kK2 = unz(0xFFFF0000u, 16), kK3 = unz(0xFFFFFF00u, 24);
  auto zc_of = [&](uint32_t e, uint32_t c) -> uint32_t {  // Z_c(e), c = 1..3
    const uint32_t bc = kLZc + 4096u * ((c - 1u) & 3u);
    return __builtin_amdgcn_bitop3_b32(lds_rd(lds, bc + ((e & 0xFFu) << 2)),
                                       lds_rd(lds, bc + 1024u + (__builtin_amdgcn_ubfe(e, 8, 8) << 2)),
                                       lds_rd(lds, bc + 2048u + (__builtin_amdgcn_ubfe(e, 16, 8) << 2)), 0x96) ^
           lds_rd(lds, bc + 3072u + ((e >> 24) << 2));
  };
  auto corr_of = [&](uint32_t e, uint32_t rp) -> uint32_t {  // Z_{64-4k}(e) ^ Z_{64-rp}(~0)
    const uint32_t bd = kLZd + 512u * ((rp >> 2) & 15u);
    uint32_t v[8];
#pragma unroll
    for (uint32_t i = 0; i < 8u; ++i) v[i] = lds_rd(lds, bd + 64u * i + (__builtin_amdgcn_ubfe(e, 4 * i, 4) << 2));
    const uint32_t t0 = __builtin_amdgcn_bitop3_b32(v[0], v[1], v[2], 0x96);
    const uint32_t t1 = __builtin_amdgcn_bitop3_b32(v[3], v[4], v[5], 0x96);
    const uint32_t t2 = __builtin_amdgcn_bitop3_b32(v[6], v[7], lds_rd(lds, kLK + (rp << 2)), 0x96);
    return __builtin_amdgcn_bitop3_b32(t0, t1, t2, 0x96);
  };
  // an event's bookkeeping (the lanes with ev): the ended frame's result, the
  // next boundary
  auto advance = [&](bool ev, uint32_t St) {
    if (wave_any(ev && k >= 1u && hold)) {  // a second end in this superstep: an extra store
      if (ev && k >= 1u && hold) store_held();
    }
    const bool end = ev && k >= 1u;
    const uint32_t crc = ~St;
    hv = end ? (MODE == CrcMode::kCrc ? crc : (x - xs >= 4u && crc == 0x2144DF1Cu ? 1u : 0u)) : hv;
    hf = end ? fa + k - 1u : hf;
    hold = hold || end;
    xs = ev ? x : xs;
    k = ev ? k + 1u : k;
    const bool adv = ev && k <= m && k - kb >= 4u;
    if (wave_any(adv && !hasB)) {  // slow path: the next block is not here yet: load it now
      uint32_t nb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) nb[i] = ld_rel(fa + kb + 4u + i <= fz ? fa + kb + 4u + i : kOOB);
      if (adv && !hasB) {
#pragma unroll
        for (int i = 0; i < 4; ++i) B[i] = nb[i];
        hasB = true, reqd = false;
      }
    }
    if (adv) {
#pragma unroll
      for (int i = 0; i < 4; ++i) A[i] = B[i];
      kb += 4u, hasB = false;
    }
    if (ev) {  // (selects by ia written as a ternary chain under a branch: hipcc keeps A in registers)
      const uint32_t ia = k - kb;
      x = k > m ? 0xFFFFFFFFu : ia == 0 ? A[0] : ia == 1 ? A[1] : ia == 2 ? A[2] : A[3];
    }
  };

  // one boundary of the superstep (the lanes where it lies in [P, P + 64)):
  // ye / we are the chain value and word of the first boundary's dword
  auto pass = [&](bool later, uint32_t ye, uint32_t we, uint32_t r0, const u32x4* Xs, uint32_t& fix, uint32_t& Sp,
                  uint32_t& xp) {
    const uint32_t rp = x - P;
    const bool ev = rp < 64u;
    const uint32_t kev = (rp >> 2) & 15u, c = rp & 3u;
    const uint32_t hm = 0xFFFFFFFFu << (8u * c);
    uint32_t e = ye ^ (we & hm);
    if (later) {
      if (ev) e = e_at(r0, Xs, kev, hm);
    }
    uint32_t S = e, corr = 0;
    if (ev) {
      // Z_c (c = 1..3): byte tables; Z_{64-4k}: nibble tables; then the constant
      const uint32_t bc = kLZc + 4096u * ((c - 1u) & 3u), bd = kLZd + 512u * kev;
      const uint32_t Sc = __builtin_amdgcn_bitop3_b32(lds_rd(lds, bc + ((e & 0xFFu) << 2)),
                                                      lds_rd(lds, bc + 1024u + (__builtin_amdgcn_ubfe(e, 8, 8) << 2)),
                                                      lds_rd(lds, bc + 2048u + (__builtin_amdgcn_ubfe(e, 16, 8) << 2)), 0x96) ^
                          lds_rd(lds, bc + 3072u + ((e >> 24) << 2));
      uint32_t v[8];
#pragma unroll
      for (uint32_t i = 0; i < 8u; ++i) v[i] = lds_rd(lds, bd + 64u * i + (__builtin_amdgcn_ubfe(e, 4 * i, 4) << 2));
      const uint32_t t0 = __builtin_amdgcn_bitop3_b32(v[0], v[1], v[2], 0x96);
      const uint32_t t1 = __builtin_amdgcn_bitop3_b32(v[3], v[4], v[5], 0x96);
      const uint32_t t2 = __builtin_amdgcn_bitop3_b32(v[6], v[7], lds_rd(lds, kLK + (rp << 2)), 0x96);
      corr = __builtin_amdgcn_bitop3_b32(t0, t1, t2, 0x96);
      S = c != 0u ? Sc : e;
    }
    uint32_t St = S;
    if (later) {  // the frame started at the previous boundary xp: its state from ~0
      if (ev) {
        uint32_t z = ~Sp;
        for (uint32_t i = 0; i < x - xp; ++i) z = z1(z);
        St ^= z;
      }
    }
    if (ev) {
      if (k >= 1u) {  // frame fa + k - 1 ends at x: held to the superstep's store
        if (hold) store_held();  // a second end in this superstep (frames < 64 B): an extra store
        const uint32_t crc = ~St;
        hv = MODE == CrcMode::kCrc ? crc : (x - xs >= 4u && crc == 0x2144DF1Cu ? 1u : 0u);
        hf = fa + k - 1u, hold = true;
      }
      if (k < m) fix = corr;  // the frame fa + k starts at x (the last start of the superstep wins)
      Sp = S, xp = x, xs = x;
      k += 1u;
    }
    // the next boundary: A[k - kb], or the next block
    const bool adv = ev && k <= m && k - kb >= 4u;
    if (wave_any(adv && !hasB)) {  // slow path: the next block is not here yet: load it now
      uint32_t nb[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) nb[i] = ld_rel(fa + kb + 4u + i <= fz ? fa + kb + 4u + i : kOOB);
      if (adv && !hasB) {
#pragma unroll
        for (int i = 0; i < 4; ++i) B[i] = nb[i];
        hasB = true, reqd = false;
      }
    }
    if (adv) {
#pragma unroll
      for (int i = 0; i < 4; ++i) A[i] = B[i];
      kb += 4u, hasB = false;
    }
    if (ev) {
      const uint32_t ia = k - kb;
      x = k > m ? 0xFFFFFFFFu : ia == 0 ? A[0] : ia == 1 ? A[1] : ia == 2 ? A[2] : A[3];
    }
  };

  bool live = wave_any(k <= m);
  while (live) {
#pragma unroll
    for (int s = 0; s < D; ++s) {
      // set s holds superstep P; younger: the store of its superstep, then D - 1
      // supersteps of (six loads, one store)
      if (HALF && s == 0)
        asm volatile("s_waitcnt vmcnt(6)");  // younger: its store, the odd set's 4 loads and store
      else
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(1 + 7 * (D - 1)));
      if (HALF && (s & 1))
        asm volatile("" : "+v"(w[s][0]), "+v"(w[s][1]), "+v"(w[s][2]), "+v"(w[s][3]));
      else
        asm volatile("" : "+v"(w[s][0]), "+v"(w[s][1]), "+v"(w[s][2]), "+v"(w[s][3]), "+v"(ob[s][0]), "+v"(ob[s][1]));
      u32x4 Xs[4] = {w[s][0], w[s][1], w[s][2], w[s][3]};
      {
        const bool b0 = (qi & 1u) != 0u, b1 = (qi & 2u) != 0u;
        quad_swap<0xB1>(Xs[0], Xs[1], b0);
        quad_swap<0xB1>(Xs[2], Xs[3], b0);
        quad_swap<0x4E>(Xs[0], Xs[2], b1);
        quad_swap<0x4E>(Xs[1], Xs[3], b1);
      }
      if (!(HALF && (s & 1)) && reqd && reqs == (uint32_t)s) {  // the requested block arrived
        B[0] = rel(ob[s][0][0]), B[1] = rel(ob[s][0][2]), B[2] = rel(ob[s][1][0]), B[3] = rel(ob[s][1][2]);
        hasB = true, reqd = false;
      }
      const bool req = !hasB && !reqd && kb + 4u <= m && !(HALF && (s & 1));
      issue(s, P + 64u * D, req, kb + 4u);
      if (req) reqd = true, reqs = (uint32_t)s;
      if constexpr (VAR == 161) {  // profiling: loads only
#pragma unroll
        for (int i = 0; i < 4; ++i) r ^= Xs[i][0] ^ Xs[i][1] ^ Xs[i][2] ^ Xs[i][3];
      } else if constexpr (VAR == 164 || VAR == 165) {
        const uint32_t r0 = r, rp1 = x - P, kev = rp1 >> 2, c1 = rp1 & 3u;  // kev >= 16: no boundary here
        const uint32_t hm1 = 0xFFFFFFFFu << (8u * c1);
        const uint32_t Kc = c1 == 1u ? kK1 : c1 == 2u ? kK2 : c1 == 3u ? kK3 : 0u;
        const bool rst = k < m;  // the boundary starts frame fa + k
        uint32_t y = 0, ec = 0;
#pragma unroll
        for (uint32_t d = 0; d < 16u; ++d) {
          const uint32_t wd = Xs[d >> 2][d & 3u];
          const uint32_t yn = d == 0 ? r0 ^ wd : u_step_xor(lds, y, wd, bu0, bu1);
          const bool at = kev == d;
          ec = at ? __builtin_amdgcn_bitop3_b32(yn, wd, hm1, 0x78) : ec;  // yn ^ (wd & hm1)
          y = at && rst ? __builtin_amdgcn_bitop3_b32(wd, hm1, Kc, 0xA6) : yn;  // (~wd & hm1) ^ Kc
        }
        r = u_step(lds, y, bu0, bu1);
        if (wave_any(rp1 < 64u)) {
          const bool ev = rp1 < 64u;
          uint32_t S = ec;
          if (ev && c1 != 0u) S = zc_of(ec, c1);
          const bool st1 = ev && rst;
          advance(ev, S);
          if (wave_any(x - P < 64u)) {  // more boundaries in this superstep (frames < 64 B)
            uint32_t cin = 0, Sp = S, xp = rp1;  // cin: the correction the fold applied (relative to P)
            if (st1) cin = corr_of(ec, rp1);
            while (wave_any(x - P < 64u)) {
              const uint32_t rp = x - P;
              const bool evj = rp < 64u;
              if (evj) {
                const uint32_t c = rp & 3u, hm = 0xFFFFFFFFu << (8u * c);
                const uint32_t e = e_at(r0, Xs, rp >> 2, hm);
                const uint32_t Sj = c != 0u ? zc_of(e, c) : e;
                uint32_t z = ~Sp;
                for (uint32_t i = 0; i < rp - xp; ++i) z = z1(z);
                const uint32_t St = Sj ^ z;
                if (k < m) {
                  const uint32_t cj = corr_of(e, rp);
                  r ^= cin ^ cj;
                  cin = cj;
                }
                Sp = Sj, xp = rp;
                S = St;
              }
              advance(evj, S);
            }
          }
        }
      } else {
        // the fold of the 16 dwords, keeping the first boundary's dword
        const uint32_t r0 = r, kev = (x - P) >> 2;  // >= 16: no boundary here
        uint32_t y = 0, ye = 0, we = 0;
#pragma unroll
        for (uint32_t d = 0; d < 16u; ++d) {
          const uint32_t wd = Xs[d >> 2][d & 3u];
          y = d == 0 ? r0 ^ wd : u_step_xor(lds, y, wd, bu0, bu1);
          ye = kev == d ? y : ye;
          we = kev == d ? wd : we;
        }
        const uint32_t rn = u_step(lds, y, bu0, bu1);
        uint32_t fix = 0, Sp = 0, xp = 0;
        if constexpr (VAR != 162) {  // 162 (profiling): loads + chain only
          if (wave_any(x - P < 64u)) {
            pass(false, ye, we, r0, Xs, fix, Sp, xp);
            while (wave_any(x - P < 64u)) pass(true, ye, we, r0, Xs, fix, Sp, xp);
          }
        }
        r = rn ^ fix;
      }
      store_held();
      P += 64u;
      if (P > Pend) k = m + 1u;  // past the run's last superstep (a bound every wave reaches)
      live = wave_any(k <= m);
      if (!live) break;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if constexpr (VAR == 161 || VAR == 162) {  // keep the fold live
    if (r == 0x9E3779B9u) __builtin_amdgcn_raw_buffer_store_b32(r, out_rsrc, 0, 0, 0);
  }
}
