// crc32_kernel.hip — batched CRC-32/IEEE (Ethernet FCS) over packed frames, gfx950.
//
// Reference semantics: ethernet.CRC32 (lneto ethernet/crc.go:19-21) =
// Go crc32.Checksum(data, IEEETable): init 0xFFFFFFFF, reflected, xorout
// 0xFFFFFFFF.  The FCS-verify mode implements the residue form of the check a
// receiver does before StackEthernet.Demux (internet/stack-ethernet.go:139).
//
// Work decomposition
// ---------------------------------
// A wave is four 16-lane rows; each row folds one frame.  A frame is viewed
// through a window that ENDS at its last byte and is a whole number J of
// 64-byte row steps long; the lead-in (< 64 bytes) before the frame start is
// zero-masked.  With init 0 the CRC register ignores leading zeros, so the
// window's register equals the frame's; the init value is folded in by XOR-ing
// 0xFF into the frame's first four bytes.
//
// Lane p of a row consumes the word at window offset 4p + 64j: one coalesced
// 256-byte dword load per wave per step covers four frames.  Each lane keeps
// its own register r and advances it with r = U(r ^ w), U = Z_64, through four
// lane-private byte tables in LDS (lds_layout.hpp) — conflict-free whatever the
// data.  After the last step lane p's register sits 4p bytes past the frame
// end; F_p = Z_{-4p} (lane-private nibble tables) moves it back and the frame
// register is the XOR over the row (four DPP steps; every lane of the row ends
// up holding it).  No MFMA: this is a per-byte GF(2) polynomial.
//
// Everything per frame (bounds, window position, masks) is a row-uniform VGPR
// value, so one instruction serves four frames; the per-frame overhead is
// amortised 4x compared with a wave per frame (DESIGN.md §4 has the numbers).
//
// Pipeline: each row's frames are cut into items of <= KS steps.  A ring of S
// slots (one item per row per slot) keeps the next S-1 slots' loads in flight
// while one slot is folded.  Streaming loads are inline-asm raw buffer loads
// over the wave's own byte range (out-of-range lanes read 0, so lead-ins, idle
// steps and dummy slots need no address clamping) with hand-counted vmcnt:
// every slot issues exactly KS+2 loads, so the count is static.  Frame bounds
// come from a per-slot prefetch of the next 4S+1 offsets (lane i holds the low
// dword of off[nf+i]), shuffled to the rows with ds_bpermute at assignment.
// Frames whose end is not 4-byte aligned load the aligned dword A_{p+1} per
// lane and rebuild their window word with v_alignbyte from A_p (lane p-1, or
// for p = 0 the previous step's lane 15) via two DPP moves.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <utility>
#include "lds_layout.hpp"

namespace lnx {

constexpr int kBlockThreads = 1024;
constexpr int kWavesPerBlock = kBlockThreads / 64;
constexpr int kRows = 4;
constexpr uint32_t kNoFrame = 0xFFFFFFFFu;
constexpr uint32_t kOOB = 0xFFFFFF00u;  // buffer offset that is always out of range

// ------------------------------------------------------------------ helpers
__device__ __forceinline__ uint32_t lds_rd(const char* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(lds + byte_addr);
}

// r' = U(x): four lane-private byte lookups; byte k of x -> address byte 1.
__device__ __forceinline__ uint32_t u_step(const char* lds, uint32_t x, uint32_t b0, uint32_t b1) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, b0, 0x0c020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, b0, 0x0c020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, b1, 0x0c020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, b1, 0x0c020700u);
  return lds_rd(lds, a0) ^ lds_rd(lds, a1 + 128) ^ lds_rd(lds, a2) ^ lds_rd(lds, a3 + 128);
}

// U(x) ^ y with the four-way XOR in two v_bitop3 (gfx950 3-input logic op).
__device__ __forceinline__ uint32_t u_step_xor(const char* lds, uint32_t x, uint32_t y, uint32_t b0, uint32_t b1) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, b0, 0x0c020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, b0, 0x0c020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, b1, 0x0c020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, b1, 0x0c020700u);
  const uint32_t t = __builtin_amdgcn_bitop3_b32(lds_rd(lds, a0), lds_rd(lds, a1 + 128), lds_rd(lds, a2), 0x96);
  return __builtin_amdgcn_bitop3_b32(t, lds_rd(lds, a3 + 128), y, 0x96);
}

// F_p(r) through eight lane-private nibble tables.
__device__ __forceinline__ uint32_t f_step(const char* lds, uint32_t r, uint32_t bf) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t a = (((r >> (4 * i)) & 15u) << 7) | bf;
    acc ^= lds_rd(lds, a + (uint32_t)(i << 11));
  }
  return acc;
}

// XOR over the 16 lanes of each row; every lane gets its row's result.
__device__ __forceinline__ uint32_t row_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return v;
}

// Bytes [lo, 4) of a little-endian word kept (lo clamped to 0..4).
__device__ __forceinline__ uint32_t keep_from(int32_t lo) {
  lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
  return (uint32_t)(0xFFFFFFFFull << (8 * lo));
}

__device__ __forceinline__ bool wave_any(bool b) { return __builtin_amdgcn_ballot_w64(b) != 0; }

// Streaming raw-buffer dword loads; their completion is the caller's business
// (hipcc does not count asm loads, cdna_hip_programming.md §5.7 item 1): every
// destination passes "+v" through the slot's vmcnt wait before its first use.
// Each statement opens with s_nop 4: hipcc may restore the descriptor SGPRs
// from a spill with v_readlane right before the statement, and a VALU SGPR
// write needs 5 wait states before a VMEM instruction reads it as a
// descriptor; hipcc pads that only for instructions it can see.
template <int IMM>
__device__ __forceinline__ uint32_t ld_buf(uint32_t voff, __amdgpu_buffer_rsrc_t rsrc) {
  uint32_t r;
  asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2, 0 offen offset:%3"
               : "=v"(r) : "v"(voff), "s"(rsrc), "i"(IMM));
  return r;
}
// w[0] <- [v0], w[1] <- [v1]
__device__ __forceinline__ void ld_buf2(uint32_t& a, uint32_t& b, uint32_t v0, uint32_t v1,
                                        __amdgpu_buffer_rsrc_t rsrc) {
  asm volatile("s_nop 4\n\tbuffer_load_dword %0, %2, %4, 0 offen\n\tbuffer_load_dword %1, %3, %4, 0 offen"
               : "=v"(a), "=v"(b) : "v"(v0), "v"(v1), "s"(rsrc));
}
// N loads from one VGPR offset at immediates IMM0, IMM0+64, ...
template <int IMM0, int N>
__device__ __forceinline__ void ld_run(uint32_t* o, uint32_t v, __amdgpu_buffer_rsrc_t rsrc) {
  constexpr int D = (int)kStepBytes;
  if constexpr (N == 6) {
    asm volatile("s_nop 4\n\t"
                 "buffer_load_dword %0, %6, %7, 0 offen offset:%8\n\t"
                 "buffer_load_dword %1, %6, %7, 0 offen offset:%9\n\t"
                 "buffer_load_dword %2, %6, %7, 0 offen offset:%10\n\t"
                 "buffer_load_dword %3, %6, %7, 0 offen offset:%11\n\t"
                 "buffer_load_dword %4, %6, %7, 0 offen offset:%12\n\t"
                 "buffer_load_dword %5, %6, %7, 0 offen offset:%13"
                 : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4]), "=v"(o[5])
                 : "v"(v), "s"(rsrc), "i"(IMM0), "i"(IMM0 + D), "i"(IMM0 + 2 * D), "i"(IMM0 + 3 * D),
                   "i"(IMM0 + 4 * D), "i"(IMM0 + 5 * D));
  } else if constexpr (N == 5) {
    asm volatile("s_nop 4\n\t"
                 "buffer_load_dword %0, %5, %6, 0 offen offset:%7\n\t"
                 "buffer_load_dword %1, %5, %6, 0 offen offset:%8\n\t"
                 "buffer_load_dword %2, %5, %6, 0 offen offset:%9\n\t"
                 "buffer_load_dword %3, %5, %6, 0 offen offset:%10\n\t"
                 "buffer_load_dword %4, %5, %6, 0 offen offset:%11"
                 : "=v"(o[0]), "=v"(o[1]), "=v"(o[2]), "=v"(o[3]), "=v"(o[4])
                 : "v"(v), "s"(rsrc), "i"(IMM0), "i"(IMM0 + D), "i"(IMM0 + 2 * D), "i"(IMM0 + 3 * D),
                   "i"(IMM0 + 4 * D));
  } else {
    static_assert(N == 5 || N == 6, "run length");
  }
}

// vmcnt wait naming every register of one slot.
template <int N, int W>
__device__ __forceinline__ void slot_wait(uint32_t (&w)[W], uint32_t& bnd) {
  if constexpr (W == 25) {
    asm volatile("s_waitcnt vmcnt(%25)"
                 : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]),
                   "+v"(w[7]), "+v"(w[8]), "+v"(w[9]), "+v"(w[10]), "+v"(w[11]), "+v"(w[12]), "+v"(w[13]),
                   "+v"(w[14]), "+v"(w[15]), "+v"(w[16]), "+v"(w[17]), "+v"(w[18]), "+v"(w[19]),
                   "+v"(w[20]), "+v"(w[21]), "+v"(w[22]), "+v"(w[23]), "+v"(w[24])
                 : "i"(N));
    asm volatile("" : "+v"(bnd));
  } else if constexpr (W == 13) {
    asm volatile("s_waitcnt vmcnt(%13)"
                 : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6]),
                   "+v"(w[7]), "+v"(w[8]), "+v"(w[9]), "+v"(w[10]), "+v"(w[11]), "+v"(w[12])
                 : "i"(N));
    asm volatile("" : "+v"(bnd));
  } else if constexpr (W == 7) {
    asm volatile("s_waitcnt vmcnt(%7)"
                 : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]), "+v"(w[6])
                 : "i"(N));
    asm volatile("" : "+v"(bnd));
  } else {
    static_assert(W == 25 || W == 13 || W == 7, "unsupported item size");
  }
}

enum class CrcMode : int { kCrc = 0, kVerify = 1 };

// ------------------------------------------------------------------ generic path
// For a wave whose byte range does not fit a 31-bit buffer offset (frames of
// gigabytes): same algorithm, byte loads with explicit bounds, no pipelining.
template <CrcMode MODE>
__device__ void rows_generic(const char* lds, const uint8_t* bytes, const uint64_t* off, uint64_t fw0,
                             uint64_t fw1, void* out, uint32_t p, uint32_t row, uint32_t bu0, uint32_t bu1,
                             uint32_t bf) {
  const uint64_t fend = fw0 + ((fw1 - fw0 + kRows - 1) / kRows) * kRows;
  for (uint64_t f = fw0 + row; f < fend; f += kRows) {
    const bool live = f < fw1;
    const uint64_t s = live ? off[f] : 0, e = live ? off[f + 1] : 0;
    const uint64_t n = e > s ? e - s : 0;
    const uint64_t J = (n + kStepBytes - 1) / kStepBytes;
    uint32_t reg = 0;
    for (uint64_t j = 0; j < J; ++j) {
      const int64_t pos = (int64_t)e - (int64_t)((J - j) * kStepBytes) + 4 * (int64_t)p;
      uint32_t x = 0;
      for (int b = 0; b < 4; ++b) {
        const int64_t q = pos + b;
        uint32_t v = 0;
        if (q >= (int64_t)s && q < (int64_t)e) {
          v = bytes[q];
          if (q < (int64_t)s + 4) v ^= 0xFFu;  // CRC init folded into the first 4 bytes
        }
        x |= v << (8 * b);
      }
      reg = u_step(lds, reg ^ x, bu0, bu1);
    }
    uint32_t R = n ? row_xor(f_step(lds, reg, bf)) : 0u;
    if (n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * n));
    const uint32_t crc = ~R;
    if (live && p == 0) {
      if (MODE == CrcMode::kCrc)
        reinterpret_cast<uint32_t*>(out)[f] = crc;
      else
        reinterpret_cast<uint8_t*>(out)[f] = (n >= 4 && crc == 0x2144DF1Cu) ? 1 : 0;
    }
  }
}

// ------------------------------------------------------------------ kernel
// Wave-uniform context shared by the item-size specialisations.
struct WaveCtx {
  const char* lds;
  uint32_t lane, p, row, bu0, bu1, bf;
  uint32_t nwf, o0_lo, adj;
  __amdgpu_buffer_rsrc_t data_rsrc, off_rsrc, out_rsrc;
};

// KS: window steps per item, S: ring slots, VAR: profiling knob (DESIGN.md
// §4: 0 = product, 1 = loads + bookkeeping only, 2 = lookups + bookkeeping on
// synthetic words).  Only VAR 0 is reachable from the C-ABI.
template <CrcMode MODE, int KS, int S, int VAR>
__device__ __forceinline__ void rows_body(const WaveCtx& cx) {
  static_assert(S >= 2 && 4 * S + 1 <= 64, "ring size");
  static_assert(KS * (int)kStepBytes <= 4095, "buffer immediate offset");
  constexpr int kW = KS + 1;                    // w[0] = the step before the item
  constexpr int kPending = (S - 1) * (VAR == 2 ? 1 : KS + 2);  // loads issued after a slot's own
  const char* lds = cx.lds;
  const uint32_t lane = cx.lane, p = cx.p, row = cx.row, bu0 = cx.bu0, bu1 = cx.bu1, bf = cx.bf;
  const uint32_t nwf = cx.nwf, o0_lo = cx.o0_lo, adj = cx.adj;
  const __amdgpu_buffer_rsrc_t data_rsrc = cx.data_rsrc, off_rsrc = cx.off_rsrc, out_rsrc = cx.out_rsrc;

  // ---- per-row cursor (row-uniform VGPRs)
  uint32_t rf = kNoFrame;   // frame index relative to fw0
  uint32_t re = 0;          // rel(end offset)
  uint32_t rn = 0;          // length
  uint32_t rJ = 0, rj = 0;  // steps of the frame, next step to issue
  uint32_t nf = 0;          // next unassigned frame of the wave (uniform)

  // ---- ring slots
  uint32_t w[S][kW];
  uint32_t bnd[S];  // lane i: low dword of off[fw0 + nfb[s] + i]
  uint32_t nfb[S];  // uniform
  uint32_t it_f[S], it_e[S], it_n[S], it_j0[S], it_ns[S];
  bool hw[S];       // uniform: slot holds work
  bool un[S];       // uniform: slot was loaded in the misaligned layout
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int k = 0; k < kW; ++k) w[s][k] = 0;
    it_f[s] = kNoFrame;
    it_e[s] = it_n[s] = it_j0[s] = it_ns[s] = 0;
    hw[s] = false;
    un[s] = false;
    nfb[s] = 0;
  }
  // first bounds window for every slot (drained before the loop)
  {
    uint32_t b = ld_buf<0>(lane * 8u, off_rsrc);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(b));
#pragma unroll
    for (int s = 0; s < S; ++s) bnd[s] = b;
  }

  uint32_t reg = 0;  // this lane's CRC register for its row's frame in progress
  int live = 0;      // slots holding work

  auto issue = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    // 1. rows that finished their frame take the next frames of the wave, in order
    const bool need = rj >= rJ;
    const uint64_t nmask = __builtin_amdgcn_ballot_w64(need && p == 0);
    const uint64_t below = (1ull << (16 * row)) - 1;
    const uint32_t rank = (uint32_t)__builtin_popcountll(nmask & below);
    const uint32_t cnt = (uint32_t)__builtin_popcountll(nmask);
    const uint32_t idx = nf + rank;
    const uint32_t li = idx - nfb[s];  // <= 4S by construction
    const uint32_t s_lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(li * 4u), (int)bnd[s]);
    const uint32_t e_lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((li + 1) * 4u), (int)bnd[s]);
    if (need) {
      if (idx < nwf) {
        const uint32_t len = e_lo - s_lo;
        rf = idx;
        re = e_lo - o0_lo + adj;
        rn = (int32_t)len > 0 ? len : 0u;  // end below start: empty frame
        rJ = (rn + kStepBytes - 1) / kStepBytes;
        rj = 0;
      } else {
        rf = kNoFrame;
        rJ = rj = 0;
      }
    }
    nf = nf + cnt < nwf ? nf + cnt : nwf;
    // 2. the item of this slot
    const bool alive = rf != kNoFrame;
    const uint32_t left = rJ - rj;
    const uint32_t ns = alive ? (left < (uint32_t)KS ? left : (uint32_t)KS) : 0u;
    it_f[s] = rf;
    it_e[s] = re;
    it_n[s] = rn;
    it_j0[s] = rj;
    it_ns[s] = ns;
    hw[s] = wave_any(alive);
    // 3. streaming loads: w[0] = step j0-1, w[k+1] = step j0+k (all KS+1 of them, always)
    // In a slot with any misaligned frame every lane loads A_{p+1} (the aligned
    // dword 4 - ra bytes on) and compute() rebuilds words with v_alignbyte;
    // otherwise every lane loads its window word directly.
    const uint32_t ra = re & 3u;
    const bool unal = wave_any(alive && ra != 0);
    un[s] = unal;
    const uint32_t voff =
        alive ? re - rJ * kStepBytes + rj * kStepBytes + (p << 2) - kStepBytes + (unal ? 4u - ra : 0u) : kOOB;
    rj += ns;
    // The buffer range check looks at the VGPR offset on its own (not offset +
    // immediate), so every load's VGPR offset must be non-negative where its
    // bytes are needed: w[0] and w[1] (which may start before the wave's first
    // byte) get clamped offsets, w[2..] share one offset two steps further on.
    const uint32_t v0 = (int32_t)voff < 0 ? kOOB : voff;
    const uint32_t v1 = (int32_t)(voff + kStepBytes) < 0 ? kOOB : voff + kStepBytes;
    const uint32_t v2 = alive ? voff + 2 * kStepBytes : kOOB;
    if constexpr (VAR == 2) {
#pragma unroll
      for (int k = 0; k < kW; ++k) w[s][k] = voff * 0x9E3779B1u + k;
    } else {
      ld_buf2(w[s][0], w[s][1], v0, v1, data_rsrc);
      if constexpr (KS == 24) {  // w[2..24]: 6 + 6 + 6 + 5
        ld_run<0, 6>(&w[s][2], v2, data_rsrc);
        ld_run<6 * (int)kStepBytes, 6>(&w[s][8], v2, data_rsrc);
        ld_run<12 * (int)kStepBytes, 6>(&w[s][14], v2, data_rsrc);
        ld_run<18 * (int)kStepBytes, 5>(&w[s][20], v2, data_rsrc);
      } else if constexpr (KS == 12) {  // w[2..12]: 6 + 5
        ld_run<0, 6>(&w[s][2], v2, data_rsrc);
        ld_run<6 * (int)kStepBytes, 5>(&w[s][8], v2, data_rsrc);
      } else {
        static_assert(KS == 6, "load runs are written out for KS = 6, 12 and 24");
        ld_run<0, 5>(&w[s][2], v2, data_rsrc);
      }
    }
    // 4. bounds of the next 4S+1 frames, for this slot's next issue
    nfb[s] = nf;
    bnd[s] = ld_buf<0>((nf + lane) * 8u, off_rsrc);
  };

  auto compute = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    slot_wait<kPending, kW>(w[s], bnd[s]);
    const uint32_t n = it_n[s], ns = it_ns[s], j0 = it_j0[s];
    const uint32_t J = (n + kStepBytes - 1) / kStepBytes;
    const uint32_t ra = it_e[s] & 3u;
    const bool alive = it_f[s] != kNoFrame;
    const bool first = alive && j0 == 0 && ns != 0;
    const bool last = alive && j0 + ns == J;
    uint32_t keep = 0xFFFFFFFFu, initm = 0, m1 = 0;
    if (first) {
      const uint32_t lead = J * kStepBytes - n;
      const uint32_t m4 = n < 4 ? n : 4u;
      const int32_t d0 = (int32_t)lead - (int32_t)(p << 2);
      keep = keep_from(d0);
      initm = keep & ~keep_from(d0 + (int32_t)m4);
      const int32_t x1 = (int32_t)(lead + m4) - (int32_t)kStepBytes;  // init bytes spilling into step 1
      if (x1 > 0 && p == 0) m1 = (uint32_t)((1ull << (8 * x1)) - 1);
      reg = 0;
    }
    const bool unaligned = un[s];
    const bool full = !wave_any(!alive || ns != (uint32_t)KS);
    auto word = [&](int k, bool unal) {
      uint32_t x = w[s][k + 1];
      if (unal) {
        const uint32_t t = (uint32_t)__builtin_amdgcn_mov_dpp((int)w[s][k], 0x121, 0xF, 0xF, false);  // row_ror:1
        const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)t, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
        x = __builtin_amdgcn_alignbyte(x, prev, ra);
      }
      if (k == 0) x = (x & keep) ^ initm;
      if (k == 1) x ^= m1;
      return x;
    };
    if constexpr (VAR == 1) {
#pragma unroll
      for (int k = 0; k < KS; ++k) reg ^= w[s][k + 1];
    } else {
      if (full && !unaligned) {
        // hot path: every row folds KS steps of a 4-byte-aligned frame, no
        // predication; the next word is XOR-ed in by the step's second bitop3
        uint32_t in = reg ^ word(0, false);
#pragma unroll
        for (int k = 0; k < KS - 1; ++k) in = u_step_xor(lds, in, word(k + 1, false), bu0, bu1);
        reg = u_step_xor(lds, in, 0u, bu0, bu1);
      } else if (!unaligned) {
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const uint32_t r2 = u_step_xor(lds, reg ^ word(k, false), 0u, bu0, bu1);
          reg = (uint32_t)k < ns ? r2 : reg;
        }
      } else {
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          const uint32_t r2 = u_step_xor(lds, reg ^ word(k, true), 0u, bu0, bu1);
          reg = (uint32_t)k < ns ? r2 : reg;
        }
      }
    }
    uint32_t crc = 0;
    if (wave_any(last)) {
      uint32_t R = row_xor(f_step(lds, reg, bf));
      R = n != 0 ? R : 0u;
      if (n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * n));
      crc = ~R;
    }
    // one store per slot, outside any branch: static vmcnt count
    const bool st = last && p == 0;
    if (MODE == CrcMode::kCrc)
      __builtin_amdgcn_raw_buffer_store_b32(crc, out_rsrc, st ? it_f[s] * 4u : kOOB, 0, 0);
    else
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)((n >= 4 && crc == 0x2144DF1Cu) ? 1 : 0), out_rsrc,
                                           st ? it_f[s] : kOOB, 0, 0);
  };

#define LNX_FENCE __builtin_amdgcn_sched_barrier(0)
  bool done = false;
  auto slot = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (done) return;
    compute(sc);
    live -= hw[s] ? 1 : 0;
    const bool more = nf < nwf || wave_any(rj < rJ);
    if (live == 0 && !more) {
      done = true;
      return;
    }
    LNX_FENCE;
    issue(sc);
    LNX_FENCE;
    live += hw[s] ? 1 : 0;
  };
  while (!done) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (slot(std::integral_constant<int, I>{}), ...);
    }(std::make_integer_sequence<int, S>{});
  }
#undef LNX_FENCE
  // drain: no asm load may still be writing registers when the wave ends
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------ kernel
// Item size per wave: long frames use 24-step items (a 1500-byte frame is one
// item, 2 slots), short frames 6-step items with 4 slots, so rows
// idle less at frame ends.  Chosen per wave from its mean frame length.
template <CrcMode MODE, int VAR = 0, int KSL = 24, int SL = 2>
__global__ void __launch_bounds__(kBlockThreads, 1)
crc32_rows_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t nframes,
                  uint64_t frames_per_wave, const uint4* __restrict__ image, void* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[kLdsDwords];
  {
    uint4* l4 = reinterpret_cast<uint4*>(lds_words);
#pragma unroll
    for (int i = 0; i < (int)(kLdsBytes / 16 / kBlockThreads); ++i)
      l4[threadIdx.x + i * kBlockThreads] = image[threadIdx.x + i * kBlockThreads];
  }

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t p = lane & 15u;
  const uint32_t row = lane >> 4;
  const uint32_t col = lane & 31u;
  const uint32_t bu0 = col << 2;
  const uint32_t bu1 = bu0 | 65536u;
  const uint32_t bf = kFBase | (col << 2);
  const uint64_t gwave = (uint64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t fw0 = gwave * frames_per_wave < nframes ? gwave * frames_per_wave : nframes;
  const uint64_t fw1 = fw0 + frames_per_wave < nframes ? fw0 + frames_per_wave : nframes;
  const uint32_t nwf = (uint32_t)(fw1 - fw0);
  __syncthreads();
  const char* lds = reinterpret_cast<const char*>(lds_words);
  if (nwf == 0) return;

  // The wave's byte range, addressed through one buffer descriptor whose base
  // is 4-byte aligned: rel(x) = x - off[fw0] + adj.
  const uint64_t o0 = off[fw0];
  const uint64_t o1 = off[fw1];
  const uint64_t range = o1 > o0 ? o1 - o0 : 0;  // non-decreasing offsets are the contract
  const uint32_t adj = (uint32_t)((reinterpret_cast<uintptr_t>(bytes) + o0) & 3u);
  if (range + adj + kStepBytes >= (1ull << 31)) {
    rows_generic<MODE>(lds, bytes, off, fw0, fw1, out, p, row, bu0, bu1, bf);
    return;
  }
  const __amdgpu_buffer_rsrc_t data_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint8_t*>(bytes + o0 - adj), (short)0, (int)((range + adj + 3) & ~3ull), 0x00020000);
  const __amdgpu_buffer_rsrc_t off_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<uint64_t*>(off + fw0), (short)0, (int)((nwf + 1) * 8u), 0x00020000);
  constexpr uint32_t elem = MODE == CrcMode::kCrc ? 4u : 1u;
  const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char*>(out) + fw0 * elem, (short)0, (int)(nwf * elem), 0x00020000);
  const uint32_t o0_lo = (uint32_t)o0;
  asm volatile("s_nop 4" ::: "memory");  // descriptors may be SGPRs just written by VALU readfirstlane

  WaveCtx cx;
  cx.lds = lds;
  cx.lane = lane;
  cx.p = p;
  cx.row = row;
  cx.bu0 = bu0;
  cx.bu1 = bu1;
  cx.bf = bf;
  cx.nwf = nwf;
  cx.o0_lo = o0_lo;
  cx.adj = adj;
  cx.data_rsrc = data_rsrc;
  cx.off_rsrc = off_rsrc;
  cx.out_rsrc = out_rsrc;
  if (range >= (uint64_t)nwf * 768u)
    rows_body<MODE, KSL, SL, VAR>(cx);
  else
    rows_body<MODE, 6, 4, VAR>(cx);
}

hipError_t launch_rows(int var, bool verify, const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out,
                       const void* image, int num_cus, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  const uint64_t per_block = (uint64_t)kWavesPerBlock * kRows;
  uint64_t grid = (n + per_block - 1) / per_block;
  if (grid > (uint64_t)num_cus) grid = (uint64_t)num_cus;
  const uint64_t waves = grid * kWavesPerBlock;
  const uint64_t fpw = (n + waves - 1) / waves;
  const uint4* img = static_cast<const uint4*>(image);
  const dim3 g((unsigned)grid), b(kBlockThreads);
#define LNX_LAUNCH(M, V, K, S) \
  hipLaunchKernelGGL((crc32_rows_kernel<M, V, K, S>), g, b, 0, stream, bytes, off, n, fpw, img, out)
  if (verify) {
    LNX_LAUNCH(CrcMode::kVerify, 0, 24, 2);
  } else {
    switch (var) {
      case 1: LNX_LAUNCH(CrcMode::kCrc, 1, 24, 2); break;
      case 2: LNX_LAUNCH(CrcMode::kCrc, 2, 24, 2); break;
      case 10: LNX_LAUNCH(CrcMode::kCrc, 0, 24, 3); break;
      case 11: LNX_LAUNCH(CrcMode::kCrc, 0, 12, 3); break;
      case 12: LNX_LAUNCH(CrcMode::kCrc, 0, 12, 4); break;
      case 13: LNX_LAUNCH(CrcMode::kCrc, 1, 24, 3); break;
      case 14: LNX_LAUNCH(CrcMode::kCrc, 1, 12, 4); break;
      default: LNX_LAUNCH(CrcMode::kCrc, 0, 24, 2); break;
    }
  }
#undef LNX_LAUNCH
  return hipGetLastError();
}

// Host-side launch helpers (called from api.cpp).
hipError_t launch_crc32_frames(const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out, bool verify,
                               const void* image, int num_cus, hipStream_t stream) {
  return launch_rows(0, verify, bytes, off, n, out, image, num_cus, stream);
}
hipError_t launch_crc32_variant(int var, const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out,
                                const void* image, int num_cus, hipStream_t stream) {
  return launch_rows(var, false, bytes, off, n, out, image, num_cus, stream);
}

}  // namespace lnx
