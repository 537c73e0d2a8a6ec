// crc32_kernel.hip — batched CRC-32/IEEE (Ethernet FCS) over packed frames, gfx950.
//
// Reference semantics: ethernet.CRC32 (lneto ethernet/crc.go:19-21) =
// Go crc32.Checksum(data, IEEETable): init 0xFFFFFFFF, reflected, xorout
// 0xFFFFFFFF.  The FCS-verify mode implements the residue form of the check a
// receiver does before StackEthernet.Demux (internet/stack-ethernet.go:139).
//
// Work decomposition
// -----------------------------------
// A wave is 64/RL rows of RL lanes; each row folds one frame (RL = 16 for long
// frames, RL = 4 for short ones; a workgroup picks one from its frames' mean
// length and loads that row width's LDS image).  A frame is viewed through a
// window that ENDS at the frame end rounded up to 4 bytes and is a whole
// number J of SB = 4*RL byte steps long; the lead-in before the frame start is
// zero-masked.  With init 0 the CRC register ignores leading zeros, so the
// window's register equals the frame's; the init value is folded in by XOR-ing
// 0xFF into the frame's first four bytes.
//
// Lane p of a row consumes the aligned word at window offset 4p + SB*j: one
// dword load per wave per step covers 64/RL frames.  Each lane keeps its own
// register r and advances it with r = U(r ^ w), U = Z_SB, through four
// lane-private byte tables in LDS (lds_layout.hpp) — conflict-free whatever
// the data.  After the last step lane p's register sits 4p bytes past the
// window end; F_p = Z_{-4p} (lane-private nibble tables) moves it back, the
// row's XOR combines the lanes (DPP), and Z_{-t} (the t = 0..3 bytes the window
// runs past the frame end; nibbles shared over the row's lanes) lands it on
// the frame end.  The t bytes themselves belong to the next frame: the last
// lane's junk is loaded once more on its own and its U-image XOR-ed out.
// No MFMA: this is a per-byte GF(2) polynomial.
//
// Everything per frame (bounds, window position, masks) is a row-uniform VGPR
// value, so one instruction serves 64/RL frames.
//
// Pipeline: each row's frames are cut into items of <= KS steps.  A ring of S
// slots (one item per row per slot) keeps the next S-1 slots' loads in flight
// while one slot is folded.  Streaming loads are inline-asm raw buffer loads
// over the wave's own byte range from ONE per-lane base offset plus immediate
// step offsets; the range check applies to the wrapped 32-bit base+immediate,
// so lead-ins before the range, idle steps past it and idle rows (base kOOB)
// read 0 and touch no memory.  vmcnt is hand-counted: every slot issues exactly
// KS + 2 loads (KS steps, the junk word, the next bounds window).  Frame bounds
// come from a per-slot prefetch of the next S*NR+1 offsets (lane i holds the
// low dword of off[nf+i]), shuffled to the rows with ds_bpermute.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include <type_traits>
#include <utility>
#include "lds_layout.hpp"
#include "dispatch.hpp"

// Cache-policy suffix of the streaming frame loads (e.g. " nt" for profiling
// builds: make CXXFLAGS+='-DLNX_LD_POL=\"\ nt\"').  Default policy by default.
#ifndef LNX_LD_POL
#define LNX_LD_POL ""
#endif

namespace lnx {

constexpr int kBlockThreads = 1024;
constexpr int kWavesPerBlock = kBlockThreads / 64;
constexpr uint32_t kNoFrame = 0xFFFFFFFFu;
// Buffer offset that is out of range with any immediate added (ranges < 2^31).
constexpr uint32_t kOOB = 0x80000000u;
// A workgroup whose frames average fewer bytes than this uses 4-lane rows.
constexpr uint64_t kShortMean = 640;

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

// F_p(r) through eight lane-private nibble tables (pairs interleaved, see
// lds_layout.hpp): the even nibbles are the bytes of r & 0x0F0F0F0F, the odd
// ones those of (r >> 4) & 0x0F0F0F0F, so each address is one v_perm with the
// lane base bf (the table offset rides in the ds_read immediate); the eight
// values are XOR-ed by three v_bitop3 and a v_xor: 14 VALU, 8 LDS.
__device__ __forceinline__ uint32_t f_step(const char* lds, uint32_t r, uint32_t bf) {
  const uint32_t y = r & 0x0F0F0F0Fu, z = (r >> 4) & 0x0F0F0F0Fu;
  uint32_t v[8];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    v[2 * k] = lds_rd(lds, __builtin_amdgcn_perm(y, bf, 0x0c020400u + ((uint32_t)k << 8)) + (uint32_t)(k << 12));
    v[2 * k + 1] =
        lds_rd(lds, __builtin_amdgcn_perm(z, bf, 0x0c020400u + ((uint32_t)k << 8)) + (uint32_t)((k << 12) + 128));
  }
  const uint32_t a = __builtin_amdgcn_bitop3_b32(v[0], v[1], v[2], 0x96);
  const uint32_t b = __builtin_amdgcn_bitop3_b32(v[3], v[4], v[5], 0x96);
  return __builtin_amdgcn_bitop3_b32(a, b, v[6] ^ v[7], 0x96);
}

// v ^ (v moved by the DPP control): bound_ctrl lets hipcc fold the move into
// one v_xor_b32_dpp (no lane reads out of bounds with these controls).
template <int CTRL>
__device__ __forceinline__ uint32_t dpp_xor(uint32_t v) {
  return v ^ (uint32_t)__builtin_amdgcn_mov_dpp((int)v, CTRL, 0xF, 0xF, true);
}
constexpr int kQuadX1 = 0xB1, kQuadX2 = 0x4E, kRowRor4 = 0x124, kRowRor8 = 0x128;

// XOR over the RL lanes of each row; every lane gets its row's result.  A
// 32-lane row spans two 16-lane DPP rows: v_permlane16_swap of v with itself
// pairs them (gfx950).
template <int RL>
__device__ __forceinline__ uint32_t row_xor(uint32_t v) {
  v = dpp_xor<kQuadX1>(v);
  v = dpp_xor<kQuadX2>(v);
  if constexpr (RL >= 16) {
    v = dpp_xor<kRowRor4>(v);
    v = dpp_xor<kRowRor8>(v);
  }
  if constexpr (RL == 32) {
    const auto sw = __builtin_amdgcn_permlane16_swap(v, v, false, false);
    v = sw[0] ^ sw[1];
  }
  return v;
}

// Z_{-t}(R) for a row-uniform R, the nibbles shared over the row (T region);
// t = 0 is the identity: each lane then contributes its nibbles in place.  A
// 32-lane row does it per 16-lane half, both halves alike (q = p & 7).
template <int RL>
__device__ __forceinline__ uint32_t t_fix(const char* lds, uint32_t R, uint32_t t, uint32_t p, uint32_t bt) {
  const uint32_t tb = bt + (((t - 1u) & 3u) << 11);  // entry (h, t, v) = 48h + 16(t-1) + v, stride 128 B
  if constexpr (RL >= 16) {
    const uint32_t q = p & 7u;  // lanes p and p+8 cover the same nibble
    const uint32_t nib = (R >> (4 * q)) & 15u;
    const uint32_t a0 = lds_rd(lds, tb + (nib << 7));
    uint32_t a = t ? a0 : nib << (4 * q);
    a = dpp_xor<kQuadX1>(a);
    a = dpp_xor<kQuadX2>(a);
    return dpp_xor<kRowRor4>(a);  // quads {0-3,4-7}, {4-7,8-11}, ... : 8 distinct nibbles
  } else {
    const uint32_t n0 = (R >> (4 * p)) & 15u, n1 = (R >> (4 * p + 16)) & 15u;
    const uint32_t a0 = lds_rd(lds, tb + (n0 << 7)) ^ lds_rd(lds, tb + ((48u + n1) << 7));
    uint32_t a = t ? a0 : (n0 << (4 * p)) | (n1 << (4 * p + 16));
    a = dpp_xor<kQuadX1>(a);
    return dpp_xor<kQuadX2>(a);
  }
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
  asm volatile("s_nop 4\n\tbuffer_load_dword %0, %1, %2, 0 offen offset:%3" LNX_LD_POL
               : "=v"(r) : "v"(voff), "s"(rsrc), "i"(IMM));
  return r;
}

#define LNX_O(k) [o##k] "=&v"(o[k])
#define LNX_I(k) [i##k] "i"(IMM0 + (k) * D)
// N (1..6) loads from one VGPR offset at immediates IMM0, IMM0 + D, ...
// NT: non-temporal policy.  Only rows that read whole 128-byte lines per
// instruction gain from it (32-lane rows, tools/ubench/pattern3.hip: +10 %
// over default-policy rows); 64-byte half lines lose 10-20 % with nt.
template <int IMM0, int N, int D, bool NT>
__device__ __forceinline__ void ld_run(uint32_t* o, uint32_t v, __amdgpu_buffer_rsrc_t rsrc) {
  static_assert(N >= 1 && N <= 6 && IMM0 + (N - 1) * D <= 4095, "run shape");
#define LNX_L(k) "buffer_load_dword %[o" #k "], %[v], %[r], 0 offen offset:%[i" #k "] nt\n\t"
  if constexpr (!NT) {
  } else if constexpr (N == 6) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3) LNX_L(4) LNX_L(5)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3), LNX_O(4), LNX_O(5)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3), LNX_I(4), LNX_I(5));
  } else if constexpr (N == 5) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3) LNX_L(4)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3), LNX_O(4)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3), LNX_I(4));
  } else if constexpr (N == 4) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3));
  } else if constexpr (N == 3) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2)
                 : LNX_O(0), LNX_O(1), LNX_O(2)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2));
  } else if constexpr (N == 2) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1)
                 : LNX_O(0), LNX_O(1)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1));
  } else {
    asm volatile("s_nop 4\n\t" LNX_L(0) : LNX_O(0) : [v] "v"(v), [r] "s"(rsrc), LNX_I(0));
  }
#undef LNX_L
#define LNX_L(k) "buffer_load_dword %[o" #k "], %[v], %[r], 0 offen offset:%[i" #k "]" LNX_LD_POL "\n\t"
  if constexpr (NT) {
  } else if constexpr (N == 6) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3) LNX_L(4) LNX_L(5)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3), LNX_O(4), LNX_O(5)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3), LNX_I(4), LNX_I(5));
  } else if constexpr (N == 5) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3) LNX_L(4)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3), LNX_O(4)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3), LNX_I(4));
  } else if constexpr (N == 4) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3));
  } else if constexpr (N == 3) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2)
                 : LNX_O(0), LNX_O(1), LNX_O(2)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2));
  } else if constexpr (N == 2) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1)
                 : LNX_O(0), LNX_O(1)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1));
  } else {
    asm volatile("s_nop 4\n\t" LNX_L(0) : LNX_O(0) : [v] "v"(v), [r] "s"(rsrc), LNX_I(0));
  }
}
#undef LNX_L
#undef LNX_O
#undef LNX_I

// All KS step loads of an item: runs of up to six from the one base offset.
template <int K0, int KS, int D, bool NT>
__device__ __forceinline__ void ld_item(uint32_t* w, uint32_t v, __amdgpu_buffer_rsrc_t rsrc) {
  if constexpr (K0 < KS) {
    constexpr int N = KS - K0 < 6 ? KS - K0 : 6;
    ld_run<K0 * D, N, D, NT>(w + K0, v, rsrc);
    ld_item<K0 + N, KS, D, NT>(w, v, rsrc);
  }
}

// The same in runs of R steps whose base is out of range (no memory traffic)
// unless the item has the run's first step (K0 < ns): an item shorter than KS
// does not read the bytes past its frame's window (R - 1 junk steps at most).
template <int K0, int KS, int D, int R>
__device__ __forceinline__ void ld_item_ns(uint32_t* w, uint32_t v, uint32_t ns, __amdgpu_buffer_rsrc_t rsrc) {
  if constexpr (K0 < KS) {
    constexpr int N = KS - K0 < R ? KS - K0 : R;
    ld_run<K0 * D, N, D, false>(w + K0, (uint32_t)K0 < ns ? v : kOOB, rsrc);
    ld_item_ns<K0 + N, KS, D, R>(w, v, ns, rsrc);
  }
}

// The same with dwordx2 loads (two words per lane; always non-temporal).
#define LNX_L(k) "buffer_load_dwordx2 %[o" #k "], %[v], %[r], 0 offen offset:%[i" #k "] nt\n\t"
#define LNX_O(k) [o##k] "=&v"(o[k])
#define LNX_I(k) [i##k] "i"(IMM0 + (k) * D)
template <int IMM0, int N, int D>
__device__ __forceinline__ void ld_run2(uint64_t* o, uint32_t v, __amdgpu_buffer_rsrc_t rsrc) {
  static_assert(N >= 1 && N <= 6 && IMM0 + (N - 1) * D <= 4095, "run shape");
  if constexpr (N == 6) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3) LNX_L(4) LNX_L(5)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3), LNX_O(4), LNX_O(5)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3), LNX_I(4), LNX_I(5));
  } else if constexpr (N == 5) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3) LNX_L(4)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3), LNX_O(4)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3), LNX_I(4));
  } else if constexpr (N == 4) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3));
  } else if constexpr (N == 3) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2)
                 : LNX_O(0), LNX_O(1), LNX_O(2)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2));
  } else if constexpr (N == 2) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1)
                 : LNX_O(0), LNX_O(1)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1));
  } else {
    asm volatile("s_nop 4\n\t" LNX_L(0) : LNX_O(0) : [v] "v"(v), [r] "s"(rsrc), LNX_I(0));
  }
}
#undef LNX_L
#undef LNX_O
#undef LNX_I
// One dwordx2 load with the default cache policy (the line stays in L2).
template <int IMM>
__device__ __forceinline__ void ld_x2d(uint64_t& o, uint32_t v, __amdgpu_buffer_rsrc_t rsrc) {
  asm volatile("s_nop 4\n\tbuffer_load_dwordx2 %0, %1, %2, 0 offen offset:%3" : "=&v"(o) : "v"(v), "s"(rsrc), "i"(IMM));
}
template <int K0, int KS, int D, bool NT>
__device__ __forceinline__ void ld_item(uint64_t* w, uint32_t v, __amdgpu_buffer_rsrc_t rsrc) {
  if constexpr (K0 < KS) {
    constexpr int N = KS - K0 < 6 ? KS - K0 : 6;
    ld_run2<K0 * D, N, D>(w + K0, v, rsrc);
    ld_item<K0 + N, KS, D, NT>(w, v, rsrc);
  }
}

// The same with dwordx4 loads (four words per lane: 4-lane rows reading 64
// contiguous bytes per row instruction, the narrow rows of the Zipf mix).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
#define LNX_L(k) "buffer_load_dwordx4 %[o" #k "], %[v], %[r], 0 offen offset:%[i" #k "]\n\t"
#define LNX_O(k) [o##k] "=&v"(o[k])
#define LNX_I(k) [i##k] "i"(IMM0 + (k) * D)
template <int IMM0, int N, int D>
__device__ __forceinline__ void ld_run4(u32x4* o, uint32_t v, __amdgpu_buffer_rsrc_t rsrc) {
  static_assert(N >= 1 && N <= 4 && IMM0 + (N - 1) * D <= 4095, "run shape");
  if constexpr (N == 4) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2) LNX_L(3)
                 : LNX_O(0), LNX_O(1), LNX_O(2), LNX_O(3)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2), LNX_I(3));
  } else if constexpr (N == 3) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1) LNX_L(2)
                 : LNX_O(0), LNX_O(1), LNX_O(2)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1), LNX_I(2));
  } else if constexpr (N == 2) {
    asm volatile("s_nop 4\n\t" LNX_L(0) LNX_L(1)
                 : LNX_O(0), LNX_O(1)
                 : [v] "v"(v), [r] "s"(rsrc), LNX_I(0), LNX_I(1));
  } else {
    asm volatile("s_nop 4\n\t" LNX_L(0) : LNX_O(0) : [v] "v"(v), [r] "s"(rsrc), LNX_I(0));
  }
}
#undef LNX_L
#undef LNX_O
#undef LNX_I
// Runs of R dwordx4 step loads whose base is out of range (no traffic) unless
// the item has the run's first step (as ld_item_ns).
template <int K0, int KS, int D, int R>
__device__ __forceinline__ void ld_item4_ns(u32x4* w, uint32_t v, uint32_t ns, __amdgpu_buffer_rsrc_t rsrc) {
  if constexpr (K0 < KS) {
    constexpr int N = KS - K0 < R ? KS - K0 : R;
    ld_run4<K0 * D, N, D>(w + K0, (uint32_t)K0 < ns ? v : kOOB, rsrc);
    ld_item4_ns<K0 + N, KS, D, R>(w, v, ns, rsrc);
  }
}

// vmcnt wait naming every register of one slot: the wait, then empty asm
// statements that "redefine" each register, so no use is scheduled above it.
template <int N, int KS, typename Word>
__device__ __forceinline__ void slot_wait(Word (&w)[KS], uint32_t& junk, uint32_t& b0, uint32_t& b1) {
  asm volatile("s_waitcnt vmcnt(%0)" ::"i"(N));
#pragma unroll
  for (int k = 0; k < KS; ++k) asm volatile("" : "+v"(w[k]));
  asm volatile("" : "+v"(junk), "+v"(b0), "+v"(b1));
}

// kAppend (segment mode only): the TX FCS append of lnx_fcs_append_batch
// (internet/stack-ethernet.go:200-214) — frame i is zero-padded to 60 bytes
// and LE32(CRC32(padded frame)) is written after it, len[i] = padded + 4,
// status[i] = 0; a frame whose padded length + 4 exceeds the capacity is left
// untouched with status 6 (ErrShortBuffer).  The CRC of the padded frame is
// the frame's register advanced over the k = 60 - n pad bytes (zero_advance):
// the pad is written, never read.
enum class CrcMode : int { kCrc = 0, kVerify = 1, kAppend = 2 };
constexpr uint32_t kMinFrame = 60;
constexpr uint8_t kErrShortBuffer = 6;

// The result of frame f: its CRC, or (verify mode) 1 if the residue matches.
template <CrcMode MODE>
__device__ __forceinline__ uint32_t result_of(uint32_t n, uint32_t crc) {
  return MODE != CrcMode::kVerify ? crc : ((n >= 4 && crc == 0x2144DF1Cu) ? 1u : 0u);
}
template <CrcMode MODE>
__device__ __forceinline__ void store_result(__amdgpu_buffer_rsrc_t out_rsrc, bool st, uint32_t f, uint32_t v) {
  if (MODE == CrcMode::kCrc)
    __builtin_amdgcn_raw_buffer_store_b32(v, out_rsrc, st ? f * 4u : kOOB, 0, 0);
  else
    __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, out_rsrc, st ? f : kOOB, 0, 0);
}

// Per-lane constants.
struct Lanes {
  uint32_t lane, p, row, bu0, bu1, bf, bt;
};

// kAppend: the byte at rel 0 of the range, its lengths (written back) and
// status bytes, and the slot capacity.
struct WaveCtxAppend {
  uint8_t* data_base;
  uint32_t* lenw;
  uint8_t* stat;
  uint32_t cap;
  uint32_t rend;  // rel end of the range's bytes (its last frame's end)
};
// he value of a held frame whose FCS is already in memory (written with its
// 64-byte sector, lines_body): the flush writes its length and status only
constexpr uint32_t kFcsWritten = 0xFFFFFFFFu;

// Z_k(x), k = 1 .. 4 SB (k zero bytes appended to the register x; k = 0:
// identity), for a row-uniform x and k, with the tables of the image the
// workgroup loaded (row width IMGRL: U = Z_SB, SB = 4 IMGRL; column c of F is
// Z_{-4 (c mod IMGRL)}; T = Z_{-t}, t < 4): Z_k = U^m o Z_{-4a} o Z_{-b} with
// m = ceil(k / SB) and m SB - k = 4a + b.  RL: lanes per row (t_fix's row).
template <int RL, int IMGRL>
__device__ __forceinline__ uint32_t zero_advance(const char* lds, uint32_t x, uint32_t k, const Lanes& L) {
  constexpr uint32_t SB = 4u * IMGRL;
  const uint32_t m = (k + SB - 1u) / SB, d = m * SB - k;
  if (wave_any((d >> 2) != 0u)) {
    const uint32_t c = ((L.lane & 31u) & ~(uint32_t)(IMGRL - 1)) | (d >> 2);
    const uint32_t y = f_step(lds, x, kFBase | (c << 2));
    x = (d >> 2) ? y : x;
  }
  x = t_fix<RL>(lds, x, d & 3u, L.p, L.bt);
  for (uint32_t i = 0; wave_any(i < m); ++i) {
    const uint32_t y = u_step(lds, x, L.bu0, L.bu1);
    x = i < m ? y : x;
  }
  return x;
}

// The append tail of one frame (row-uniform n, R = its register before the
// final complement, e = address of its end byte): the k = 60 - n pad bytes and
// the LE FCS are written by the row's lanes (byte j = j0 + p), lane 0 writes
// the new length and the status.  live: the row holds a finished frame.
// The pad half of append_tail for the pipelined bodies: R advanced over the
// k = 60 - n pad bytes, which the row's lanes write at e (rare: runts only);
// the FCS, length and status are held and flushed with the other results
// (store_held), so the ring's vmcnt waits do not wait on a store per slot.
template <int RL, int IMGRL>
__device__ __forceinline__ uint32_t append_pad(const char* lds, const Lanes& L, bool live, uint32_t n, uint32_t R,
                                               uint8_t* e, uint32_t cap, uint32_t& k) {
  // a runt that would outgrow its slot once padded is left untouched (status 6)
  k = live && n < kMinFrame && kMinFrame + 4u <= cap ? kMinFrame - n : 0u;
  if (wave_any(k != 0u)) {
    const uint32_t z = zero_advance<RL, IMGRL>(lds, R, k, L);
    R = k ? z : R;
    for (uint32_t j0 = 0; wave_any(j0 < k); j0 += RL) {
      const uint32_t j = j0 + L.p;
      if (j < k) e[j] = 0;
    }
  }
  return R;
}
// Held append results of a lane: frame hf (relative), FCS hv at rel position
// he, new length hpl (0: the frame did not fit, status ErrShortBuffer).
__device__ __forceinline__ void store_held(const WaveCtxAppend& a, bool st, uint32_t hf, uint32_t hv, uint32_t he,
                                           uint32_t hpl) {
  if (st && hpl) {
    if (he != kFcsWritten) {
      uint8_t* q = a.data_base + he;
      if ((reinterpret_cast<uintptr_t>(q) & 3u) == 0) {  // one dword store (LE: the FCS byte order)
        *reinterpret_cast<uint32_t*>(q) = hv;
      } else {
        q[0] = (uint8_t)hv, q[1] = (uint8_t)(hv >> 8), q[2] = (uint8_t)(hv >> 16), q[3] = (uint8_t)(hv >> 24);
      }
    }
    a.lenw[hf] = hpl;
  }
  if (st) a.stat[hf] = hpl ? (uint8_t)0 : kErrShortBuffer;
}

template <int RL, int IMGRL>
__device__ __forceinline__ void append_tail(const char* lds, const Lanes& L, bool live, uint32_t n, uint32_t R,
                                            uint8_t* e, uint32_t cap, uint32_t* len_at, uint8_t* status_at) {
  const uint32_t k = live && n < kMinFrame ? kMinFrame - n : 0u;
  if (wave_any(k != 0u)) {
    const uint32_t z = zero_advance<RL, IMGRL>(lds, R, k, L);
    R = k ? z : R;
  }
  const uint32_t crc = ~R;
  const uint32_t pl = n + k;
  const bool ok = live && (uint64_t)pl + 4u <= cap;
  const uint32_t tot = k + 4u;
  for (uint32_t j0 = 0; wave_any(ok && j0 < tot); j0 += RL) {
    const uint32_t j = j0 + L.p;
    if (ok && j < tot) e[j] = j < k ? (uint8_t)0 : (uint8_t)(crc >> (8u * (j - k)));
  }
  if (live && L.p == 0) {
    if (ok) *len_at = pl + 4u;
    *status_at = ok ? (uint8_t)0 : kErrShortBuffer;
  }
}

// ------------------------------------------------------------------ generic path
// For a wave whose byte range does not fit a 31-bit buffer offset (frames of
// gigabytes): same algorithm with the window ending exactly at the frame end,
// byte loads with explicit bounds, no pipelining.
template <CrcMode MODE, int RL>
__device__ void rows_generic(const char* lds, const Lanes& L, const uint8_t* bytes, const uint64_t* off,
                             const uint32_t* seg_len, uint64_t fw0, uint64_t fw1, void* out, uint32_t cap) {
  constexpr uint32_t NR = 64 / RL, SB = 4 * RL;
  const uint64_t fend = fw0 + ((fw1 - fw0 + NR - 1) / NR) * NR;
  for (uint64_t f = fw0 + L.row; f < fend; f += NR) {
    const bool live = f < fw1;
    const uint64_t s = live ? off[f] : 0, e = live ? (seg_len ? s + seg_len[f] : off[f + 1]) : 0;
    const uint64_t n = e > s ? e - s : 0;
    const uint64_t J = (n + SB - 1) / SB;
    uint32_t reg = 0;
    for (uint64_t j = 0; j < J; ++j) {
      const int64_t pos = (int64_t)e - (int64_t)((J - j) * SB) + 4 * (int64_t)L.p;
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
      reg = u_step(lds, reg ^ x, L.bu0, L.bu1);
    }
    uint32_t R = n ? row_xor<RL>(f_step(lds, reg, L.bf)) : 0u;
    if (n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * n));
    if constexpr (MODE == CrcMode::kAppend) {  // segment mode: n < 2^32
      append_tail<RL, RL>(lds, L, live, (uint32_t)n, R, const_cast<uint8_t*>(bytes) + e, cap,
                          const_cast<uint32_t*>(seg_len) + f, reinterpret_cast<uint8_t*>(out) + f);
      continue;
    }
    const uint32_t crc = ~R;
    if (live && L.p == 0) {
      if (MODE == CrcMode::kCrc)
        reinterpret_cast<uint32_t*>(out)[f] = crc;
      else
        reinterpret_cast<uint8_t*>(out)[f] = (n >= 4 && crc == 0x2144DF1Cu) ? 1 : 0;
    }
  }
}

// ------------------------------------------------------------------ ring body
// Workgroup-uniform context of the pipelined path.  Positions are
// rel(x) = x - off[fb0] + adj, frame indices relative to fb0.
struct WaveCtx {
  uint32_t nfb, o0_lo, adj;  // frames of the range, low dword of its first offset, alignment
  uint32_t* ctr;             // LDS frame-chunk counter (lds_layout.hpp kCtrBase)
  __amdgpu_buffer_rsrc_t data_rsrc, off_rsrc, out_rsrc;
  __amdgpu_buffer_rsrc_t len_rsrc;  // segment mode: the length array
  WaveCtxAppend ap;                 // kAppend
};

// RL: lanes per row, KS: window steps per item, S: ring slots, CH: frames per
// chunk, VAR: profiling knob (0 = product, 1 = loads +
// bookkeeping only, 2 = lookups + bookkeeping on synthetic words).  Only VAR 0
// is reachable from the C-ABI.
//
// Work distribution: the waves of a workgroup claim chunks of CH consecutive
// frames from an LDS counter (one ds_add_rtn per chunk), so a wave that the
// memory system serves faster simply takes more chunks; with static ranges the
// waves of one CU finished up to 1.5x apart (tools/prof/timeline.py).  A wave
// sees its chunks as one virtual frame sequence v = 0, 1, ...: it holds the
// bases of the chunk v is in (bc) and of the next one (bn), which covers the
// S*NR-frame bounds window every slot prefetches.
//
// WL: words per lane per step.  WL = 2 (16-lane rows only): each lane loads
// two consecutive dwords (buffer_load_dwordx2), so a row reads a whole
// 128-byte line per instruction like a 32-lane row, while a wave still
// carries four frames.  Lane p then holds the registers of "virtual lanes"
// v = 2p and 2p + 1 of a 32-virtual-lane row; all the window algebra below is
// in virtual lanes.
template <CrcMode MODE, int RL, int KS, int S, int CH, int VAR, bool SEG, int WL = 1, bool EDGE = true, int NSR = 0>
__device__ __forceinline__ void rows_body(const char* lds, const Lanes& L, const WaveCtx& cx) {
  constexpr uint32_t NR = 64 / RL;  // rows (frames in flight) per wave
  constexpr uint32_t VL = RL * WL;  // virtual lanes per row
  constexpr uint32_t SB = 4 * VL;   // bytes a row consumes per step
  constexpr uint32_t kSbLog = VL == 32 ? 7 : VL == 16 ? 6 : 4;  // (4 x 4 words: VL 16)
  static_assert(RL == 4 || RL == 16 || RL == 32, "row width");
  static_assert(WL == 1 || (WL == 2 && RL == 16) || (WL == 4 && RL == 4),
                "two words per lane: 16-lane rows; four words per lane: 4-lane rows");
  using Word = std::conditional_t<WL == 4, u32x4, std::conditional_t<WL == 2, uint64_t, uint32_t>>;
  // word h of a step's load
  auto wsel = [](const Word& x, int h) -> uint32_t {
    if constexpr (WL == 4) return x[h];
    else return (uint32_t)((uint64_t)x >> (32 * h));
  };

  // Rows of 32 virtual lanes read whole 128-byte lines: the window runs
  // between line boundaries (the range descriptor is line-aligned, cx.adj),
  // the loads are non-temporal, t = 4a + b window bytes follow the frame end
  // (a < 32), the virtual lanes v >= 32 - a skip the frame's last step (their
  // word there is all junk), virtual lane 31 - a takes the U-image of its b
  // junk bytes out, and the finish rotates the registers by a virtual lanes
  // before F (tests/cpp/rows_emulator.cpp crc32w).  Narrower
  // rows: window end = frame end rounded up to 4 bytes, t = 0..3 on the last
  // lane.
  constexpr bool kLine = VL == 32;
  // the row width of the LDS image the workgroup loaded (four-word 4-lane
  // rows: 16 virtual lanes, the RL = 16 image)
  constexpr int kImg = kLine ? 32 : (WL == 4 ? 16 : RL);
  // Four-word 4-lane rows read 16-byte chunks: the window (and the range
  // descriptor's base) is 16-byte aligned so that no lane's chunk straddles the
  // range start (a dwordx4 whose offset wraps below 0 returns all-zero, the
  // valid dwords included); the t = 4a + b window bytes past the frame end then
  // follow the line rows' algebra on 16 virtual lanes.
  constexpr bool kSkip = kLine || WL == 4;  // lanes past the end skip the last step
  constexpr uint32_t kEndAlign = kLine ? 128u : WL == 4 ? 16u : 4u;
  static_assert(S >= 1 && NR <= (uint32_t)CH && CH <= 64 && S * NR <= 64, "chunk and bounds window shape");
  static_assert(KS >= 2 && (KS - 1) * SB <= 4095, "buffer immediate offset");
  constexpr int kLoads = (VAR == 2 ? 0 : KS) + 3;  // steps, junk, start + end
  // bounds window: only lanes < S*NR are ever read back (ds_bpermute index
  // li < S*NR); the other lanes' offset loads are out of range (VAR 3: all 64
  // lanes load, the earlier behaviour, for A/B timing)
  constexpr uint32_t kWin = VAR == 3 ? 64u : S * NR;
  constexpr int kPending = (S - 1) * kLoads;       // loads issued after a slot's own
  const uint32_t lane = L.lane, p = L.p, row = L.row, bu0 = L.bu0, bu1 = L.bu1, bf = L.bf, bt = L.bt;
  const uint32_t nfb = cx.nfb, o0_lo = cx.o0_lo, adj = cx.adj;
  const __amdgpu_buffer_rsrc_t data_rsrc = cx.data_rsrc, off_rsrc = cx.off_rsrc, out_rsrc = cx.out_rsrc;
  // four-word 4-lane rows: a T column of the RL = 16 image whose nibble pair is
  // (p, p + 4), spread over the banks by row
  const uint32_t bt4 = kTBase | ((p + ((row & 1u) << 3) + (((row >> 1) & 1u) << 4)) << 2);
  Lanes Lz = L;  // the lane constants zero_advance uses (append mode)
  if constexpr (WL == 4) Lz.bt = bt4;

  // ---- chunks (uniform): one ds_add_rtn on the workgroup's LDS counter
  auto claim = [&]() -> uint32_t {
    uint32_t b = 0;
    if (lane == 0) b = __hip_atomic_fetch_add(cx.ctr, (uint32_t)CH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
  };
  // The bounds window [nf, nf + S*NR) starts inside chunk cc, so it touches
  // chunks cc .. cc + NB - 1; their first frames are held in cb[].
  constexpr uint32_t NB = 1 + (CH + S * NR - 2) / CH;
  static_assert((CH & (CH - 1)) == 0, "power-of-two chunks");
  constexpr uint32_t kChLog = __builtin_ctz(CH);
  uint32_t cc = 0;          // virtual chunk index of cb[0]
  uint32_t cb[NB];          // first frame of chunk cc + k
#pragma unroll
  for (uint32_t k = 0; k < NB; ++k) cb[k] = claim();
  auto vframe = [&](uint32_t v) -> uint32_t {  // frame of virtual index v, kNoFrame past the work
    const uint32_t r = v - cc * CH;  // v >= cc * CH
    const uint32_t k = r >> kChLog;
    uint32_t f = kNoFrame;
#pragma unroll
    for (uint32_t i = 0; i < NB; ++i) f = k == i ? cb[i] + (r & (CH - 1)) : f;
    return f < nfb ? f : kNoFrame;
  };

  // ---- per-row cursor (row-uniform VGPRs)
  uint32_t rf = kNoFrame;   // frame index
  uint32_t rea = 0;         // rel(end) rounded up to 4: the window end
  uint32_t rn = 0, rt = 0;  // length, window bytes past the frame end
  uint32_t rJ = 0, rj = 0;  // steps of the frame, next step to issue
  uint32_t nf = 0;          // next unassigned virtual frame of the wave (uniform)

  // ---- ring slots
  Word w[S][KS];
  uint32_t jk[S];             // the word holding the frame end (junk bytes past it)
  uint32_t fi[S], sb[S], eb[S];  // lane i: frame of virtual index nfv[s] + i, its start / end (low dwords)
  uint32_t nfv[S];            // uniform
  uint32_t it_f[S], it_n[S], it_t[S], it_j0[S], it_ns[S];
  uint32_t it_e[S];           // kAppend: rel(end) of the item's frame
  bool hw[S];                 // uniform: slot holds work
#pragma unroll
  for (int s = 0; s < S; ++s) {
#pragma unroll
    for (int k = 0; k < KS; ++k) w[s][k] = 0;
    jk[s] = 0;
    it_f[s] = kNoFrame;
    it_n[s] = it_t[s] = it_j0[s] = it_ns[s] = it_e[s] = 0;
    hw[s] = false;
    nfv[s] = 0;
  }
  // first bounds window for every slot (drained before the loop)
  {
    const uint32_t f = lane < kWin ? vframe(lane) : kNoFrame;
    const uint32_t o = f != kNoFrame ? f * 8u : kOOB;
    uint32_t a = ld_buf<0>(o, off_rsrc);
    uint32_t b = SEG ? ld_buf<0>(f != kNoFrame ? f * 4u : kOOB, cx.len_rsrc) : ld_buf<8>(o, off_rsrc);
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(a), "+v"(b));
#pragma unroll
    for (int s = 0; s < S; ++s) fi[s] = f, sb[s] = a, eb[s] = b;
  }

  uint32_t reg[WL];  // this lane's CRC registers (one per virtual lane) for its row's frame in progress
#pragma unroll
  for (int h = 0; h < WL; ++h) reg[h] = 0;
  int live = 0;      // slots holding work
  // Results are held in registers: lane p of a row holds the row's p-th
  // finished frame (hf) and its result (hv); pc counts them.  A store per
  // slot trickles writes into the read stream, which costs HBM read rate
  // (tools/ubench/cluster.hip: 6 % for 4 B per frame).
  //  * 4-lane rows (up to 16 frames per wave per slot) flush when a row holds
  //    RL results: a store per 4 frames per row (3 % on the Zipf mix).
  //  * 16-lane rows flush at the first slot after each 2^kWinLog ticks
  //    (41 us) of the global 100 MHz clock, or when a row is full.  The
  //    workgroup's waves then write their pieces of each output line within
  //    one slot of each other, so lines are written whole and the chip
  //    writes in bursts (+2.4 % at 1500 B, +1.6 % at 9000 B).  Flushing when
  //    full alone wrote 16-byte pieces of lines at uncorrelated times, and
  //    the partial-line writebacks made it 3 % slower than per-slot stores.
  // VAR 4: one store per slot (A/B); VAR 5: clock windows for 4-lane rows too.
  constexpr bool kHold = VAR != 4;
  constexpr bool kWinFlush = kHold && (RL >= 16 || VAR == 5);
  constexpr int kWinLog = 12;
  uint32_t hf = 0, hv = 0, pc = 0;
  uint32_t he = 0, hpl = 0;  // kAppend: FCS position and new length of the held frame
  uint32_t win = kWinFlush ? (uint32_t)(__builtin_amdgcn_s_memrealtime() >> kWinLog) : 0u;
  auto flush = [&]() {
    if constexpr (MODE == CrcMode::kAppend)
      store_held(cx.ap, p < pc, hf, hv, he, hpl);
    else
      store_result<MODE>(out_rsrc, p < pc, hf, hv);
    pc = 0;
  };

  auto issue = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    // 1. rows that finished their frame take the next frames of the wave, in order
    const bool need = rj >= rJ;
    const uint64_t nmask = __builtin_amdgcn_ballot_w64(need && p == 0);
    const uint64_t below = (1ull << (RL * row)) - 1;
    const uint32_t rank = (uint32_t)__builtin_popcountll(nmask & below);
    const uint32_t cnt = (uint32_t)__builtin_popcountll(nmask);
    const uint32_t li = nf + rank - nfv[s];  // < S*NR by construction
    const uint32_t f = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(li * 4u), (int)fi[s]);
    const uint32_t s_lo = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(li * 4u), (int)sb[s]);
    const uint32_t e_raw = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(li * 4u), (int)eb[s]);
    const uint32_t e_lo = SEG ? s_lo + e_raw : e_raw;  // segment mode: eb holds the length
    if (need) {
      if (f != kNoFrame) {
        const uint32_t len = e_lo - s_lo;
        const uint32_t n = (int32_t)len > 0 ? len : 0u;  // end below start: empty frame
        const uint32_t re = e_lo - o0_lo + adj;
        rf = f;
        rea = (re + kEndAlign - 1u) & ~(kEndAlign - 1u);
        rt = rea - re;
        rn = n;
        rJ = n ? (n + rt + SB - 1) >> kSbLog : 0u;
        rj = 0;
      } else {
        rf = kNoFrame;
        rJ = rj = 0;
      }
    }
    nf += cnt;
    // 2. the item of this slot
    const bool alive = rf != kNoFrame;
    const uint32_t left = rJ - rj;
    const uint32_t ns = alive ? (left < (uint32_t)KS ? left : (uint32_t)KS) : 0u;
    it_f[s] = rf;
    it_n[s] = rn;
    it_t[s] = rt;
    it_e[s] = rea - rt;
    it_j0[s] = rj;
    it_ns[s] = ns;
    hw[s] = wave_any(alive);
    // 3. streaming loads: w[k] = step rj + k from one base (negative for a
    // lead-in before the workgroup's first byte: those words read 0)
    const uint32_t voff = alive ? rea - ((rJ - rj) << kSbLog) + p * 4u * WL : kOOB;
    const bool ends = alive && rj + ns == rJ && rJ != 0;
    // the (virtual) lane whose word holds the frame end, when junk bytes follow it in that word
    const uint32_t jl = kSkip ? VL - 1u - (rt >> 2) : VL - 1u;
    const uint32_t jv = ends && p == jl / WL && (rt & 3u) != 0 ? rea - SB + (jl << 2) : kOOB;
    rj += ns;
    if constexpr (VAR == 2) {
#pragma unroll
      for (int k = 0; k < KS; ++k) {
        if constexpr (WL == 4) {
          const uint32_t z = voff * 0x9E3779B1u + k;
          w[s][k] = u32x4{z, z ^ 1u, z ^ 2u, z ^ 3u};
        } else {
          w[s][k] = (Word)(voff * 0x9E3779B1u + k) * 0x100000001ull;
        }
      }
    } else {
      if constexpr (WL == 4) {
        // four-word 4-lane rows: runs of NSR steps the item has (64-byte row steps)
        ld_item4_ns<0, KS, (int)SB, NSR>(w[s], voff, ns, data_rsrc);
      } else if constexpr (kLine && WL == 1 && EDGE && KS >= 4) {
        // whole-line rows: an item's first step (a frame's first line) and
        // its last two (where a frame's last line lies when its items end on
        // a full one, e.g. 9000 B) at the default cache policy, so the line two
        // frames share is fetched once (lines_body EP = 1); the rest nt
        w[s][0] = ld_buf<0>(voff, data_rsrc);
        ld_item<1, KS - 2, (int)SB, true>(w[s], voff, data_rsrc);
        w[s][KS - 2] = ld_buf<(KS - 2) * (int)SB>(voff, data_rsrc);
        w[s][KS - 1] = ld_buf<(KS - 1) * (int)SB>(voff, data_rsrc);
      } else if constexpr (kLine && WL == 2 && EDGE && KS >= 4) {
        // the same for two-word 16-lane rows (dwordx2 per lane, one line per row)
        ld_x2d<0>(w[s][0], voff, data_rsrc);
        ld_item<1, KS - 2, (int)SB, true>(w[s], voff, data_rsrc);
        ld_x2d<(KS - 2) * (int)SB>(w[s][KS - 2], voff, data_rsrc);
        ld_x2d<(KS - 1) * (int)SB>(w[s][KS - 1], voff, data_rsrc);
      } else if constexpr (!kLine && WL == 1 && NSR > 0) {
        // narrow rows: only the runs the item has (the rest of a short last
        // item would read the next frames' bytes: 4.82 against 4.56 GB of
        // HBM traffic on the Zipf mix, profiles/r2zcf_narrow_load_runs.txt)
        ld_item_ns<0, KS, (int)SB, NSR>(w[s], voff, ns, data_rsrc);
      } else {
        ld_item<0, KS, (int)SB, kLine>(w[s], voff, data_rsrc);
      }
    }
    jk[s] = ld_buf<0>(jv, data_rsrc);
    // 4. bounds of the next S*NR frames, for this slot's next issue
    if (nf >= (cc + 1) * CH) {  // at most one chunk boundary per issue (cnt <= NR <= CH)
      ++cc;
#pragma unroll
      for (uint32_t k = 0; k + 1 < NB; ++k) cb[k] = cb[k + 1];
      cb[NB - 1] = claim();
    }
    const uint32_t g = lane < kWin ? vframe(nf + lane) : kNoFrame;
    const uint32_t go = g != kNoFrame ? g * 8u : kOOB;
    nfv[s] = nf;
    fi[s] = g;
    sb[s] = ld_buf<0>(go, off_rsrc);
    eb[s] = SEG ? ld_buf<0>(g != kNoFrame ? g * 4u : kOOB, cx.len_rsrc) : ld_buf<8>(go, off_rsrc);
  };

  // A slot's frames after its fold, carried over the next issue: the finish
  // (F_p, row XOR, Z_{-t}, store) runs after the slot's next loads are out,
  // so its LDS round trips overlap them instead of idling the wave.
  struct Fin {
    uint32_t reg[WL];
    uint32_t junk, f, n, t, e;
    bool last, any;
  };
  auto compute = [&](auto sc) -> Fin {
    constexpr int s = decltype(sc)::value;
    slot_wait<kPending, KS>(w[s], jk[s], sb[s], eb[s]);
    const uint32_t n = it_n[s], t = it_t[s], ns = it_ns[s], j0 = it_j0[s];
    const uint32_t J = n ? (n + t + SB - 1) >> kSbLog : 0u;
    const bool alive = it_f[s] != kNoFrame;
    const bool first = alive && j0 == 0 && ns != 0;
    const bool last = alive && j0 + ns == J;
    uint32_t keep[WL], initm[WL], m1 = 0;
#pragma unroll
    for (int h = 0; h < WL; ++h) keep[h] = 0xFFFFFFFFu, initm[h] = 0;
    if (first) {
      const uint32_t lead = (J << kSbLog) - n - t;
      const uint32_t m4 = n < 4 ? n : 4u;
#pragma unroll
      for (int h = 0; h < WL; ++h) {
        const int32_t d0 = (int32_t)lead - (int32_t)((p * WL + h) << 2);
        keep[h] = keep_from(d0);
        initm[h] = keep[h] & ~keep_from(d0 + (int32_t)m4);
        reg[h] = 0;
      }
      const int32_t x1 = (int32_t)(lead + m4) - (int32_t)SB;  // init bytes spilling into step 1
      if (x1 > 0 && p == 0) m1 = (uint32_t)((1ull << (8 * x1)) - 1);
    }
    // steps each virtual lane folds: with line windows the junk lanes skip the
    // frame's last step
    uint32_t nsl[WL];
    bool all_full = true, all_near = true;
    // a 1500-byte frame spans 12 or 13 lines and its junk lanes skip one, so
    // a one-item frame's lanes fold KS - 2 .. KS steps: only the last kTail
    // steps need predication
    constexpr int kTail = kLine && KS > 2 ? 2 : KS;
#pragma unroll
    for (int h = 0; h < WL; ++h) {
      nsl[h] = kSkip && last && ns != 0 && p * WL + h >= VL - (t >> 2) ? ns - 1u : ns;
      all_full = all_full && alive && nsl[h] == (uint32_t)KS;
      all_near = all_near && alive && nsl[h] + (uint32_t)kTail >= (uint32_t)KS;
    }
    const bool full = !wave_any(!all_full);
    const bool near = !full && !wave_any(!all_near);
    auto word = [&](int k, int h) -> uint32_t {
      uint32_t x = wsel(w[s][k], h);
      if (k == 0) x = (x & keep[h]) ^ initm[h];
      if (k == 1 && h == 0) x ^= m1;
      return x;
    };
    if constexpr (VAR == 1) {
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int h = 0; h < WL; ++h) reg[h] ^= word(k, h);
    } else {
      if (full) {
        // hot path: every row folds KS steps, no predication; the next word is
        // XOR-ed in by the step's second bitop3
        uint32_t in[WL];
#pragma unroll
        for (int h = 0; h < WL; ++h) in[h] = reg[h] ^ word(0, h);
#pragma unroll
        for (int k = 0; k < KS - 1; ++k)
#pragma unroll
          for (int h = 0; h < WL; ++h) in[h] = u_step_xor(lds, in[h], word(k + 1, h), bu0, bu1);
#pragma unroll
        for (int h = 0; h < WL; ++h) reg[h] = u_step_xor(lds, in[h], 0u, bu0, bu1);
      } else if (kTail < KS && near) {
        uint32_t in[WL];
#pragma unroll
        for (int h = 0; h < WL; ++h) in[h] = reg[h] ^ word(0, h);
#pragma unroll
        for (int k = 0; k < KS - kTail - 1; ++k)
#pragma unroll
          for (int h = 0; h < WL; ++h) in[h] = u_step_xor(lds, in[h], word(k + 1, h), bu0, bu1);
#pragma unroll
        for (int h = 0; h < WL; ++h) reg[h] = u_step_xor(lds, in[h], 0u, bu0, bu1);
#pragma unroll
        for (int k = KS - kTail; k < KS; ++k)
#pragma unroll
          for (int h = 0; h < WL; ++h) {
            const uint32_t r2 = u_step_xor(lds, reg[h] ^ word(k, h), 0u, bu0, bu1);
            reg[h] = (uint32_t)k < nsl[h] ? r2 : reg[h];
          }
      } else {
#pragma unroll
        for (int k = 0; k < KS; ++k)
#pragma unroll
          for (int h = 0; h < WL; ++h) {
            const uint32_t r2 = u_step_xor(lds, reg[h] ^ word(k, h), 0u, bu0, bu1);
            reg[h] = (uint32_t)k < nsl[h] ? r2 : reg[h];
          }
      }
    }
    Fin fin;
#pragma unroll
    for (int h = 0; h < WL; ++h) fin.reg[h] = reg[h];
    fin.junk = jk[s] & ~(uint32_t)(0xFFFFFFFFull >> (8 * (t & 3u)));
    fin.f = it_f[s];
    fin.n = n;
    fin.t = t;
    fin.e = it_e[s];
    fin.last = last;
    fin.any = wave_any(last);
    return fin;
  };
  auto finish = [&](const Fin& fin) {
    uint32_t crc = 0, kpad = 0;
    const uint32_t n = fin.n, t = fin.t;
    if (fin.any) {
      // the lane holding the frame end absorbed t & 3 junk bytes past it: take
      // their U-image out (junk is 0 on every other lane, and U(0) = 0)
      uint32_t R;
      if constexpr (WL == 2) {
        uint32_t r0 = fin.reg[0], r1 = fin.reg[1];
        if (wave_any(fin.junk != 0)) {
          const uint32_t u = u_step(lds, fin.junk, bu0, bu1);
          const bool odd = ((31u - (t >> 2)) & 1u) != 0;  // virtual lane 31 - a is register (31 - a) & 1
          r0 ^= odd ? 0u : u;
          r1 ^= odd ? u : 0u;
        }
        // rows 2m, 2m+1 (lanes 32m .. 32m+31): lane c of the pair applies its
        // own F_c to virtual lane (c - a) mod 32 of each of the two frames
        const auto ts = __builtin_amdgcn_permlane16_swap(t, t, false, false);  // t of row 2m, of row 2m+1
        const uint32_t c = lane & 31u, base = lane & 32u;
        const uint32_t vA = (c - (ts[0] >> 2)) & 31u, vB = (c - (ts[1] >> 2)) & 31u;
        const int sA = (int)((base | (vA >> 1)) << 2), sB = (int)((base | 16u | (vB >> 1)) << 2);
        const uint32_t a0 = (uint32_t)__builtin_amdgcn_ds_bpermute(sA, (int)r0);
        const uint32_t a1 = (uint32_t)__builtin_amdgcn_ds_bpermute(sA, (int)r1);
        const uint32_t b0 = (uint32_t)__builtin_amdgcn_ds_bpermute(sB, (int)r0);
        const uint32_t b1 = (uint32_t)__builtin_amdgcn_ds_bpermute(sB, (int)r1);
        const uint32_t fA = row_xor<16>(f_step(lds, (vA & 1u) ? a1 : a0, bf));
        const uint32_t fB = row_xor<16>(f_step(lds, (vB & 1u) ? b1 : b0, bf));
        // the pair's halves: row 2m gets fA.h0 ^ fA.h1, row 2m+1 fB.h0 ^ fB.h1
        const auto sw = __builtin_amdgcn_permlane16_swap(fA, fB, false, false);
        R = t_fix<16>(lds, sw[0] ^ sw[1], t & 3u, p, bt);
      } else if constexpr (WL == 4) {
        // t = 4a + b window bytes follow the frame end; virtual lane v = 4p + h
        // ends 4((v + a) mod 16) + b bytes past it (lanes v >= 16 - a skipped
        // the last step), so it takes F from column (v + a) mod 16 (+16) of the
        // RL = 16 image, then Z_{-b}.  Pass j applies F to the register h with
        // v + a = j + row (mod 4): the 8 rows of a half-wave use each residue
        // twice, on the two copies (row bit 2), and p spreads the quotient: 32
        // distinct banks.  The b junk bytes sit in virtual lane 15 - a.
        const uint32_t a = t >> 2;
        uint32_t r[4] = {fin.reg[0], fin.reg[1], fin.reg[2], fin.reg[3]};
        if (wave_any(fin.junk != 0)) {
          const uint32_t u = u_step(lds, fin.junk, bu0, bu1);  // zero off the junk lane
          const uint32_t hj = (15u - a) & 3u;
          r[0] ^= hj == 0 ? u : 0u, r[1] ^= hj == 1 ? u : 0u, r[2] ^= hj == 2 ? u : 0u, r[3] ^= hj == 3 ? u : 0u;
        }
        uint32_t acc = 0;
#pragma unroll
        for (uint32_t j = 0; j < 4; ++j) {
          const uint32_t h = (j + row - a) & 3u;
          const uint32_t x = h == 0 ? r[0] : h == 1 ? r[1] : h == 2 ? r[2] : r[3];
          const uint32_t c = ((4u * p + h + a) & 15u) + (((row >> 2) & 1u) << 4);
          acc ^= f_step(lds, x, kFBase | (c << 2));
        }
        R = t_fix<4>(lds, row_xor<4>(acc), t & 3u, p, bt4);
      } else {
        uint32_t r = fin.reg[0];
        if (wave_any(fin.junk != 0)) r ^= u_step(lds, fin.junk, bu0, bu1);
        if constexpr (kLine) {  // lane q takes the register of lane q - a (mod 32) of its row
          const uint32_t src = (row << 5) | ((p - (t >> 2)) & 31u);
          r = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(src << 2), (int)r);
        }
        R = t_fix<RL>(lds, row_xor<RL>(f_step(lds, r, bf)), t & 3u, p, bt);
      }
      R = n != 0 ? R : 0u;
      if (n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * n));
      if constexpr (MODE == CrcMode::kAppend) {
        const bool lv = fin.last && fin.f != kNoFrame;
        if constexpr (kHold)
          R = append_pad<RL, kImg>(lds, Lz, lv, n, R, cx.ap.data_base + fin.e, cx.ap.cap, kpad);
        else  // VAR 4: the FCS, length and status stored at once (A/B)
          append_tail<RL, kImg>(lds, Lz, lv, n, R, cx.ap.data_base + fin.e, cx.ap.cap, cx.ap.lenw + fin.f,
                                cx.ap.stat + fin.f);
      }
      crc = ~R;
    }
    // hold the result; a flush adds a vmcnt event after the slot's loads,
    // which only makes the waits of rows_body stricter
    if constexpr (!kHold) {
      if constexpr (MODE != CrcMode::kAppend)
        store_result<MODE>(out_rsrc, fin.last && p == 0, fin.f, result_of<MODE>(n, crc));
    } else {
      if (fin.last && p == pc) {
        hf = fin.f, hv = result_of<MODE>(n, crc);
        if constexpr (MODE == CrcMode::kAppend) {
          he = fin.e + kpad;
          const uint32_t kf = n < kMinFrame ? kMinFrame - n : 0u;  // the pad the frame needs
          hpl = (uint64_t)n + kf + 4u <= cx.ap.cap ? n + kf + 4u : 0u;
        }
      }
      pc += fin.last ? 1u : 0u;
      bool fl = wave_any(pc == (uint32_t)RL);
      if constexpr (kWinFlush) {
        const uint32_t now = (uint32_t)(__builtin_amdgcn_s_memrealtime() >> kWinLog);
        fl = fl || (now != win && wave_any(pc != 0));
        win = now;
      }
      if (fl) flush();
    }
  };

#define LNX_FENCE __builtin_amdgcn_sched_barrier(0)
  bool done = false;
  auto slot = [&](auto sc) {
    constexpr int s = decltype(sc)::value;
    if (done) return;
    const Fin fin = compute(sc);
    live -= hw[s] ? 1 : 0;
    const bool more = vframe(nf) != kNoFrame || wave_any(rj < rJ);
    if (live == 0 && !more) {
      done = true;
      finish(fin);
      return;
    }
    LNX_FENCE;
    issue(sc);
    LNX_FENCE;
    finish(fin);
    live += hw[s] ? 1 : 0;
  };
  while (!done) {
    [&]<int... I>(std::integer_sequence<int, I...>) {
      (slot(std::integral_constant<int, I>{}), ...);
    }(std::make_integer_sequence<int, S>{});
  }
#undef LNX_FENCE
  // the slots that held no work at the end still issued their (out-of-range)
  // loads: retire them before the flush reuses registers (audit_ring.py)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (kHold && wave_any(pc != 0)) flush();
  // drain: no asm load may still be writing registers when the wave ends
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------ lean line rows
// Two-word 16-lane rows (buffer_load_dwordx2 nt: each row instruction reads one
// whole 128-byte line) with the per-slot bookkeeping cut to what frames of up
// to KS lines need (DESIGN.md §3.1 "lean line rows").  rows_body spends
// ~130-160 VALU per wave-slot on item cursors, ballot ranks, bounds windows and
// multi-chunk frame lookups (PMC: 82 VALU per 1500-B frame for one-word rows,
// 117 for two-word rows); here:
//  * a chunk is exactly one slot: CH = 4 frames, one per row, claimed from the
//    LDS counter two slots ahead; its 5 offsets arrive in lanes 0..4 one slot
//    ahead and reach the rows with two ds_bpermute;
//  * every row folds its whole frame in the slot: window = the lines holding
//    the frame (J = 1..KS of them), loads from the window start, the last two
//    steps predicated (frames of J = KS - 1 or KS lines, e.g. 1500 B at any
//    alignment with KS = 13); any other J predicates every step, and frames of
//    more than KS lines take further items inside the slot (correct, slower);
//  * no register rotation: virtual lane v's register ends 4((v + a) mod 32) + b
//    bytes past the frame end (t = 4a + b window bytes follow it), so it takes
//    F_{(v+a) mod 32} straight from that column of the RL = 32 image.  A lane
//    applies F to its two registers in two instructions; which register goes
//    first is chosen per row so that the 32 lanes of two rows always read 32
//    distinct banks (rows 2m and 2m+1 differ in column parity).  One row XOR
//    of the two F results, then Z_{-b}.
//
// WL = 1 runs the same slot structure on 32-lane rows (one dword per lane,
// two frames per wave): lane p is virtual lane p, its register takes F from
// column (p + a) mod 32, and the row XOR spans the 32 lanes.
// SEG: segment mode (frame i = bytes[start[i] : start[i] + len[i]], in address
// order, not overlapping: ring slots, lnx_crc32_segments / the TX FCS append):
// lanes 0..3 load the chunk's starts and lengths instead of five offsets.
template <CrcMode MODE, int KS, int VAR, int WL = 2, bool JM = true, int EP = 0, bool SEG = false>
__device__ __forceinline__ void lines_body(const char* lds, const Lanes& L, const WaveCtx& cx) {
  static_assert(WL == 1 || WL == 2, "words per lane");
  constexpr uint32_t RL = 32 / WL;  // lanes per row
  constexpr uint32_t CH = 64 / RL;  // frames per chunk = rows per wave
  using Word = std::conditional_t<WL == 2, uint64_t, uint32_t>;
  static_assert(KS >= 4 && (KS - 1) * 128 <= 4095, "item shape");
  const uint32_t lane = L.lane, p = L.p, row = L.row, bu0 = L.bu0, bu1 = L.bu1, bt = L.bt;
  const uint32_t nfb = cx.nfb, o0_lo = cx.o0_lo, adj = cx.adj;
  const __amdgpu_buffer_rsrc_t data_rsrc = cx.data_rsrc, off_rsrc = cx.off_rsrc, out_rsrc = cx.out_rsrc;

  // a claim's result stays in lane 0's VGPR until the next slot reads it
  // (readfirstlane), so the wave never waits on the LDS atomic's latency
  auto claim = [&]() -> uint32_t {
    uint32_t b = 0;
    if (lane == 0) b = __hip_atomic_fetch_add(cx.ctr, CH, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    return b;
  };
  auto uni = [](uint32_t v) -> uint32_t { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); };
  // lane i < 5: low dword of off[b + i] (the range's offsets array has nfb + 1
  // entries); SEG: lane i < 4 the low dword of start[b + i], and in bl len[b + i]
  uint32_t bl = 0;
  auto ld_bounds = [&](uint32_t b) -> uint32_t {
    if constexpr (SEG) {
      const bool in = b + lane < nfb && lane < CH;
      bl = ld_buf<0>(in ? (b + lane) * 4u : kOOB, cx.len_rsrc);
      return ld_buf<0>(in ? (b + lane) * 8u : kOOB, off_rsrc);
    } else {
      return ld_buf<0>(b < nfb && lane <= CH ? (b + lane) * 8u : kOOB, off_rsrc);
    }
  };

  // row-uniform parameters of the frame in progress
  struct Rowp {
    uint32_t f, n, t, J, ws, e;
  };
  auto setup = [&](uint32_t b, uint32_t bd) -> Rowp {
    Rowp r;
    const uint32_t s = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(row << 2), (int)bd);
    const uint32_t e = SEG ? s + (uint32_t)__builtin_amdgcn_ds_bpermute((int)(row << 2), (int)bl)
                           : (uint32_t)__builtin_amdgcn_ds_bpermute((int)((row + 1) << 2), (int)bd);
    const uint32_t f = b + row;
    const uint32_t len = e - s;
    r.f = f < nfb ? f : kNoFrame;
    r.n = f < nfb && (int32_t)len > 0 ? len : 0u;  // end below start: empty frame
    const uint32_t rs = s - o0_lo + adj, re = e - o0_lo + adj;
    const uint32_t wend = (re + 127u) & ~127u;
    r.ws = rs & ~127u;
    r.e = re;
    r.t = wend - re;
    r.J = r.n ? (wend - r.ws) >> 7 : 0u;
    return r;
  };

  // wave-uniform min (over rows with lines) and max of a row-uniform J
  auto wave_min_max = [&](uint32_t J, uint32_t& jmin, uint32_t& jmax) {
    jmin = ~0u, jmax = 0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if ((uint32_t)r >= CH) break;
      const uint32_t x = (uint32_t)__builtin_amdgcn_readlane((int)J, (int)RL * r);
      jmax = x > jmax ? x : jmax;
      jmin = x != 0 && x < jmin ? x : jmin;
    }
  };

  Word w[KS];
  uint32_t jk = 0;
  // runs of up to six step loads; a run no row of the wave reaches loads from
  // an out-of-range offset (no memory traffic).  Always issued: an asm load
  // under a branch makes hipcc merge its output with the old value by copies
  // placed before the ring's wait (tools/prof/audit_ring.py caught that).
  // Cache policy of the step loads (two words per lane).  Consecutive frames
  // share a line (the one holding the frame boundary), and a wave's four rows
  // fold four consecutive frames, so most shared lines are asked for twice
  // within one slot; the first and last chunks' shared lines are asked for by
  // two different waves.  With non-temporal loads the line is gone from L2 by
  // the second request and HBM serves it twice.
  //   EP = 0: every step nt (r1);
  //   EP = 1: the first step and the last two steps (where a frame's last line
  //           lies) with the default policy, the middle steps nt (product);
  //   EP = 2: only the first step with the default policy;
  //   EP = 3: every step with the default policy.
  constexpr bool kEdge = (EP == 1 || EP == 2) && WL == 2;
  constexpr bool kTail = EP == 1 && WL == 2;
  constexpr bool kAllDef = EP == 3 && WL == 2;
  auto ld_runs = [&]<int K0>(auto self, std::integral_constant<int, K0>, uint32_t voff, uint32_t jmax) {
    if constexpr (kAllDef && K0 < KS - 1) {
      if constexpr (WL == 2) ld_x2d<K0 * 128>(w[K0], (uint32_t)K0 < jmax ? voff : kOOB, data_rsrc);
      self(self, std::integral_constant<int, K0 + 1>{}, voff, jmax);
    } else if constexpr (kAllDef) {
    } else if constexpr (kEdge && K0 == 0) {
      if constexpr (WL == 2) ld_x2d<0>(w[0], voff, data_rsrc);
      self(self, std::integral_constant<int, 1>{}, voff, jmax);
    } else if constexpr (kTail && K0 == KS - 2) {
      if constexpr (WL == 2) ld_x2d<(KS - 2) * 128>(w[KS - 2], (uint32_t)K0 < jmax ? voff : kOOB, data_rsrc);
    } else if constexpr (K0 < KS - 1) {
      constexpr int KE = kTail ? KS - 2 : KS - 1;  // end of this run of nt loads
      constexpr int N = KE - K0 < 6 ? KE - K0 : 6;
      if constexpr (WL == 2)
        ld_run2<K0 * 128, N, 128>(w + K0, (uint32_t)K0 < jmax ? voff : kOOB, data_rsrc);
      else
        ld_run<K0 * 128, N, 128, true>(w + K0, (uint32_t)K0 < jmax ? voff : kOOB, data_rsrc);
      self(self, std::integral_constant<int, K0 + N>{}, voff, jmax);
    }
  };
  auto issue = [&](const Rowp& r) {
    const uint32_t voff = r.J ? r.ws + p * (4u * WL) : kOOB;
    if constexpr (VAR == 2) {
#pragma unroll
      for (int k = 0; k < KS; ++k) w[k] = (Word)((uint64_t)(voff * 0x9E3779B1u + k) * 0x100000001ull);
    } else {
      uint32_t jmin, jmax;
      wave_min_max(r.J, jmin, jmax);
      ld_runs(ld_runs, std::integral_constant<int, 0>{}, voff, jmax);
      // the last step from its own offset: out of range unless the frame has
      // KS lines (a 1500-B frame spans 12 lines at 29 % of start alignments;
      // the 13th line belongs to the next frame and would be fetched twice)
      if constexpr (kTail || kAllDef)
        ld_x2d<(KS - 1) * 128>(w[KS - 1], r.J >= (uint32_t)KS ? voff : kOOB, data_rsrc);
      else if constexpr (WL == 2)
        ld_run2<(KS - 1) * 128, 1, 128>(w + KS - 1, r.J >= (uint32_t)KS ? voff : kOOB, data_rsrc);
      else
        ld_run<(KS - 1) * 128, 1, 128, true>(w + KS - 1, r.J >= (uint32_t)KS ? voff : kOOB, data_rsrc);
    }
    // JM = false: the word holding the frame end, when junk bytes follow it
    // there (virtual lane 31 - a), loaded once more for the finish to take
    // its U-image out.  JM = true masks those bytes in the fold instead (r2:
    // 0.2521 -> 0.2465 ms at 1500 B, profiles/r2b_var_mtu1500.log).
    if constexpr (!JM) {
      const uint32_t jl = 31u - (r.t >> 2);
      const bool jn = r.J != 0 && p == jl / WL && (r.t & 3u) != 0;
      jk = ld_buf<0>(jn ? r.ws + ((r.J - 1u) << 7) + (jl << 2) : kOOB, data_rsrc);
    }
  };

  // VAR 7 (kAppend, two-word rows; A/B, not the product): the FCS is written
  // with the whole 64-byte sector that holds it (the frame's last line is in
  // the lanes' registers: the bytes before the FCS are the frame's, the ones
  // after it the slot's, rewritten as loaded).  In tools/ubench/scatter_write.hip
  // whole-sector writes cost a read stream +24 % against +33 % for a dword; in
  // this kernel they measured 2 % slower than the held dword
  // (profiles/r3j_fcs_append_sector_ab.txt): every TCC write request became a
  // 64-byte one, and the time per write stayed.
  constexpr bool kSector = MODE == CrcMode::kAppend && WL == 2 && VAR == 7;
  struct Fin {
    uint32_t r0, r1, junk, f, n, t, e;
    uint64_t tl;  // kSector: this lane's 8 bytes of the frame's last line
  };
  auto fold = [&](const Rowp& r) -> Fin {
    const uint32_t n = r.n, t = r.t, J = r.J, a = t >> 2;
    const uint32_t lead = (r.J ? (J << 7) - n - t : 0u);
    const uint32_t m4 = n < 4 ? n : 4u;
    // step 0: the lane's 8 bytes keep [lead - 8p, 8) and take the init 0xFF
    // over [lead - 8p, lead - 8p + m4); bytes [d, 8) of a qword are
    // (~0 << 4d) << 4d for d in 0..8 (two shifts: a 64-bit shift by 64 is 0)
    auto keep8 = [](int32_t d) -> uint64_t {
      const uint32_t q = 4u * (uint32_t)(d < 0 ? 0 : (d > 8 ? 8 : d));
      return (~0ull << q) << q;
    };
    const int32_t d0 = (int32_t)lead - (int32_t)(p * 4u * WL);
    Word w0;
    if constexpr (WL == 2) {
      const uint64_t keep = keep8(d0), initm = keep & ~keep8(d0 + (int32_t)m4);
      w0 = (w[0] & keep) ^ initm;
    } else {
      const uint32_t keep = keep_from(d0), initm = keep & ~keep_from(d0 + (int32_t)m4);
      w0 = (w[0] & keep) ^ initm;
    }
    uint32_t nsl[WL];
#pragma unroll
    for (int h = 0; h < WL; ++h) nsl[h] = J ? J - (WL * p + h >= 32u - a ? 1u : 0u) : 0u;
    const int32_t x1 = (int32_t)(lead + m4) - 128;  // init bytes spilling into step 1
    const uint32_t m1 = x1 > 0 && p == 0 ? (uint32_t)((1ull << (8 * x1)) - 1) : 0u;
    auto word = [&](int k, int h) -> uint32_t {
      uint32_t x = (uint32_t)((uint64_t)(k == 0 ? w0 : w[k]) >> (32 * h));
      if (k == 1 && h == 0) x ^= m1;
      return x;
    };
    // JM: the frame's last step J - 1 keeps only the frame's bytes of virtual
    // lane 31 - a's word (its top t & 3 bytes belong to the next frame)
    uint32_t jm[WL];
#pragma unroll
    for (int h = 0; h < WL; ++h)
      jm[h] = JM && WL * p + h == 31u - a ? (uint32_t)(0xFFFFFFFFull >> (8 * (t & 3u))) : 0xFFFFFFFFu;
    const uint32_t jlast = J - 1u;
    auto wordj = [&](int k, int h) -> uint32_t {  // word(k, h) in a step that may be the frame's last
      const uint32_t x = word(k, h);
      return JM ? x & ((uint32_t)k == jlast ? jm[h] : 0xFFFFFFFFu) : x;
    };
    uint32_t reg[WL] = {};
    uint64_t tl = 0;  // kSector: step J - 1's 8 bytes of this lane
    if constexpr (VAR == 1) {
#pragma unroll
      for (int k = 0; k < KS; ++k)
#pragma unroll
        for (int h = 0; h < WL; ++h) reg[h] ^= word(k, h);
    } else {
      // fast: every row's frame spans KS - 1 or KS lines (or none)
      const bool fast = !wave_any(J != 0 && J + 1u < (uint32_t)KS) && !wave_any(J > (uint32_t)KS);
      if (fast) {
        uint32_t in[WL];
#pragma unroll
        for (int h = 0; h < WL; ++h) in[h] = word(0, h);
#pragma unroll
        for (int k = 0; k < KS - 3; ++k)
#pragma unroll
          for (int h = 0; h < WL; ++h) in[h] = u_step_xor(lds, in[h], word(k + 1, h), bu0, bu1);
#pragma unroll
        for (int h = 0; h < WL; ++h) reg[h] = u_step_xor(lds, in[h], 0u, bu0, bu1);
#pragma unroll
        for (int k = KS - 2; k < KS; ++k)
#pragma unroll
          for (int h = 0; h < WL; ++h) {
            const uint32_t r2 = u_step_xor(lds, reg[h] ^ wordj(k, h), 0u, bu0, bu1);
            reg[h] = (uint32_t)k < nsl[h] ? r2 : reg[h];
          }
        if constexpr (kSector) tl = (uint64_t)(J == (uint32_t)KS ? w[KS - 1] : w[KS - 2]);
      } else {
        // any J: step k is skipped when no row has k lines, unpredicated while
        // every row with lines has more than k + 1, predicated otherwise
        // (wave-uniform branches; the junk lanes skip their row's last step)
        uint32_t jmin, jmax;
        wave_min_max(J, jmin, jmax);
#pragma unroll
        for (int k = 0; k < KS; ++k) {
          if ((uint32_t)k >= jmax) continue;  // (no break: the loop must stay unrolled)
          if constexpr (kSector) tl = (uint32_t)k + 1u == J ? (uint64_t)w[k] : tl;
          if ((uint32_t)k + 1u < jmin) {
#pragma unroll
            for (int h = 0; h < WL; ++h) reg[h] = u_step_xor(lds, reg[h] ^ word(k, h), 0u, bu0, bu1);
          } else {
#pragma unroll
            for (int h = 0; h < WL; ++h) {
              const uint32_t r2 = u_step_xor(lds, reg[h] ^ wordj(k, h), 0u, bu0, bu1);
              reg[h] = (uint32_t)k < nsl[h] ? r2 : reg[h];
            }
          }
        }
        // frames of more than KS lines: further items, loaded and folded in turn
        // (six lines at a time: rare, latency-bound, kept small in registers)
        constexpr int KX = 6;
        for (uint32_t j0 = KS; wave_any(j0 < J); j0 += KX) {
          // a separate array: reloading w here would give the ring registers
          // two definitions and hipcc copies between them at the loop head,
          // before the ring's wait
          Word wx[KX];
          const uint32_t voff = j0 < J ? r.ws + (j0 << 7) + p * (4u * WL) : kOOB;
          ld_item<0, KX, 128, true>(wx, voff, data_rsrc);  // (uint32_t: ld_run nt, uint64_t: ld_run2)
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
          for (int k = 0; k < KX; ++k) asm volatile("" : "+v"(wx[k]));
#pragma unroll
          for (int k = 0; k < KX; ++k) {
            if constexpr (kSector) tl = j0 + (uint32_t)k + 1u == J ? (uint64_t)wx[k] : tl;
          }
#pragma unroll
          for (int k = 0; k < KX; ++k)
#pragma unroll
            for (int h = 0; h < WL; ++h) {
              uint32_t x = (uint32_t)((uint64_t)wx[k] >> (32 * h));
              if (JM) x &= j0 + (uint32_t)k == jlast ? jm[h] : 0xFFFFFFFFu;
              const uint32_t r2 = u_step_xor(lds, reg[h] ^ x, 0u, bu0, bu1);
              reg[h] = j0 + (uint32_t)k < nsl[h] ? r2 : reg[h];
            }
        }
      }
    }
    Fin fin;
    fin.r0 = reg[0];
    fin.r1 = WL == 2 ? reg[WL - 1] : 0u;
    fin.junk = jk & ~(uint32_t)(0xFFFFFFFFull >> (8 * (t & 3u)));
    fin.f = r.f;
    fin.n = n;
    fin.t = t;
    fin.e = r.e;
    fin.tl = tl;
    return fin;
  };

  // results held in registers, flushed in clock windows (as rows_body)
  constexpr int kWinLog = 12;
  uint32_t hf = 0, hv = 0, pc = 0;
  uint32_t he = 0, hpl = 0;  // kAppend (store_held)
  uint32_t win = (uint32_t)(__builtin_amdgcn_s_memrealtime() >> kWinLog);
  auto finish = [&](const Fin& fin) {
    const uint32_t n = fin.n, t = fin.t, a = t >> 2;
    const bool live = fin.f != kNoFrame;
    uint32_t R;
    if constexpr (WL == 2) {
      uint32_t r0 = fin.r0, r1 = fin.r1;
      if (!JM && wave_any(fin.junk != 0)) {
        const uint32_t u = u_step(lds, fin.junk, bu0, bu1);
        const bool odd = ((31u - a) & 1u) != 0;  // virtual lane 31 - a is register (31 - a) & 1
        r0 ^= odd ? 0u : u;
        r1 ^= odd ? u : 0u;
      }
      // register h of lane p (virtual lane 2p + h) takes F_q, q = (2p + h + a) mod 32;
      // the odd row of each pair goes first with the register whose column
      // parity differs from the even row's
      const auto as = __builtin_amdgcn_permlane16_swap(a, a, false, false);  // a of row 2m, of row 2m+1
      const uint32_t hs = (row & 1u) ? (((as[0] ^ as[1]) & 1u) ^ 1u) : 0u;
      const uint32_t x1 = hs ? r1 : r0, x2 = hs ? r0 : r1;
      const uint32_t q1 = (2u * p + hs + a) & 31u, q2 = (2u * p + (hs ^ 1u) + a) & 31u;
      const uint32_t F = f_step(lds, x1, kFBase | (q1 << 2)) ^ f_step(lds, x2, kFBase | (q2 << 2));
      R = t_fix<16>(lds, row_xor<16>(F), t & 3u, p, bt);
    } else {
      // lane p (virtual lane p) takes F_q, q = (p + a) mod 32: 32 distinct
      // columns per row, and the two rows sit in different halves of the wave
      uint32_t r0 = fin.r0;
      if (!JM && wave_any(fin.junk != 0)) r0 ^= u_step(lds, fin.junk, bu0, bu1);
      R = t_fix<32>(lds, row_xor<32>(f_step(lds, r0, kFBase | (((p + a) & 31u) << 2))), t & 3u, p, bt);
    }
    R = n != 0 ? R : 0u;
    if (n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * n));
    uint32_t kpad = 0;
    if constexpr (MODE == CrcMode::kAppend && VAR == 4) {  // the FCS, length and status stored at once (A/B)
      append_tail<WL == 2 ? 16 : 32, 32>(lds, L, live, n, R, cx.ap.data_base + fin.e, cx.ap.cap, cx.ap.lenw + fin.f,
                                         cx.ap.stat + fin.f);
      return;
    } else if constexpr (MODE == CrcMode::kAppend) {
      R = append_pad<WL == 2 ? 16 : 32, 32>(lds, L, live, n, R, cx.ap.data_base + fin.e, cx.ap.cap, kpad);
    }
    const uint32_t crc = ~R;
    bool sec = false;  // kSector: this row's FCS went out with its sector
    if constexpr (kSector) {
      // the sector [e & ~63, + 64) (rel and absolute alignment agree: the
      // range base is line-aligned) when it holds the whole FCS (e mod 64 in
      // 1..60: then it lies inside the frame's last line, e mod 128 != 0), lies
      // in the frame's slot ([start, start + cap), start = e - n) and inside the
      // range's bytes (the range's last frame: bytes past its end read as 0)
      const uint32_t em = fin.e & 63u;
      sec = live && kpad == 0 && em - 1u < 60u && (uint64_t)n + 64u - em <= cx.ap.cap &&
            fin.e - em + 64u <= cx.ap.rend;
      if (wave_any(sec)) {
        const uint32_t l0 = fin.e & ~127u, pc0 = l0 + 8u * p;  // this lane's piece of the last line
        const int32_t d = (int32_t)(fin.e - pc0);               // FCS byte 0 at piece byte d
        const uint64_t c64 = crc;
        const uint64_t m = d >= 0 ? (d < 8 ? 0xFFFFFFFFull << (8 * d) : 0ull)
                                  : (d > -4 ? 0xFFFFFFFFull >> (-8 * d) : 0ull);
        const uint64_t fv = d >= 0 ? (d < 8 ? c64 << (8 * d) : 0ull) : (d > -4 ? c64 >> (-8 * d) : 0ull);
        if (sec && pc0 - (fin.e - em) < 64u)
          *reinterpret_cast<uint64_t*>(cx.ap.data_base + pc0) = (fin.tl & ~m) | (fv & m);
      }
    }
    if (live && p == pc) {
      hf = fin.f, hv = result_of<MODE>(n, crc);
      if constexpr (MODE == CrcMode::kAppend) {
        he = sec ? kFcsWritten : fin.e + kpad;
        const uint32_t kf = n < kMinFrame ? kMinFrame - n : 0u;  // the pad the frame needs
        hpl = (uint64_t)n + kf + 4u <= cx.ap.cap ? n + kf + 4u : 0u;
      }
    }
    pc += live ? 1u : 0u;
    bool fl = wave_any(pc == RL);
    const uint32_t now = (uint32_t)(__builtin_amdgcn_s_memrealtime() >> kWinLog);
    fl = fl || (now != win && wave_any(pc != 0));
    win = now;
    if (fl) {
      if constexpr (MODE == CrcMode::kAppend)
        store_held(cx.ap, p < pc, hf, hv, he, hpl);
      else
        store_result<MODE>(out_rsrc, p < pc, hf, hv);
      pc = 0;
    }
  };

  const uint32_t c0 = uni(claim());
  uint32_t bd = ld_bounds(c0);
  asm volatile("s_waitcnt vmcnt(0)" : "+v"(bd), "+v"(bl));
  if (c0 >= nfb) return;
  uint32_t c1 = uni(claim());
  Rowp cur = setup(c0, bd);
  issue(cur);
  bd = ld_bounds(c1);
  uint32_t c2v = claim();
#define LNX_FENCE __builtin_amdgcn_sched_barrier(0)
  for (;;) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int k = 0; k < KS; ++k) asm volatile("" : "+v"(w[k]));
    asm volatile("" : "+v"(jk), "+v"(bd), "+v"(bl));
    const Fin fin = fold(cur);
    if (c1 >= nfb) {
      finish(fin);
      break;
    }
    LNX_FENCE;
    cur = setup(c1, bd);
    issue(cur);
    c1 = uni(c2v);
    bd = ld_bounds(c1);
    c2v = claim();
    LNX_FENCE;
    finish(fin);
  }
#undef LNX_FENCE
  // the loop leaves through a tail hipcc may share with the issue path: no
  // load is outstanding here, but the explicit wait lets the linear ISA audit
  // (tools/prof/audit_ring.py) see that before the epilogue reuses registers
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (wave_any(pc != 0)) {
    if constexpr (MODE == CrcMode::kAppend)
      store_held(cx.ap, p < pc, hf, hv, he, hpl);
    else
      store_result<MODE>(out_rsrc, p < pc, hf, hv);
  }
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
}

// ------------------------------------------------------------------ kernel
// Row width per workgroup from its frames' mean length (RLF = 0): 4-lane rows
// below kShortMean, 32-lane rows from kLineMean on, 16-lane rows with MIDW
// words per lane between; or forced (RLF = 4 / 16 / 32, profiling).  Item
// size, ring depth and chunk: KSW, SW, CHW for 32-lane rows, KSM, SM, CHM
// for 16-lane rows, KS4, S4, CH4 for 4-lane rows.
//
// 32-lane rows and 16-lane rows of two words per lane both read whole lines
// with nt loads (loads alone: 6.4 TB/s at 1500 B against 6.0 for one-word
// 16-lane rows), and both win at 9000 B (6.70 / 6.74 TB/s against 6.14).  At
// 1500 B (one 13-line item per frame) their per-frame finish costs more:
// 32-lane rows finish 2 frames per wave-slot where 16-lane rows finish 4
// (VALU-bound, 4.9 TB/s), and two-word rows apply F to 32 registers per frame
// (5.7-5.8 TB/s against 5.9 for one-word rows).  So MIDW = 1 in the product
// (profiles/r1f_line_rows_variants.txt).
constexpr uint64_t kLineMean = 4096;
// Lean line rows (lines_body) from kShortMean up to this mean frame length
// (MIDW = 4): one frame per row per slot needs frames of at most KSL lines.
constexpr uint64_t kLeanMean = 1600;
#ifdef LNX_RESEARCH  // the losing short-frame designs: research library only
#include "research/stream_rows.hpp"
#include "research/stream_lanes.hpp"
#endif

template <CrcMode MODE, int VAR = 0, int RLF = 0, int KSW = 24, int SW = 1, int KS4 = 16, int S4 = 2,
          int CHW = 4, int CH4 = 32, bool SEG = false, int MIDW = 4, int KSM = 24, int SM = 1, int CHM = 4,
          int KSL = 13, int LWL = 2, bool LJM = true, int LEP = 1, bool REDGE = true, int NSR4 = 4, int NW4 = 1,
          int STR = 0>
__global__ void __launch_bounds__(kBlockThreads, 1)
crc32_rows_kernel(const uint8_t* bytes,  /* not __restrict__: kAppend writes the FCS through it */ const uint64_t* __restrict__ off, uint64_t nframes,
                  uint64_t frames_per_wave, const uint4* __restrict__ images, void* __restrict__ out,
                  uint64_t* __restrict__ timeline,
                  const uint32_t* seg_len, uint32_t cap, uint32_t policy, uint32_t* __restrict__ stage_flag,
                  uint32_t epoch) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[kLdsDwords];
  // profiling (tools/prof/timeline.py): per wave, 100 MHz clock at entry,
  // after the LDS image copy and at exit; null in the product path
  const uint64_t t_entry = timeline ? __builtin_amdgcn_s_memrealtime() : 0;
  const uint64_t per_block = frames_per_wave * kWavesPerBlock;
  const uint64_t fb0 = (uint64_t)blockIdx.x * per_block < nframes ? (uint64_t)blockIdx.x * per_block : nframes;
  const uint64_t fb1 = fb0 + per_block < nframes ? fb0 + per_block : nframes;
  // the plain entries launch this kernel and the staged one over the same
  // slices (dispatch.hpp): a slice that is not the rows kernel's exits here
  // slices: the staged launch behind this one reads one word before anything
  // else and exits at once unless some workgroup here stored this call's
  // epoch there (its slice is the staged kernel's, or giant)
  if (!SEG && policy != kPolicyRows) {
    const uint32_t kind = slice_kind(bytes, off, fb0, fb1, policy, batch_mean(off, nframes));
    if (kind != kSliceRows) {
      if (kind != kSliceNone && stage_flag && threadIdx.x == 0) *stage_flag = epoch;
      return;
    }
  }
  // byte bounds of frames [f0, f1): offsets mode off[f0], off[f1]; segment
  // mode (frames in address order, not overlapping) start[f0], end of f1 - 1
  auto lo_of = [&](uint64_t f0, uint64_t f1) -> uint64_t { return SEG ? (f1 > f0 ? off[f0] : 0) : off[f0]; };
  auto hi_of = [&](uint64_t f0, uint64_t f1) -> uint64_t {
    return SEG ? (f1 > f0 ? off[f1 - 1] + seg_len[f1 - 1] : 0) : off[f1];
  };
  const uint64_t ob0 = lo_of(fb0, fb1), ob1 = hi_of(fb0, fb1);
  // Segment mode: the pipelined rows address the slice's frames relative to
  // its first start and store the TX tail through that base, so they need the
  // slice in address order without overlap, start[i] + len[i] <= start[i + 1].
  // A slice that is not (any order is legal at the C-ABI) takes the per-frame
  // path below, which addresses every frame from its own 64-bit start.  The
  // check's loads overlap the LDS image copy; its verdict is combined through
  // LDS after the image's barrier.  (A wave-uniform trip count: the audit's
  // loop rule)
  bool seg_bad = false;
  if constexpr (SEG) {
    for (uint64_t i0 = fb0; i0 < fb1; i0 += kBlockThreads) {  // (clamped indices: no branch, every lane loads)
      const uint64_t i = i0 + threadIdx.x < fb1 ? i0 + threadIdx.x : fb1 - 1;
      const uint64_t s = off[i], e = s + seg_len[i], o1 = off[i + 1 < fb1 ? i + 1 : i];
      seg_bad = seg_bad || (i + 1 < fb1 && e > o1);
    }
  }
  int rl = RLF;
  // MIDW (16-lane rows): 1 = one word per lane, 2 = two words, 3 = lean line
  // rows, 4 = lean line rows below kLeanMean, one word per lane above
  // (24-line lean items for 1600-3000 B were tried: w[24] pushed the kernel
  // past its VGPR budget into scratch)
  bool lean = MIDW == 3;
  if constexpr (RLF == 0) {
    const uint64_t nf_ = fb1 - fb0, nb_ = ob1 > ob0 ? ob1 - ob0 : 0;
    rl = nf_ == 0 || nb_ < kShortMean * nf_ ? 4 : nb_ < kLineMean * nf_ ? 16 : 32;
    if (MIDW == 4) lean = rl == 16 && nb_ < kLeanMean * nf_;
  }
  const bool narrow = rl == 4;
  // whole-line windows: the RL = 32 image
  const bool line = rl == 32 || (rl == 16 && (MIDW == 2 || lean));
  // streaming rows (research/stream_rows.hpp) for the narrow rows' frames in offsets
  // mode, when the slice's bytes fit 31-bit buffer offsets from a line-aligned base
  bool strm = STR != 0 && narrow && !SEG && MODE != CrcMode::kAppend;
  if (strm) {
    const uint64_t nb_ = ob1 > ob0 ? ob1 - ob0 : 0;
    const uint64_t adj_ = (reinterpret_cast<uintptr_t>(bytes) + ob0) & 127u;
    strm = nb_ + adj_ + 4096 < (1ull << 31);
  }
  {
    // compact image (lds_layout.hpp): thread t expands U value t into its 32
    // bank replicas (128 contiguous bytes, eight 16-byte writes started at a
    // lane-rotated position so the wave's writes spread over the banks), then
    // the F/T tail is copied verbatim; it is zero at kCtrBase, which starts
    // the chunk counter at 0
    static_assert(kCompactUDwords == kBlockThreads, "one U value per thread");
    // (4-lane rows of four words per lane fold 16 virtual lanes: the RL = 16 image)
    const uint32_t* img = reinterpret_cast<const uint32_t*>(images) +
                          image_index(strm ? (STR == 3 ? 10 : STR == 2 ? 9 : 8) : line ? 32 : (narrow && NW4 == 4) ? 16 : rl) *
                              kCompactDwords;
    const uint32_t t = threadIdx.x;
    const uint32_t uv = img[t];
    const uint4* tail = reinterpret_cast<const uint4*>(img + kCompactUDwords);
    constexpr int kTail = (int)((kLdsBytes - kFBase) / 16 / kBlockThreads);
    uint4 tv[kTail];
#pragma unroll
    for (int i = 0; i < kTail; ++i) tv[i] = tail[t + i * kBlockThreads];
    uint4* urow = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds_words) + u_addr(t >> 8, t & 255u, 0));
    const uint4 u4 = {uv, uv, uv, uv};
#pragma unroll
    for (int i = 0; i < 8; ++i) urow[(i + t) & 7u] = u4;
    uint4* l4 = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds_words) + kFBase);
#pragma unroll
    for (int i = 0; i < kTail; ++i) l4[t + i * kBlockThreads] = tv[i];
  }

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t col = lane & 31u;
  Lanes L;
  L.lane = lane;
  L.bu0 = col << 2;
  L.bu1 = L.bu0 | 65536u;
  L.bf = kFBase | (col << 2);
  L.bt = kTBase | (col << 2);
  const uint64_t gwave = (uint64_t)blockIdx.x * kWavesPerBlock + __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  __syncthreads();
  if constexpr (SEG) {
    // any thread's frame out of order: the whole slice per frame (a spare
    // dword of the image's zero tail, past the chunk counter)
    uint32_t* flag = lds_words + kCtrBase / 4 + 16;
    if (__builtin_amdgcn_ballot_w64(seg_bad) != 0 && (threadIdx.x & 63u) == 0) *flag = 1u;
    __syncthreads();
    seg_bad = __builtin_amdgcn_readfirstlane((int)*flag) != 0;  // (uniform: keeps the branch scalar)
  }
  const char* lds = reinterpret_cast<const char*>(lds_words);
  uint64_t* tl = nullptr;
  if (timeline) {
    tl = timeline + 3 * gwave;
    if (lane == 0) tl[0] = t_entry, tl[1] = __builtin_amdgcn_s_memrealtime(), tl[2] = 0;
  }
  if (fb1 == fb0) return;

  // A range (a workgroup's slice of frames) is addressed through one buffer
  // descriptor whose base is 4-byte aligned (128-byte aligned for 32-lane
  // rows, whose windows run between lines): rel(x) = x - off[fb0] + adj.
  const uint32_t amask = (line || strm) ? 127u : (narrow && NW4 == 4) ? 15u : 3u;
  struct Range {
    uint64_t f0, f1, o0, o1;
    bool fits;  // byte range within 31-bit buffer offsets
  };
  auto range_of = [&](uint64_t b, uint64_t o0, uint64_t o1) -> Range {
    Range r;
    r.f0 = b * per_block < nframes ? b * per_block : nframes;
    r.f1 = r.f0 + per_block < nframes ? r.f0 + per_block : nframes;
    r.o0 = o0, r.o1 = o1;
    const uint64_t bytes_ = o1 > o0 ? o1 - o0 : 0;  // non-decreasing offsets are the contract
    const uint32_t adj = (uint32_t)((reinterpret_cast<uintptr_t>(bytes) + o0) & amask);
    r.fits = bytes_ + adj + 4096 < (1ull << 31);
    return r;
  };
  auto ctx_of = [&](const Range& r) -> WaveCtx {
    WaveCtx cx;
    const uint64_t bytes_ = r.o1 > r.o0 ? r.o1 - r.o0 : 0;
    cx.adj = (uint32_t)((reinterpret_cast<uintptr_t>(bytes) + r.o0) & amask);
    cx.nfb = (uint32_t)(r.f1 - r.f0);
    cx.data_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(bytes + r.o0 - cx.adj), (short)0,
                                                     (int)((bytes_ + cx.adj + 3) & ~3ull), 0x00020000);
    cx.off_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint64_t*>(off + r.f0), (short)0,
                                                    (int)((cx.nfb + (SEG ? 0u : 1u)) * 8u), 0x00020000);
    cx.len_rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t*>(SEG ? seg_len + r.f0 : seg_len), (short)0,
                                                    (int)(SEG ? cx.nfb * 4u : 0u), 0x00020000);
    constexpr uint32_t elem = MODE == CrcMode::kCrc ? 4u : 1u;
    cx.out_rsrc = __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<char*>(out) + r.f0 * elem, (short)0,
                                                    (int)(cx.nfb * elem), 0x00020000);
    cx.o0_lo = (uint32_t)r.o0;
    cx.ctr = lds_words + kCtrBase / 4;
    cx.ap.data_base = const_cast<uint8_t*>(bytes + r.o0 - cx.adj);
    cx.ap.lenw = const_cast<uint32_t*>(SEG ? seg_len + r.f0 : seg_len);
    cx.ap.stat = reinterpret_cast<uint8_t*>(out) + r.f0;
    cx.ap.cap = cap;
    cx.ap.rend = (uint32_t)(bytes_ + cx.adj);
    return cx;
  };
  const Range own = range_of(blockIdx.x, ob0, ob1);
  if (!own.fits || seg_bad) {
    // gigabyte frames, or segments out of address order: static per-wave
    // ranges on the unpipelined path, each frame from its own start
    const uint64_t fw0 = gwave * frames_per_wave < nframes ? gwave * frames_per_wave : nframes;
    const uint64_t fw1 = fw0 + frames_per_wave < nframes ? fw0 + frames_per_wave : nframes;
    if (narrow && NW4 != 4) {
      L.p = lane & 3u, L.row = lane >> 2;
      rows_generic<MODE, 4>(lds, L, bytes, off, SEG ? seg_len : nullptr, fw0, fw1, out, cap);
    } else if (!line) {  // (also the narrow rows of four words: the RL = 16 image)
      L.p = lane & 15u, L.row = lane >> 4;
      rows_generic<MODE, 16>(lds, L, bytes, off, SEG ? seg_len : nullptr, fw0, fw1, out, cap);
    } else {  // the RL = 32 image: 32-lane rows
      L.p = lane & 31u, L.row = lane >> 5;
      rows_generic<MODE, 32>(lds, L, bytes, off, SEG ? seg_len : nullptr, fw0, fw1, out, cap);
    }
  } else {
    // chunks of the own slice from the LDS counter
    const WaveCtx cx = ctx_of(own);
    asm volatile("s_nop 4" ::: "memory");  // descriptors may be SGPRs just written by VALU readfirstlane
#ifdef LNX_RESEARCH
    if constexpr (STR != 0 && !SEG && MODE != CrcMode::kAppend) {
      if (strm) {
        if constexpr (STR == 3) {
          lanes_body<MODE, VAR>(lds, L, cx);
        } else {
          constexpr int RLS = STR == 2 ? 4 : 8;
          L.p = lane & (RLS - 1u), L.row = lane / RLS;
          stream_body<MODE, VAR, RLS>(lds, L, cx);
        }
        if (tl && lane == 0) tl[2] = __builtin_amdgcn_s_memrealtime();
        return;
      }
    }
#else
    static_assert(STR == 0 && VAR == 0, "variants are built into the research library only");
#endif
    if (narrow) {
      L.p = lane & 3u, L.row = lane >> 2;
      rows_body<MODE, 4, KS4, S4, CH4, VAR, SEG, NW4, true, NSR4>(lds, L, cx);
    } else if (rl == 16 && lean) {
      // lean rows: 16 lanes x two words (LWL = 2) or 32 lanes x one word (LWL = 1)
      L.p = lane & (32u / LWL - 1u), L.row = lane / (32u / LWL);
      lines_body<MODE, KSL, VAR, LWL, LJM, LEP, SEG>(lds, L, cx);
    } else if (rl == 16) {
      L.p = lane & 15u, L.row = lane >> 4;
      rows_body<MODE, 16, KSM, SM, CHM, VAR, SEG, MIDW == 2 ? 2 : 1, true, MIDW == 2 ? 0 : NSR4>(lds, L, cx);
    } else if (RLF != 16) {
      L.p = lane & 31u, L.row = lane >> 5;
      rows_body<MODE, 32, KSW, SW, CHW, VAR, SEG, 1, REDGE>(lds, L, cx);
    }
  }
  if (tl && lane == 0) tl[2] = __builtin_amdgcn_s_memrealtime();
}

hipError_t launch_rows(int var, CrcMode mode, const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out,
                       const void* images, int num_cus, hipStream_t stream, uint64_t* timeline = nullptr,
                       const uint32_t* seg_len = nullptr, uint32_t cap = 0, uint32_t policy = kPolicyRows,
                       uint32_t* stage_flag = nullptr, uint32_t epoch = 0) {
  const bool verify = mode == CrcMode::kVerify;
  if (n == 0) return hipSuccess;
  // the slices of dispatch.hpp (the staged launch uses the same): at least
  // one 16-lane row set per wave
  const SlicePlan pl = slice_plan(n, num_cus);
  static_assert(kWavesPerBlock == 16, "slice_plan's slices are whole 16-wave sets");
  const uint64_t grid = pl.grid;
  const uint64_t fpw = pl.per / kWavesPerBlock;
  const uint4* img = static_cast<const uint4*>(images);
  const dim3 g((unsigned)grid), b(kBlockThreads);
#define LNX_LAUNCH(M, ...) \
  hipLaunchKernelGGL((crc32_rows_kernel<M, __VA_ARGS__>), g, b, 0, stream, bytes, off, n, fpw, img, out, \
                     timeline, seg_len, cap, policy, stage_flag, epoch)
  if (seg_len) {  // segment mode (lnx_crc32_segments, the TX FCS append, the receive ring)
    // (every lean-row step non-temporal, EP = 0, was measured no faster for
    // ring slots and is not built: profiles/r2s2r_segment_ep_rejected.txt)
    if (verify)
      LNX_LAUNCH(CrcMode::kVerify, 0, 0, 24, 1, 12, 2, 4, 16, true);
#ifdef LNX_RESEARCH
    else if (mode == CrcMode::kAppend && var == 4)  // profiling: FCS stored at once, no hold
      LNX_LAUNCH(CrcMode::kAppend, 4, 0, 24, 1, 12, 2, 4, 16, true);
    else if (mode == CrcMode::kAppend && var == 7)  // profiling: the FCS written with its 64-byte sector
      LNX_LAUNCH(CrcMode::kAppend, 7, 0, 24, 1, 12, 2, 4, 16, true);
#endif
    else if (mode == CrcMode::kAppend)
      LNX_LAUNCH(CrcMode::kAppend, 0, 0, 24, 1, 12, 2, 4, 16, true);
    else
      LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 12, 2, 4, 16, true);
  } else if (verify) {
    LNX_LAUNCH(CrcMode::kVerify, 0);
  } else {
#ifndef LNX_RESEARCH
    (void)var;
    LNX_LAUNCH(CrcMode::kCrc, 0);
#else
    // profiling variants (tools/prof/variants.py).  Arguments:
    // VAR, forced row width (0 = per workgroup), KSW, SW, KS4, S4, CHW, CH4,
    // SEG, MIDW, KSM, SM, CHM
#define LNX_16(W, KS_, S_, CH_) LNX_LAUNCH(CrcMode::kCrc, 0, 16, 24, 1, 12, 2, 4, 16, false, W, KS_, S_, CH_)
    switch (var) {
      case 1: LNX_LAUNCH(CrcMode::kCrc, 1); break;  // loads + bookkeeping only
      case 2: LNX_LAUNCH(CrcMode::kCrc, 2); break;  // lookups + bookkeeping only
      case 3: LNX_LAUNCH(CrcMode::kCrc, 3); break;  // bounds window loaded by all 64 lanes
      case 5: LNX_LAUNCH(CrcMode::kCrc, 5); break;  // clock-window flushes for 4-lane rows too
      // 10-16: forced 32-lane rows (KSW, SW, CHW vary)
      case 10: LNX_LAUNCH(CrcMode::kCrc, 0, 32, 13, 1, 12, 2, 4, 16); break;  // one 13-line item per 1500 B
      case 11: LNX_LAUNCH(CrcMode::kCrc, 0, 32, 13, 2, 12, 2, 4, 16); break;  // two-slot ring
      case 12: LNX_LAUNCH(CrcMode::kCrc, 0, 32, 14, 1, 12, 2, 4, 16); break;
      case 13: LNX_LAUNCH(CrcMode::kCrc, 0, 32, 13, 1, 12, 2, 2, 16); break;  // 2-frame chunks
      case 14: LNX_LAUNCH(CrcMode::kCrc, 0, 32, 13, 1, 12, 2, 8, 16); break;  // 8-frame chunks
      case 15: LNX_LAUNCH(CrcMode::kCrc, 0, 32, 24, 1, 12, 2, 4, 16); break;  // 24-line items
      case 16: LNX_LAUNCH(CrcMode::kCrc, 0, 32, 18, 1, 12, 2, 4, 16); break;
      // forced 16-lane rows: one word per lane (17, 21), two words per lane (18, 19, 28, 29, 40-42)
      case 17: LNX_16(1, 24, 1, 4); break;  // round-1 product
      case 21: LNX_16(1, 12, 3, 4); break;
      case 18: LNX_16(2, 13, 1, 4); break;  // one 13-line item per 1500 B
      case 19: LNX_16(2, 13, 2, 4); break;  // two-slot ring
      case 28: LNX_16(2, 14, 1, 4); break;
      case 29: LNX_16(2, 24, 1, 4); break;  // 24-line items
      case 43: LNX_16(2, 32, 1, 4); break;  // 32-line items
      case 44: LNX_16(2, 18, 1, 4); break;
      case 40: LNX_16(2, 13, 1, 8); break;  // 8-frame chunks
      case 41: LNX_16(2, 12, 2, 4); break;
      case 42: LNX_16(2, 13, 1, 16); break;
      // forced lean line rows (lines_body): KSL 13 / 14 / 12, loads only, math only
#define LNX_LEAN(V, KSL_) LNX_LAUNCH(CrcMode::kCrc, V, 16, 24, 1, 12, 2, 4, 16, false, 3, 24, 1, 4, KSL_)
      case 50: LNX_LEAN(0, 13); break;
      case 51: LNX_LEAN(0, 14); break;
      case 52: LNX_LEAN(0, 12); break;
      case 53: LNX_LEAN(1, 13); break;
      case 54: LNX_LEAN(2, 13); break;
      // forced lean rows on 32 lanes x one word (KSL 13), loads only, math only
      case 70: LNX_LAUNCH(CrcMode::kCrc, 0, 16, 24, 1, 12, 2, 4, 16, false, 3, 24, 1, 4, 13, 1); break;
      case 71: LNX_LAUNCH(CrcMode::kCrc, 1, 16, 24, 1, 12, 2, 4, 16, false, 3, 24, 1, 4, 13, 1); break;
      case 72: LNX_LAUNCH(CrcMode::kCrc, 2, 16, 24, 1, 12, 2, 4, 16, false, 3, 24, 1, 4, 13, 1); break;
      // product dispatch with one-word 16-lane rows instead of lean rows (the r1f product)
      case 56: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 12, 2, 4, 16, false, 1); break;
      // the product dispatch with the r1 lean rows (junk word reloaded, its U-image taken out), and its loads only
      case 57: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 12, 2, 4, 16, false, 4, 24, 1, 4, 13, 2, false); break;
      case 58: LNX_LAUNCH(CrcMode::kCrc, 1, 0, 24, 1, 12, 2, 4, 16, false, 4, 24, 1, 4, 13, 2, false); break;
      // lean rows by the cache policy of their step loads (lines_body EP): all nt (the r2b product) and
      // its loads only, the first step at the default policy, every step at the default policy
      case 90: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 12, 2, 4, 16, false, 4, 24, 1, 4, 13, 2, true, 0); break;
      case 91: LNX_LAUNCH(CrcMode::kCrc, 1, 0, 24, 1, 12, 2, 4, 16, false, 4, 24, 1, 4, 13, 2, true, 0); break;
      case 92: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 12, 2, 4, 16, false, 4, 24, 1, 4, 13, 2, true, 2); break;
      case 93: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 12, 2, 4, 16, false, 4, 24, 1, 4, 13, 2, true, 3); break;
      // the product dispatch with 32-lane line rows all nt (the r1 form)
      case 97: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, false); break;
#undef LNX_LEAN
      // forced 4-lane rows
      case 22: LNX_LAUNCH(CrcMode::kCrc, 0, 4); break;
      case 23: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 8, 3, 4, 64); break;
      case 24: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 12, 2, 4, 32); break;
      case 25: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 6, 3, 4, 64); break;
      case 60: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 16, 2, 4, 16); break;  // longer 4-lane items
      case 61: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 20, 1, 4, 16); break;
      case 62: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 12, 2, 4, 32); break;
      case 63: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 16, 2, 4, 32); break;
      case 64: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 12, 2, 4, 64); break;
      case 65: LNX_LAUNCH(CrcMode::kCrc, 0, 4, 24, 1, 16, 2, 4, 64); break;
      // narrow and one-word 16-lane rows by the runs their item loads (NSR4): 125 every step of
      // the item (the r2 product: a short last item reads the next frames' bytes), 124 / 120 / 126
      // runs of 1 / 2 / 6 steps (the product: 4; r2ze/r2zf Zipf 1.057 ms against 1.071 for 2, 1.077
      // for every step, 1.056 for 6)
      case 125: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 0); break;
      case 120: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 2); break;
      case 124: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 1); break;
      case 126: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 6); break;
      // four-word 4-lane rows (dwordx4: 64 contiguous bytes per row instruction) under the product
      // dispatch: KS4 steps of 64 B, S4 slots, CH4-frame chunks, NSR4-step load runs
#define LNX_W4(V, KS_, S_, CH_, NSR_) \
  LNX_LAUNCH(CrcMode::kCrc, V, 0, 24, 1, KS_, S_, 4, CH_, false, 4, 24, 1, 4, 13, 2, true, 1, true, NSR_, 4)
      case 130: LNX_W4(0, 4, 2, 32, 1); break;
      case 135: LNX_W4(1, 4, 2, 32, 1); break;  // loads + bookkeeping only
      case 136: LNX_W4(2, 4, 2, 32, 1); break;  // math + bookkeeping only
      case 138: LNX_W4(0, 4, 2, 16, 1); break;
      case 139: LNX_W4(0, 3, 2, 32, 1); break;
      case 140: LNX_W4(0, 5, 2, 32, 1); break;
#undef LNX_W4
      // streaming rows (research/stream_rows.hpp) for the narrow rows' frames, under the product dispatch
      case 150: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 1); break;
      // its loads + chain only (no frame boundaries), loads only
      case 151: LNX_LAUNCH(CrcMode::kCrc, 151, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 1); break;
      case 152: LNX_LAUNCH(CrcMode::kCrc, 152, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 1); break;
      // the same on 4-lane rows (64-byte row steps, at most one boundary per step): full, loads + chain, loads
      case 153: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 2); break;
      case 154: LNX_LAUNCH(CrcMode::kCrc, 151, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 2); break;
      case 155: LNX_LAUNCH(CrcMode::kCrc, 152, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 2); break;
      // lane streams (research/stream_lanes.hpp): full, loads only, loads + chain only
      case 160: LNX_LAUNCH(CrcMode::kCrc, 0, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 3); break;
      case 161: LNX_LAUNCH(CrcMode::kCrc, 161, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 3); break;
      case 162: LNX_LAUNCH(CrcMode::kCrc, 162, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 3); break;
      case 164: LNX_LAUNCH(CrcMode::kCrc, 164, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 3); break;  // reset in the fold
      case 165: LNX_LAUNCH(CrcMode::kCrc, 165, 0, 24, 1, 16, 2, 4, 32, false, 4, 24, 1, 4, 13, 2, true, 1, true, 4, 1, 3); break;  // + offsets on even sets only
      case 26: LNX_LAUNCH(CrcMode::kCrc, 1, 4); break;  // 4-lane rows, loads only
      case 27: LNX_LAUNCH(CrcMode::kCrc, 2, 4); break;  // 4-lane rows, math only
      default: LNX_LAUNCH(CrcMode::kCrc, 0); break;
    }
#undef LNX_16
#endif  // LNX_RESEARCH
  }
#undef LNX_LAUNCH
  return hipGetLastError();
}

// Host-side launch helpers (called from api.cpp).
hipError_t launch_crc32_frames(const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out, bool verify,
                               const void* images, int num_cus, hipStream_t stream, uint32_t policy,
                               uint32_t* stage_flag, uint32_t epoch) {
  return launch_rows(0, verify ? CrcMode::kVerify : CrcMode::kCrc, bytes, off, n, out, images, num_cus, stream,
                     nullptr, nullptr, 0, policy, stage_flag, epoch);
}
#ifdef LNX_RESEARCH
hipError_t launch_crc32_variant(int var, const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out,
                                const void* images, int num_cus, hipStream_t stream, uint64_t* timeline) {
  // 80 / 81: the product with 2 / 4 workgroups per CU over the launch (one is
  // resident at a time: the later ones go to the CUs that finish first)
  if (var == 80 || var == 81)
    return launch_rows(0, CrcMode::kCrc, bytes, off, n, out, images, num_cus * (var == 80 ? 2 : 4), stream, nullptr);
  return launch_rows(var, CrcMode::kCrc, bytes, off, n, out, images, num_cus, stream, timeline);
}
#endif
hipError_t launch_crc32_segments(const uint8_t* bytes, const uint64_t* start, const uint32_t* len, uint64_t n,
                                 void* out, const void* images, int num_cus, hipStream_t stream) {
  return launch_rows(0, CrcMode::kCrc, bytes, start, n, out, images, num_cus, stream, nullptr, len);
}
hipError_t launch_fcs_verify_segments(const uint8_t* bytes, const uint64_t* start, const uint32_t* len, uint64_t n,
                                      uint8_t* ok, const void* images, int num_cus, hipStream_t stream) {
  return launch_rows(0, CrcMode::kVerify, bytes, start, n, ok, images, num_cus, stream, nullptr, len);
}
// TX FCS append in place (kAppend, one launch): pad to 60, LE FCS, len += pad + 4, status.
hipError_t launch_fcs_append(uint8_t* bytes, const uint64_t* start, uint32_t* len, uint64_t n, uint32_t capacity,
                             uint8_t* status, const void* images, int num_cus, hipStream_t stream, int var) {
  return launch_rows(var, CrcMode::kAppend, bytes, start, n, status, images, num_cus, stream, nullptr, len, capacity);
}
#ifdef LNX_RESEARCH
// TX FCS append, second launch (lnx__fcs_append_variant 200): frame i's CRC, taken
// by the segment-mode CRC kernel into a compact array, goes into the frame's
// slot here, with the runt padding, the new length and the status
// (internet/stack-ethernet.go:200-214; oracle.fcs_append).  Stores in place
// during the CRC kernel's read stream cost it about 30 %; the same 1 M stores
// as a launch of their own take 16 us (tools/ubench/scatter_write.hip modes 1,
// 3, 11).
__global__ void __launch_bounds__(256) fcs_scatter_kernel(uint8_t* __restrict__ bytes, const uint64_t* __restrict__ start,
                                                          uint32_t* __restrict__ len, const uint32_t* __restrict__ crc,
                                                          uint64_t n, uint32_t cap, uint8_t* __restrict__ status) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t fl = len[i];
    const uint32_t k = fl < kMinFrame ? kMinFrame - fl : 0u;  // zero pad of a runt
    if ((uint64_t)fl + k + 4u > cap) {
      status[i] = kErrShortBuffer;  // left untouched
      continue;
    }
    uint8_t* fr = bytes + start[i];
    uint32_t c = crc[i];
    if (k) {  // CRC of the padded frame: the register advanced over k zero bytes
      uint32_t r = ~c;
      for (uint32_t b = 0; b < 8u * k; ++b) r = (r >> 1) ^ ((r & 1u) ? 0xEDB88320u : 0u);
      c = ~r;
      for (uint32_t j = 0; j < k; ++j) fr[fl + j] = 0;
    }
    uint8_t* q = fr + fl + k;
    if ((reinterpret_cast<uintptr_t>(q) & 3u) == 0) {
      *reinterpret_cast<uint32_t*>(q) = c;  // LE: the FCS byte order
    } else {
      q[0] = (uint8_t)c, q[1] = (uint8_t)(c >> 8), q[2] = (uint8_t)(c >> 16), q[3] = (uint8_t)(c >> 24);
    }
    len[i] = fl + k + 4u;
    status[i] = 0;
  }
}
hipError_t launch_fcs_scatter(uint8_t* bytes, const uint64_t* start, uint32_t* len, const uint32_t* crc, uint64_t n,
                              uint32_t capacity, uint8_t* status, int num_cus, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  uint64_t grid = (n + 255) / 256;
  const uint64_t gmax = (uint64_t)num_cus * 16;
  if (grid > gmax) grid = gmax;
  hipLaunchKernelGGL(fcs_scatter_kernel, dim3((unsigned)grid), dim3(256), 0, stream, bytes, start, len, crc, n,
                     capacity, status);
  return hipGetLastError();
}
#endif  // LNX_RESEARCH

// Waves of a launch (sizes the timeline buffer: 3 uint64 per wave).
uint64_t crc32_launch_waves(uint64_t n, int num_cus) {
  const uint64_t per_block = (uint64_t)kWavesPerBlock * 4;
  uint64_t grid = (n + per_block - 1) / per_block;
  if (grid > (uint64_t)num_cus) grid = (uint64_t)num_cus;
  return grid * kWavesPerBlock;
}

}  // namespace lnx
