// crc32_kernel.hip — batched CRC-32/IEEE (Ethernet FCS) over packed frames, gfx950.
//
// Reference semantics: ethernet.CRC32 (lneto ethernet/crc.go:19-21) =
// Go crc32.Checksum(data, IEEETable): init 0xFFFFFFFF, reflected, xorout
// 0xFFFFFFFF.  The FCS-verify mode implements the residue form of the check a
// receiver does before StackEthernet.Demux (internet/stack-ethernet.go:139).
//
// Work decomposition: one wave owns one frame at a time.  The
// frame is viewed through a window that ENDS at the frame's last byte and is a
// whole number J of 256-byte steps long; the lead-in (< 256 bytes) before the
// frame start is zero-masked.  With init 0 the CRC register ignores leading
// zeros, so the window's register equals the frame's.  The init value is
// folded in by XOR-ing 0xFF into the frame's first four bytes.
//
// Lane l consumes the 4-byte word at window offset 4l + 256j (j = 0..J-1): one
// fully coalesced 256-byte dword load per wave per step.  Each lane keeps its
// own register r_l and advances it with r_l = U(r_l ^ w), U = Z_256, through
// four lane-private byte tables in LDS (lds_layout.hpp).  After the last step
// lane l's register sits 4l bytes past the frame end; F_l = Z_{-4l} moves it
// back, and the frame register is the XOR of the 64 lane registers (a DPP
// butterfly + four readlanes).  No MFMA: this is a per-byte GF(2) polynomial.
//
// Latency hiding: a wave's frames are cut into "items" of <= kSteps window
// steps; a 4-slot register ring keeps the loads of the next three items in
// flight while one item is folded into the registers (software pipeline,
// DESIGN.md §2.3).  Frames whose end is not 4-byte aligned load the aligned
// dword A_{l+1} per lane and rebuild their window word with v_alignbyte from
// A_l, which comes from lane l-1 through DPP wave_shr:1 (lane 0 takes the last
// lane's A_64 of the previous step, carried in an SGPR).
#include <hip/hip_runtime.h>
#include <cstdint>
#include "lds_layout.hpp"

namespace lnx {

constexpr int kBlockThreads = 1024;
constexpr int kWavesPerBlock = kBlockThreads / 64;
constexpr int kSteps = 6;  // window steps per pipeline item (1500-B frame = 6 steps)
constexpr int kSlots = 4;  // pipeline depth (items whose loads are in flight)

__device__ __forceinline__ uint32_t lds_rd(const char* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(lds + byte_addr);
}

// Streaming dword load whose completion the CALLER waits for (vmcnt is not
// tracked by hipcc for asm loads, cdna_hip_programming.md §5.7 item 1).  Every
// destination is later passed "+v" through slot_wait() before its first use.
__device__ __forceinline__ uint32_t ld_stream(const uint32_t* p) {
  uint32_t r;
  asm volatile("global_load_dword %0, %1, off nt" : "=v"(r) : "v"(p));
  return r;
}

// Scalar (SMEM) loads of wave-uniform metadata.  Written as asm so they can
// never become VMEM loads: a compiler-generated VMEM load here comes with an
// s_waitcnt vmcnt(0) that would drain the whole streaming ring.  The s_nop
// covers a VALU (readfirstlane) -> SMEM-address SGPR dependency.
__device__ __forceinline__ uint64_t uniform_ptr(const void* p) {
  const uint64_t v = reinterpret_cast<uint64_t>(p);
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)v);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(v >> 32));
  return (uint64_t)lo | ((uint64_t)hi << 32);
}
__device__ __forceinline__ void sload_bounds(const uint64_t* p, uint64_t& s, uint64_t& e) {
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
  u32x4 v;
  asm volatile("s_nop 4\n\ts_load_dwordx4 %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(v) : "s"(uniform_ptr(p)) : "memory");
  s = (uint64_t)v.x | ((uint64_t)v.y << 32);
  e = (uint64_t)v.z | ((uint64_t)v.w << 32);
}
__device__ __forceinline__ uint32_t sload_dword(const void* p) {
  uint32_t v;
  asm volatile("s_nop 4\n\ts_load_dword %0, %1, 0x0\n\ts_waitcnt lgkmcnt(0)"
               : "=s"(v) : "s"(uniform_ptr(p)) : "memory");
  return v;
}

// r' = U(x): four lane-private byte lookups; byte k of x -> address byte 1.
__device__ __forceinline__ uint32_t u_step(const char* lds, uint32_t x, uint32_t b0, uint32_t b1) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, b0, 0x0c020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, b0, 0x0c020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, b1, 0x0c020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, b1, 0x0c020700u);
  return lds_rd(lds, a0) ^ lds_rd(lds, a1 + 128) ^ lds_rd(lds, a2) ^ lds_rd(lds, a3 + 128);
}

// F_l(r) through eight lane-private nibble tables.
__device__ __forceinline__ uint32_t f_step(const char* lds, uint32_t r, uint32_t bf) {
  uint32_t acc = 0;
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const uint32_t a = (((r >> (4 * i)) & 15u) << 7) | bf;
    acc ^= lds_rd(lds, a + (uint32_t)(i << 11));
  }
  return acc;
}

// XOR of a value over the 64 lanes of the wave; result is wave-uniform.
__device__ __forceinline__ uint32_t wave_xor(uint32_t v) {
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x124, 0xF, 0xF, false);  // row_ror:4
  v ^= (uint32_t)__builtin_amdgcn_mov_dpp((int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return (uint32_t)(__builtin_amdgcn_readlane((int)v, 0) ^ __builtin_amdgcn_readlane((int)v, 16) ^
                    __builtin_amdgcn_readlane((int)v, 32) ^ __builtin_amdgcn_readlane((int)v, 48));
}

// Bytes [lo, 4) of a little-endian word kept (lo clamped to 0..4).
__device__ __forceinline__ uint32_t keep_from(int32_t lo) {
  lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
  return (uint32_t)(0xFFFFFFFFull << (8 * lo));
}

enum class CrcMode : int { kCrc = 0, kVerify = 1 };

// Wave-uniform description of one pipeline item (lives in SGPRs).
struct Item {
  uint64_t f;    // frame index
  uint64_t e;    // frame end offset
  uint64_t n;    // frame length
  uint32_t j0;   // first window step of the item
  uint32_t ns;   // steps in the item
  bool valid;
  bool last;     // item finishes its frame
};

// Wave-uniform cursor over the wave's frames.
struct Cursor {
  uint64_t f, fend;
  uint64_t e, n;
  uint32_t J, j;
};

template <CrcMode MODE>
__global__ void __launch_bounds__(kBlockThreads, 1)
crc32_frames_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                    uint64_t nframes, uint64_t frames_per_block,
                    const uint4* __restrict__ image, void* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint32_t lds_words[kLdsDwords];
  {
    uint4* l4 = reinterpret_cast<uint4*>(lds_words);
#pragma unroll
    for (int i = 0; i < (int)(kLdsBytes / 16 / kBlockThreads); ++i)
      l4[threadIdx.x + i * kBlockThreads] = image[threadIdx.x + i * kBlockThreads];
  }
  __syncthreads();
  const char* lds = reinterpret_cast<const char*>(lds_words);

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t col = lane & 31u;
  const uint32_t bu0 = col << 2;
  const uint32_t bu1 = bu0 | 65536u;
  const uint32_t bf = kFBase | ((lane >> 5) << 14) | (col << 2);
  const uintptr_t base = reinterpret_cast<uintptr_t>(bytes);

  const uint64_t fbeg = (uint64_t)blockIdx.x * frames_per_block;
  // Output descriptor covering this block's frames only (32-bit offsets).
  const uint32_t elem = MODE == CrcMode::kCrc ? 4u : 1u;
  char* out_blk = reinterpret_cast<char*>(out) + fbeg * elem;
  const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      out_blk, (short)0, (int)(frames_per_block * elem), 0x00020000);
  Cursor cur;
  {
    cur.fend = fbeg + frames_per_block < nframes ? fbeg + frames_per_block : nframes;
    cur.f = fbeg + wave - kWavesPerBlock;  // advanced onto the first frame by next_item
    cur.J = 0;
    cur.j = 1;  // "frame exhausted" -> first next_item() moves to frame fbeg + wave
    cur.e = cur.n = 0;
  }

  // An item that loads and computes nothing (pipeline fill).
  Item bubble;
  bubble.f = fbeg;
  bubble.e = bubble.n = 0;
  bubble.j0 = bubble.ns = 0;
  bubble.valid = true;
  bubble.last = false;

  // Produce the next item of this wave's stream (scalar work only).
  auto next_item = [&](Item& it) {
    if (cur.j >= cur.J && !(cur.J == 0 && cur.j == 0)) {
      cur.f += kWavesPerBlock;
      if (cur.f < cur.fend) {
        uint64_t s, e;
        sload_bounds(off + cur.f, s, e);
        cur.e = e;
        cur.n = e > s ? e - s : 0;
        cur.J = (uint32_t)((cur.n + kWindowBytes - 1) / kWindowBytes);
        cur.j = 0;
      }
    }
    it.valid = cur.f < cur.fend;
    it.f = cur.f;
    it.e = cur.e;
    it.n = cur.n;
    it.j0 = cur.j;
    const uint32_t left = cur.J - cur.j;
    it.ns = left < (uint32_t)kSteps ? left : (uint32_t)kSteps;
    it.last = (it.j0 + it.ns == cur.J);
    cur.j += it.ns;
    if (cur.J == 0) cur.j = 1;  // empty frame: one item of zero steps, then move on
  };

  // Issue the loads of an item into w[0..kSteps).  Straight-line on purpose:
  // every item issues exactly kSteps loads (steps past the item, and lanes
  // whose step-0 dword holds no frame byte, read a harmless dummy address and
  // their value is masked later), so the compiler can count vmcnt statically
  // and wait only for the slot being consumed, never vmcnt(0).
  auto issue = [&](const Item& it, uint32_t (&w)[kSteps]) {
    const uint32_t J = (uint32_t)((it.n + kWindowBytes - 1) / kWindowBytes);
    const uint32_t ra = (uint32_t)((base + it.e) & 3u);
    const uint32_t lead = J * kWindowBytes - (uint32_t)it.n;
    const uint8_t* win = bytes + (it.e - (uint64_t)J * kWindowBytes);
    const uint32_t lane_off = (lane << 2) + (ra ? 4u - ra : 0u);
    const int32_t d0 = (int32_t)lead - (int32_t)(lane << 2);
    // Step 0: load only dwords holding at least one frame byte.
    const bool need0 = ra ? (d0 <= (int32_t)(7 - ra)) : (d0 < 4);
    const uint32_t* dummy = reinterpret_cast<const uint32_t*>(off);
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
      const uint32_t j = it.j0 + k;
      const bool live = it.valid && (uint32_t)k < it.ns && (j != 0 || need0);
      const uint32_t* p = reinterpret_cast<const uint32_t*>(win + (uint64_t)j * kWindowBytes + lane_off);
      w[k] = ld_stream(live ? p : dummy);
    }
  };

  uint32_t reg = 0;    // this lane's CRC register for the frame in progress
  uint32_t carry = 0;  // A_0 of the next step (unaligned frames), wave-uniform

  // Fold an item's words into the registers; finalize the frame if it ends here.
  auto compute = [&](const Item& it, uint32_t (&w)[kSteps]) {
    // This slot's kSteps loads are older than the (kSlots-1)*kSteps loads of
    // the three other slots issued since (plus at most three stores), so
    // vmcnt <= (kSlots-1)*kSteps guarantees they have landed.
    static_assert(kSteps == 6 && kSlots == 4, "vmcnt literal below");
    asm volatile("s_waitcnt vmcnt(18)" : "+v"(w[0]), "+v"(w[1]), "+v"(w[2]), "+v"(w[3]), "+v"(w[4]), "+v"(w[5]));
    const uint32_t J = (uint32_t)((it.n + kWindowBytes - 1) / kWindowBytes);
    const uint32_t ra = (uint32_t)((base + it.e) & 3u);
    const uint32_t lead = J * kWindowBytes - (uint32_t)it.n;
    const uint32_t m4 = it.n < 4 ? (uint32_t)it.n : 4u;
    if (it.j0 == 0) {
      reg = 0;
      carry = 0;
      if (ra != 0 && J != 0 && (int32_t)lead <= (int32_t)(3 - ra)) {
        // A_0 (dword before lane 0's A_1) holds frame bytes: scalar load.
        const uint8_t* win = bytes + (it.e - (uint64_t)J * kWindowBytes);
        carry = sload_dword(win - ra);
      }
    }
#pragma unroll
    for (int k = 0; k < kSteps; ++k) {
      if ((uint32_t)k < it.ns) {
        const uint32_t j = it.j0 + k;
        uint32_t x = w[k];
        if (ra != 0) {
          const uint32_t prev = (uint32_t)__builtin_amdgcn_update_dpp((int)carry, (int)x, 0x138, 0xF, 0xF, false);
          carry = (uint32_t)__builtin_amdgcn_readlane((int)x, 63);
          x = __builtin_amdgcn_alignbyte(x, prev, ra);
        }
        if (j == 0) {
          // zero the lead-in, XOR the CRC init into the frame's first bytes
          const int32_t d0 = (int32_t)lead - (int32_t)(lane << 2);
          const uint32_t keep = keep_from(d0);
          x = (x & keep) ^ (keep & ~keep_from(d0 + (int32_t)m4));
        } else if (j == 1) {
          const int32_t x1 = (int32_t)(lead + m4) - (int32_t)kWindowBytes;  // init bytes spilling into step 1
          if (x1 > 0 && lane == 0) x ^= (uint32_t)((1ull << (8 * x1)) - 1);
        }
        reg = u_step(lds, reg ^ x, bu0, bu1);
      }
    }
    uint32_t crc = 0;
    if (it.last) {
      uint32_t R = 0;
      if (J != 0) R = wave_xor(f_step(lds, reg, bf));
      if (it.n < 4) R ^= (uint32_t)(0xFFFFFFFFull >> (8 * it.n));
      crc = ~R;
    }
    // Unconditional buffer store (outside any branch, so the vmcnt count stays
    // static): only lane 0 of an item that finishes its frame gets an in-range
    // offset; the hardware drops the other lanes' out-of-range stores.
    const uint32_t rel = (uint32_t)(it.f - fbeg);
    const bool st = it.valid && it.last && lane == 0;
    if (MODE == CrcMode::kCrc)
      __builtin_amdgcn_raw_buffer_store_b32(crc, out_rsrc, st ? rel * 4u : 0xFFFFFFF0u, 0, 0);
    else
      __builtin_amdgcn_raw_buffer_store_b8((uint8_t)((it.n >= 4 && crc == 0x2144DF1Cu) ? 1 : 0), out_rsrc,
                                           st ? rel : 0xFFFFFFF0u, 0, 0);
  };

  // The ring starts with four empty "bubble" items (no loads, no output), so
  // the loop body is the only code that issues the streaming loads and the
  // fixed vmcnt(18) in compute() holds from the first iteration on.
  // sched_barrier keeps each slot's loads in program order.
#define LNX_FENCE __builtin_amdgcn_sched_barrier(0)
  Item it0 = bubble, it1 = bubble, it2 = bubble, it3 = bubble;
  uint32_t w0[kSteps] = {}, w1[kSteps] = {}, w2[kSteps] = {}, w3[kSteps] = {};
  static_assert(kSlots == 4, "ring is unrolled by hand");
  while (true) {
    if (!it0.valid) break;
    compute(it0, w0); next_item(it0); LNX_FENCE; issue(it0, w0); LNX_FENCE;
    if (!it1.valid) break;
    compute(it1, w1); next_item(it1); LNX_FENCE; issue(it1, w1); LNX_FENCE;
    if (!it2.valid) break;
    compute(it2, w2); next_item(it2); LNX_FENCE; issue(it2, w2); LNX_FENCE;
    if (!it3.valid) break;
    compute(it3, w3); next_item(it3); LNX_FENCE; issue(it3, w3); LNX_FENCE;
  }
#undef LNX_FENCE
}

// Host-side launch helper (called from api.cpp).
hipError_t launch_crc32_frames(const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out,
                               bool verify, const void* image, int num_cus, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  uint64_t grid = (n + kWavesPerBlock - 1) / kWavesPerBlock;
  if (grid > (uint64_t)num_cus) grid = (uint64_t)num_cus;
  const uint64_t fpb = (n + grid - 1) / grid;
  if (verify)
    hipLaunchKernelGGL(crc32_frames_kernel<CrcMode::kVerify>, dim3((unsigned)grid), dim3(kBlockThreads),
                       0, stream, bytes, off, n, fpb, static_cast<const uint4*>(image), out);
  else
    hipLaunchKernelGGL(crc32_frames_kernel<CrcMode::kCrc>, dim3((unsigned)grid), dim3(kBlockThreads),
                       0, stream, bytes, off, n, fpb, static_cast<const uint4*>(image), out);
  return hipGetLastError();
}

}  // namespace lnx
