// stage_research.hip — RESEARCH LIBRARY ONLY (liblneto_amd_research.so,
// -DLNX_RESEARCH): the round-4 staged lane-stream variants 300-335 and the
// timing-only diagnostics, kept for tools/prof/variants.py
// and one parity test per live form (tests/test_stage.py).  The product
// kernel is stage_kernel.hip (the slicing-by-8 fold with the patched boundary
// word, variant 314, plus the round-5 dispatch, giant slices and the
// out-of-order fallback); nothing here is reachable from include/lneto_amd.h.
//
// stage_kernel.hip — batched CRC-32 / FCS verify by staged lane streams, gfx950
// (round 4).  Reference semantics: ethernet.CRC32 (lneto
// ethernet/crc.go:19-21) = Go crc32.Checksum(data, IEEETable); the verify mode
// is the residue form of the FCS check.  The schedule is restated on the host
// in tests/stage_algebra.py and checked there against zlib.
//
// Why: on short frames (the Zipf mix, mean 246 B) every per-frame window
// layout is bound by the L2 request rate (a line two frames share is asked for
// twice, a short frame's partial lines cost a request each).
// Here each line is requested once, whole, and a lane still folds a
// CONTIGUOUS byte stream, so a frame boundary costs no cross-lane work:
//
//  * a wave takes a block of kStageBF consecutive frames, bytes [A, E), and
//    cuts 64 stretches of Q bytes (Q a multiple of 128) from A rounded down to
//    128; lane k folds stretch k one dword at a time, r <- Z4(r ^ w), through
//    lane-private slicing-by-2 tables (Z4 = Z2 o Z2, Z2(v) = (v >> 16) ^
//    A[v & 0xFF] ^ B[(v >> 8) & 0xFF]; 64 KiB instead of the 128 KiB of
//    slicing-by-4, which leaves LDS for the staging);
//  * per round each lane needs its stretch's next 128-byte line: 8
//    buffer_load_dwordx4, instruction m / lane t reading piece
//    ((t & 7) - s) & 7 of stretch s = 8 (t >> 3) + m, so every instruction
//    covers 8 whole lines; the pieces go to the wave's 8 KiB of LDS at
//    1024 m + 16 t and lane s reads its line back with 8 ds_read_b128 at
//    1024 (s & 7) + 128 (s >> 3) + 16 ((i + s) & 7), conflict-free;
//  * a boundary x (an offset of the block) in the dword at 4d, byte c:
//    e = r ^ (w & lomask(c)), the ending frame's state is Z_c(e) (its CRC the
//    complement); r <- Z4((w & ~lomask(c)) ^ K_c), K_c = Z_{-c}(~0), is the
//    new frame's state after the dword from the CRC init.  One boundary per
//    64-byte half is handled by selects inside the fold; a half where some
//    lane has two (frames under 64 bytes, empty frames) runs byte by byte;
//  * a stretch starts inside a frame: its first boundary's state is local.
//    After the block, P_k (the true register at stretch k's start) is the
//    previous lane's end register (or, past a frame longer than a stretch,
//    Z_Q(P_{k-1}) ^ E_{k-1}), and the first frame's state gains Z_d(P_k),
//    d = x - S_k, by binary powers Z_{2^m} from shared nibble tables.
#ifdef LNX_RESEARCH
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lnx {
namespace rs {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

enum class StageMode : int { kCrc = 0, kVerify = 1 };

constexpr uint32_t kStageBF = 382;  // frames per block: the boundary list (bf + 1 + 2 sentinels) fits 384 dwords
constexpr uint32_t kStageBFBig = 766;  // variants 308 / 309: 768-dword lists, half the per-block overhead
constexpr uint32_t kStageBFSmall = 190, kStageBFMid = 254;  // variants 318-321: shorter blocks, a shorter tail
constexpr uint32_t kStageBF510 = 510;  // variants 324 / 325: the longest lists that leave the nibble tables in LDS
// LDS layout (bytes) for W waves per workgroup.  W = 8: the Z_{2^m} nibble
// tables live in LDS too; W = 10 (variants 304-307): they are read from the
// image in HBM (only the carries use them, once per stretch), which frees the
// room for two more waves' transposes and lists.
constexpr uint32_t kSTab = 0;  // A (Z_2) / B (Z_1): e << 8 | m << 7 | c << 2
template <int W, uint32_t BF = kStageBF, uint32_t ZXB = 0>
struct StageLds {
  static_assert((BF + 2) % 64 == 0, "whole-wave list loads");
  static constexpr uint32_t kList = (BF + 2) * 4;      // boundary list bytes per wave (bf + 1 entries + sentinel)
  static constexpr uint32_t kTr = 65536;               // transposes: 8 KiB per wave
  static constexpr uint32_t kBnd = kTr + W * 8192;     // boundary lists
  // ZXB bytes of shared single-column byte tables after the lists: Z_16, Z_32,
  // Z_64 (DEFER, variants 312 / 313, 12 KiB) or Z_8, Z_16, Z_24, Z_32 (two
  // chains per half, variants 316 / 317, 16 KiB); the nibble tables then
  // stay in HBM
  static constexpr uint32_t kZx = kBnd + W * kList;
  static constexpr uint32_t kZxBytes = ZXB;
  static constexpr bool kNibInLds = ZXB == 0 && kBnd + W * kList + 31 * 512 + 16 <= 163840;
  static constexpr uint32_t kNib = kZx + kZxBytes;     // Z_{2^m}, m = 0..30: (m, i, v) at 512 m + 64 i + 4 v
  static constexpr uint32_t kCtr = kNib + (kNibInLds ? 31 * 512 : 0);  // the workgroup's block counter
  static constexpr uint32_t kBytes = kCtr + 16;
  static_assert(kBytes <= 163840, "stage LDS");
};
// compact image in HBM (api.cpp build_stage_image): A[256], B[256], then the
// nibble tables verbatim (512 + 31 * 128 dwords), then (FOLD 4) the four Z_4
// byte tables, table k entry e at kStageZ4Img + 256 k + e
constexpr uint32_t kStageZ4Img = 512 + 31 * 128;
// then (FOLD 8) the eight slicing-by-8 byte tables T8_k[e] = Z_{8-k}(e), table
// k entry e at kStageZ8Img + 256 k + e
constexpr uint32_t kStageZ8Img = kStageZ4Img + 1024;
// then (DEFER) Z_16, Z_32, Z_64 as four byte tables each: (t, k, e) at kStageZxImg + 1024 t + 256 k + e
constexpr uint32_t kStageZxImg = kStageZ8Img + 2048;
// then (two chains per half) Z_8, Z_16, Z_24, Z_32: (t, k, e) at kStageZyImg + 1024 t + 256 k + e = Z_{8(t+1)}(e << 8k)
constexpr uint32_t kStageZyImg = kStageZxImg + 3072;

constexpr uint32_t kSOOB = 0x80000000u;
constexpr uint32_t kSNone = 0xFFFFFFFFu;

__device__ __forceinline__ uint32_t s_lds(const char* lds, uint32_t a) {
  return *reinterpret_cast<const uint32_t*>(lds + a);
}
// Z_2(v) through the lane-private tables (b0 = this lane's column << 2)
__device__ __forceinline__ uint32_t s_z2(const char* lds, uint32_t v, uint32_t b0) {
  const uint32_t a = __builtin_amdgcn_perm(v, b0, 0x0c020400u), b = __builtin_amdgcn_perm(v, b0, 0x0c020500u);
  return __builtin_amdgcn_bitop3_b32(v >> 16, s_lds(lds, kSTab + a), s_lds(lds, kSTab + b + 128u), 0x96);
}
// FOLD 2: Z_1 is table B.  FOLD 4 (variants 302 / 303): the four Z_4 byte
// tables in 16 bank columns, entry e of table k, column c at e << 8 | k << 6 |
// c << 2 (64 KiB like FOLD 2's), one LDS round trip per dword instead of two;
// Z_1 is its table 3 (Z_4(e << 24) = Z_1(e)).  Lanes c and c + 16 share column
// c, and table k sits in bank half k & 1, so the k-th lookup of lane half h =
// (lane >> 4) & 1 reads table (k + h) & 3: in every instruction the two halves
// of a 32-lane pass read opposite bank halves (conflict-free; the XOR of the
// four lookups does not depend on their order).
template <int FOLD>
__device__ __forceinline__ uint32_t s_z1(const char* lds, uint32_t v, uint32_t b0) {
  return (v >> 8) ^
         s_lds(lds, kSTab + __builtin_amdgcn_perm(v, b0, 0x0c020400u) + (FOLD == 8 ? 224u : FOLD == 4 ? 192u : 128u));
}
// FOLD 8 (variants 310 / 311): slicing-by-8 over 8-byte units, the eight byte
// tables T8_k[e] = Z_{8-k}(e) in 8 bank columns, entry e of table k, column c
// at e << 8 | k << 5 | c << 2 (64 KiB).  A unit (w0, w1) entered with r leaves
// Z_8(r ^ w0) ^ Z_4(w1) = XOR_k T8_k[byte k of r ^ w0] ^ XOR_k T8_{4+k}[byte k
// of w1]: the w1 half is off the chain, so a lane's chain takes one LDS round
// trip per 8 bytes.  Table k sits in bank octet k & 3; the four 8-lane groups
// g = (lane >> 3) & 3 of a pass read tables (i + g) & 3 (and 4 + that) in
// lookup i, so each lookup instruction is conflict-free.
struct Z8Lane {
  uint32_t base[8], sel[4];  // base[i] (table (i + g) & 3), base[4 + i] (table 4 + ((i + g) & 3))
  __device__ explicit Z8Lane(uint32_t lane) {
    const uint32_t g = (lane >> 3) & 3u, c = lane & 7u;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t k = (i + g) & 3u;
      base[i] = (k << 5) | (c << 2);
      base[4 + i] = ((4u + k) << 5) | (c << 2);
      sel[i] = 0x0c020400u + (k << 8);
    }
  }
};
// XOR_k T8_{4h+k}[byte k of v]: h = 0 the r-side half of Z_8, h = 1 Z_4(v)
__device__ __forceinline__ uint32_t s_z8half(const char* lds, uint32_t v, const Z8Lane& z8, uint32_t h) {
  uint32_t y[4];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) y[i] = s_lds(lds, kSTab + __builtin_amdgcn_perm(v, z8.base[4 * h + i], z8.sel[i]));
  return __builtin_amdgcn_bitop3_b32(y[0], y[1], y[2], 0x96) ^ y[3];
}
// a whole unit: Z_8(v0) ^ Z_4(v1), the eight lookups folded in four ops (the
// v1 side, off the chain, first)
__device__ __forceinline__ uint32_t s_z8unit(const char* lds, uint32_t v0, uint32_t v1, const Z8Lane& z8) {
  uint32_t y[8];
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) y[4 + i] = s_lds(lds, kSTab + __builtin_amdgcn_perm(v1, z8.base[4 + i], z8.sel[i]));
#pragma unroll
  for (uint32_t i = 0; i < 4; ++i) y[i] = s_lds(lds, kSTab + __builtin_amdgcn_perm(v0, z8.base[i], z8.sel[i]));
  const uint32_t t = __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(y[4], y[5], y[6], 0x96), y[7], y[0], 0x96);
  return __builtin_amdgcn_bitop3_b32(t, y[1], y[2], 0x96) ^ y[3];
}
// the FOLD 4 lookups' per-lane v_perm bases / selectors: lookup i reads table
// k = (i + h) & 3 at byte (v.byte_k << 8) | (k << 6) | (c << 2)
struct Z4Lane {
  uint32_t base[4], sel[4];
  __device__ explicit Z4Lane(uint32_t lane) {
    const uint32_t h = (lane >> 4) & 1u, c = lane & 15u;
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) {
      const uint32_t k = (i + h) & 3u;
      base[i] = (k << 6) | (c << 2);
      sel[i] = 0x0c020400u + (k << 8);
    }
  }
};
// Z_4(v)
template <int FOLD>
__device__ __forceinline__ uint32_t s_z4(const char* lds, uint32_t v, uint32_t b0, const Z4Lane& zl) {
  if constexpr (FOLD == 4) {
    uint32_t y[4];
#pragma unroll
    for (uint32_t i = 0; i < 4; ++i) y[i] = s_lds(lds, kSTab + __builtin_amdgcn_perm(v, zl.base[i], zl.sel[i]));
    return __builtin_amdgcn_bitop3_b32(y[0], y[1], y[2], 0x96) ^ y[3];
  } else {
    return s_z2(lds, s_z2(lds, v, b0), b0);
  }
}

// Z_{2^m}(v) through the shared nibble tables (every lane reads table m: a
// nibble value picks one of 16 banks, equal values broadcast), from LDS or,
// for W > 8, from the image in HBM (dword (m, i, v) at 512 + 128 m + 16 i + v)
template <class LY>
__device__ __forceinline__ uint32_t s_zpow2(const char* lds, const uint32_t* image, uint32_t m, uint32_t v) {
  uint32_t a = 0;
  if constexpr (LY::kNibInLds) {
    const uint32_t t = LY::kNib + 512u * m;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) a ^= s_lds(lds, t + 64u * i + (__builtin_amdgcn_ubfe(v, 4 * i, 4) << 2));
  } else {
    const uint32_t* t = image + 512u + 128u * m;
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i) a ^= t[16u * i + __builtin_amdgcn_ubfe(v, 4 * i, 4)];
  }
  return a;
}
// Z_d(v), d < 2^31, by binary powers; lanes whose d is done keep their value
template <class LY>
__device__ __forceinline__ uint32_t s_zd(const char* lds, const uint32_t* image, uint32_t d, uint32_t v) {
  for (uint32_t m = 0; __builtin_amdgcn_ballot_w64((d >> m) != 0u) != 0; ++m) {
    const uint32_t z = s_zpow2<LY>(lds, image, m, v);
    v = ((d >> m) & 1u) ? z : v;
  }
  return v;
}

// K_c = Z_{-c}(0xFFFFFFFF): (w & ~lomask(c)) ^ K_c folded by Z4 is the state,
// after the dword, of a frame that starts at its byte c
constexpr uint32_t s_unz(uint32_t v, int nbytes) {
  for (int i = 0; i < 8 * nbytes; ++i) {
    const uint32_t b = v >> 31, t = b ? v ^ 0xEDB88320u : v;
    v = (t << 1) | b;
  }
  return v;
}
constexpr uint32_t kK1 = s_unz(0xFFFFFFFFu, 1), kK2 = s_unz(0xFFFFFFFFu, 2), kK3 = s_unz(0xFFFFFFFFu, 3);

template <StageMode MODE, int FOLD, int W, uint32_t BF = kStageBF, bool DEFER = false, int PATCH = 0>
__global__ void __launch_bounds__(W * 64, 1)
crc32_stage_rs_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t nframes,
                   uint64_t frames_per_wg, const uint32_t* __restrict__ image, void* __restrict__ out) {
  using LY = StageLds<W, BF, DEFER ? 3u * 4096u : PATCH == 2 ? 4u * 4096u : 0u>;
  static_assert(!DEFER || FOLD == 8, "the deferred correction runs on the slicing-by-8 fold");
  static_assert(PATCH == 0 || (FOLD == 8 && !DEFER), "the patched boundary word runs on the slicing-by-8 fold");
  // PATCH: 1 the patched boundary word (the product form), 2 two chains per
  // half, 3 offsets prefetched, 4-7 and 8 / 9 timing-only diagnostics
  constexpr uint32_t kLast = BF + 1;  // the list's last entry (a sentinel past bf)
  constexpr uint32_t kThreads = W * 64;
  __shared__ __attribute__((aligned(16))) char lds[LY::kBytes];
  // ---- image: A / B values expanded into their 32 bank columns (FOLD 4: the
  // Z_4 values into 16), nibble tables verbatim
  {
    const uint32_t t = threadIdx.x;
    if constexpr (FOLD == 8) {
      for (uint32_t vi = t; vi < 2048u; vi += kThreads) {
        const uint32_t v = image[kStageZ8Img + vi];
        uint4* row = reinterpret_cast<uint4*>(lds + kSTab + ((vi & 255u) << 8) + ((vi >> 8) << 5));
        const uint4 v4 = {v, v, v, v};
        row[0] = v4;
        row[1] = v4;
      }
    } else if constexpr (FOLD == 4) {
      for (uint32_t vi = t; vi < 1024u; vi += kThreads) {
        const uint32_t v = image[kStageZ4Img + vi];
        uint4* row = reinterpret_cast<uint4*>(lds + kSTab + ((vi & 255u) << 8) + ((vi >> 8) << 6));
        const uint4 v4 = {v, v, v, v};
#pragma unroll
        for (int i = 0; i < 4; ++i) row[(i + vi) & 3u] = v4;
      }
    } else {
      for (uint32_t vi = t; vi < 512u; vi += kThreads) {
        const uint32_t v = image[vi];
        const uint32_t m = vi >> 8, e = vi & 255u;
        uint4* row = reinterpret_cast<uint4*>(lds + kSTab + (e << 8) + (m << 7));
        const uint4 v4 = {v, v, v, v};
#pragma unroll
        for (int i = 0; i < 8; ++i) row[(i + vi) & 7u] = v4;
      }
    }
    if constexpr (LY::kNibInLds)
      for (uint32_t i = t; i < 31u * 128u; i += kThreads)
        reinterpret_cast<uint32_t*>(lds + LY::kNib)[i] = image[512 + i];
    if constexpr (LY::kZxBytes != 0)
      for (uint32_t i = t; i < LY::kZxBytes / 4u; i += kThreads)
        reinterpret_cast<uint32_t*>(lds + LY::kZx)[i] = image[(DEFER ? kStageZxImg : kStageZyImg) + i];
    if (t == 0) *reinterpret_cast<uint32_t*>(lds + LY::kCtr) = 0;
  }
  __syncthreads();
  const uint64_t fb0 = (uint64_t)blockIdx.x * frames_per_wg;
  if (fb0 >= nframes) return;
  const uint64_t fb1 = fb0 + frames_per_wg < nframes ? fb0 + frames_per_wg : nframes;
  const uint32_t nslice = (uint32_t)(fb1 - fb0);
  const uint32_t lane = threadIdx.x & 63u, wv = threadIdx.x >> 6;
  const uint32_t b0 = (lane & (FOLD == 8 ? 7u : FOLD == 4 ? 15u : 31u)) << 2;
  const Z8Lane z8(lane);
  const Z4Lane zl(lane);
  char* tr = lds + LY::kTr + 8192u * wv;
  uint32_t* list = reinterpret_cast<uint32_t*>(lds + LY::kBnd + LY::kList * wv);
  constexpr uint32_t elem = MODE == StageMode::kCrc ? 4u : 1u;
  const __amdgpu_buffer_rsrc_t out_rsrc = __builtin_amdgcn_make_buffer_rsrc(
      reinterpret_cast<char*>(out) + fb0 * elem, (short)0, (int)(nslice * elem), 0x00020000);
  // this lane's read-back addresses: piece i of its line at rb + 16 ((i + lane) & 7)
  const uint32_t rb = 1024u * (lane & 7u) + 128u * (lane >> 3), rot = lane & 7u;

  auto grab = [&]() -> uint32_t {
    uint32_t b = 0;
    if (lane == 0) b = __hip_atomic_fetch_add(reinterpret_cast<uint32_t*>(lds + LY::kCtr), 1u, __ATOMIC_RELAXED,
                                              __HIP_MEMORY_SCOPE_WORKGROUP);
    return (uint32_t)__builtin_amdgcn_readfirstlane((int)b);
  };
  // PF (variants 322 / 323): the next block's offsets (its boundary list, A
  // and E among them) are loaded while this block folds.  The loads are inline
  // asm, so hipcc neither waits for them early nor counts them; the ring's
  // vmcnt(0) at the block end (and once before the first block) makes them
  // ready, and that asm names them as operands, so no use moves above it.
  // They are older than every ring operation, so the ring's static vmcnt(10)
  // still covers its slot.
  constexpr bool PF = PATCH == 3;
  constexpr uint32_t kNL = (BF + 2) / 64;
  static_assert(!PF || kNL == 6, "the prefetch asm names six offsets per lane");
  uint64_t pre[6] = {0, 0, 0, 0, 0, 0};
  auto prefetch = [&](uint32_t b) {
    const uint64_t fr = (uint64_t)b * BF;
    const uint32_t bfx = fr < nslice ? (uint32_t)(nslice - fr < BF ? nslice - fr : BF) : 0u;
    const uint64_t* p0 = off + fb0 + (fr < nslice ? fr : 0u);  // (past the slice: entry fb0, a valid address)
#pragma unroll
    for (uint32_t i = 0; i < 6; ++i) {
      const uint32_t jj = lane + 64u * i;
      const uint64_t* p = p0 + (jj <= bfx ? jj : bfx);
      asm volatile("global_load_dwordx2 %0, %1, off" : "=&v"(pre[i]) : "v"(p));
    }
  };
  auto pre_ready = [&]() {
    asm volatile("s_waitcnt vmcnt(0)"
                 : "+v"(pre[0]), "+v"(pre[1]), "+v"(pre[2]), "+v"(pre[3]), "+v"(pre[4]), "+v"(pre[5]));
  };
  uint32_t blk_pf = 0;
  if constexpr (PF) {
    blk_pf = grab();
    prefetch(blk_pf);
    pre_ready();
  }

  for (;;) {
    const uint32_t blk = PF ? blk_pf : grab();
    const uint64_t f0r = (uint64_t)blk * BF;  // relative to fb0
    if (f0r >= nslice) break;
    const uint32_t bf = (uint32_t)(nslice - f0r < BF ? nslice - f0r : BF);
    const uint64_t f0 = fb0 + f0r;
    uint64_t A, E;
    if constexpr (PF) {
      uint64_t ev = pre[0];
#pragma unroll
      for (uint32_t i = 1; i < 6; ++i) ev = (bf >> 6) == i ? pre[i] : ev;
      const uint32_t el = bf & 63u;
      A = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)pre[0], 0) |
          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(pre[0] >> 32), 0) << 32);
      E = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)ev, (int)el) |
          ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(ev >> 32), (int)el) << 32);
    } else {
      A = off[f0], E = off[f0 + bf];
    }
    const uint8_t* pa = bytes + A;
    const uint32_t adj = (uint32_t)(reinterpret_cast<uintptr_t>(pa) & 127u);
    const uint64_t span = E > A ? E - A + adj : adj;
    // ---- boundary list (relative to the line-aligned base): x_j = off[f0 + j] - A + adj
#pragma unroll
    for (uint32_t i = 0; i < (BF + 2) / 64; ++i) {  // (whole-wave loads: entry j > bf re-reads entry bf)
      const uint32_t j = lane + 64u * i;
      const uint64_t o = PF ? pre[i] : off[f0 + (j <= bf ? j : bf)];
      const uint32_t x = o > A ? (uint32_t)(o - A) + adj : adj;  // (non-decreasing offsets: o >= A)
      list[j] = j <= bf ? x : kSNone;
    }
    if constexpr (PF) {
      blk_pf = grab();
      prefetch(blk_pf);
    }
    __builtin_amdgcn_wave_barrier();
    if (span >= (1ull << 31) - 65536) {
      // gigabyte frames: byte-serial fold per frame, one lane per frame
      // (the byte loop runs with the whole wave active: a lane past its frame
      // re-reads byte A and keeps its register, so no load issues under
      // narrowed exec — the audit's loop rule)
      for (uint32_t j0 = 0; j0 < bf; j0 += 64u) {
        const uint32_t j = j0 + lane;
        uint32_t r = 0xFFFFFFFFu;
        const uint64_t s = j < bf ? off[f0 + j] : A, e0 = j < bf ? off[f0 + j + 1] : A;
        const uint64_t e = e0 > s ? e0 : s;
        for (uint64_t q = s;; ++q) {
          const bool act = q < e;
          if (__builtin_amdgcn_ballot_w64(act) == 0) break;
          const uint32_t b = bytes[act ? q : A];
          const uint32_t nr = s_z1<FOLD>(lds, r ^ b, b0);
          r = act ? nr : r;
        }
        if (j < bf) {
          const uint32_t crc = ~r;
          const uint32_t v = MODE == StageMode::kCrc ? crc : (uint32_t)(e - s >= 4 && crc == 0x2144DF1Cu);
          if (MODE == StageMode::kCrc)
            __builtin_amdgcn_raw_buffer_store_b32(v, out_rsrc, (uint32_t)(f0r + j) * 4u, 0, 0);
          else
            __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, out_rsrc, (uint32_t)(f0r + j), 0, 0);
        }
      }
      if constexpr (PF) pre_ready();
      continue;
    }
    const uint32_t sp = (uint32_t)span;
    // 64 Q > sp: the block's last boundary (at sp) must lie inside a stretch
    uint32_t Q = ((sp + 64u) / 64u + 127u) & ~127u;
    Q = Q < 128u ? 128u : Q;
    const uint32_t rounds = Q / 128u;
    // the range rounded up to whole 16-byte pieces: a load that straddles the
    // range end reads as 0, and the block's last frame ends in it (the bytes
    // past E only feed states past the last boundary; the base is 128-aligned,
    // so the piece holding E's last byte never crosses a page)
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(pa - adj), (short)0,
                                                                        (int)((sp + 15u) & ~15u), 0x00020000);
    // load offsets: instruction m reads stretch s = 8 (lane >> 3) + m, piece ((lane & 7) - s) & 7
    uint32_t lo_m[8];
#pragma unroll
    for (uint32_t m = 0; m < 8; ++m) {
      const uint32_t s = 8u * (lane >> 3) + m;
      lo_m[m] = s * Q + 16u * (((lane & 7u) - s) & 7u);
    }
    // Streaming loads are inline asm (hipcc neither counts them nor merges
    // their waits across the fold's branches into vmcnt(0)): every round
    // issues exactly 8 of them (rounds past the stretch get an offset past
    // the range: no memory traffic) after exactly 2 result stores, so the wait
    // for a slot is a static vmcnt(10).  The statement opens with s_nop 4 (a
    // descriptor SGPR restored by VALU needs 5 wait states before a VMEM
    // instruction reads it), outputs early-clobber.
    auto issue = [&](u32x4(&b)[8], uint32_t rr) {
      const uint32_t so = rr < rounds ? rr * 128u : kSOOB;
      asm volatile(
          "s_nop 4\n\t"
          "buffer_load_dwordx4 %0, %8, %16, %17 offen\n\t"
          "buffer_load_dwordx4 %1, %9, %16, %17 offen\n\t"
          "buffer_load_dwordx4 %2, %10, %16, %17 offen\n\t"
          "buffer_load_dwordx4 %3, %11, %16, %17 offen\n\t"
          "buffer_load_dwordx4 %4, %12, %16, %17 offen\n\t"
          "buffer_load_dwordx4 %5, %13, %16, %17 offen\n\t"
          "buffer_load_dwordx4 %6, %14, %16, %17 offen\n\t"
          "buffer_load_dwordx4 %7, %15, %16, %17 offen"
          : "=&v"(b[0]), "=&v"(b[1]), "=&v"(b[2]), "=&v"(b[3]), "=&v"(b[4]), "=&v"(b[5]), "=&v"(b[6]), "=&v"(b[7])
          : "v"(lo_m[0]), "v"(lo_m[1]), "v"(lo_m[2]), "v"(lo_m[3]), "v"(lo_m[4]), "v"(lo_m[5]), "v"(lo_m[6]),
            "v"(lo_m[7]), "s"(rs), "s"(so));
    };
    // results of the fast halves, held to the next round's flush (one per half)
    uint32_t hv0 = 0, hf0 = kSOOB, hv1 = 0, hf1 = kSOOB;
    auto store = [&](uint32_t v, uint32_t at) {
      if constexpr (MODE == StageMode::kCrc)
        __builtin_amdgcn_raw_buffer_store_b32(v, out_rsrc, at, 0, 0);
      else
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)v, out_rsrc, at, 0, 0);
    };
    // exactly two stores per flush, in asm so that hipcc cannot merge or drop
    // them (the ring's vmcnt(10) counts them)
    auto flush = [&]() {
      if constexpr (MODE == StageMode::kCrc)
        asm volatile("buffer_store_dword %0, %1, %4, 0 offen\n\tbuffer_store_dword %2, %3, %4, 0 offen"
                     ::"v"(hv0), "v"(hf0), "v"(hv1), "v"(hf1), "s"(out_rsrc) : "memory");
      else
        asm volatile("buffer_store_byte %0, %1, %4, 0 offen\n\tbuffer_store_byte %2, %3, %4, 0 offen"
                     ::"v"(hv0), "v"(hf0), "v"(hv1), "v"(hf1), "s"(out_rsrc) : "memory");
      hf0 = hf1 = kSOOB;
    };
    // the block's first two rounds go out before the boundary search
    u32x4 buf0[8], buf1[8];
    flush();  // (two stores, so that the first waits count alike)
    issue(buf0, 0);
    flush();
    issue(buf1, 1);
    // ---- this lane's stretch [Sk, Sk + Q) and its first boundary j = lower_bound(list, Sk)
    const uint32_t Sk = lane * Q;
    uint32_t lo = 0, hi = bf + 1u;
    while (__builtin_amdgcn_ballot_w64(lo < hi) != 0) {
      const uint32_t mid = (lo + hi) >> 1;
      const uint32_t xm = list[mid < kLast ? mid : kLast];
      if (lo < hi) {
        if (xm >= Sk) hi = mid; else lo = mid + 1u;
      }
    }
    const uint32_t jstart = lo;
    uint32_t j = lo;
    // the lane's next three boundaries: x (due), x1 (the slow-half test), x2
    // (read one advance ahead, so that an advance never waits for the list)
    uint32_t x = list[j], x1 = list[j + 1u < kLast ? j + 1u : kLast];  // (j = bf + 1 past the block end)
    uint32_t x2 = list[j + 2u < kLast ? j + 2u : kLast];
    uint32_t xprev = j > 0 ? list[j - 1u] : 0u;
    uint32_t r = 0;
    bool first = true;
    uint32_t rec_j = 0, rec_S = 0, rec_d = 0;  // the first boundary's frame (carry pending)
    bool rec = false;
    // the end of the frame at boundary j (state S, at position xe): a result,
    // or the stretch's first frame, held until the carries are known; the
    // result goes to the half's hold (slot h) or, in a byte-serial half, out at once
    auto end_at = [&](bool ev, uint32_t S, uint32_t xe, int h) {
      const bool is_first = ev && first && j > 0;
      rec_j = is_first ? j : rec_j;
      rec_S = is_first ? S : rec_S;
      rec_d = is_first ? xe - Sk : rec_d;
      rec = rec || is_first;
      const bool res = ev && !first && j > 0;
      first = ev ? false : first;
      const uint32_t crc = ~S;
      const uint32_t fr = (uint32_t)f0r + j - 1u;
      const uint32_t val = MODE == StageMode::kCrc ? crc : ((xe - xprev >= 4u && crc == 0x2144DF1Cu) ? 1u : 0u);
      const uint32_t at = res ? fr * elem : kSOOB;
      if (h == 0) {
        hv0 = res ? val : hv0, hf0 = res ? at : hf0;
      } else if (h == 1) {
        hv1 = res ? val : hv1, hf1 = res ? at : hf1;
      } else {
        store(val, at);
      }
    };
    auto advance = [&](bool ev) {
      xprev = ev ? x : xprev;
      j = ev ? j + 1u : j;
      x = ev ? x1 : x;
      x1 = ev ? x2 : x1;
      const uint32_t x3 = list[j + 2u < kLast ? j + 2u : kLast];
      x2 = ev ? x3 : x2;
    };

    // one round: wait for the slot, stage its pieces in LDS, flush the held
    // results, refill the slot two rounds ahead, fold the lane's line in two
    // 64-byte halves
    auto round_step = [&](u32x4(&cur)[8], uint32_t rr) {
      asm volatile("s_waitcnt vmcnt(10)"
                   : "+v"(cur[0]), "+v"(cur[1]), "+v"(cur[2]), "+v"(cur[3]), "+v"(cur[4]), "+v"(cur[5]),
                     "+v"(cur[6]), "+v"(cur[7]));
      if constexpr (PATCH == 8) {  // (variant 340, timing only: the ring's loads alone)
        uint32_t a = r;
#pragma unroll
        for (int m = 0; m < 8; ++m) a ^= cur[m][0] ^ cur[m][1] ^ cur[m][2] ^ cur[m][3];
        r = a;
        flush();
        issue(cur, rr + 2u);
        return;
      }
      if constexpr (PATCH != 4)  // (variant 328, timing only: the lines read back stale)
#pragma unroll
        for (int m = 0; m < 8; ++m) *reinterpret_cast<u32x4*>(tr + 1024 * m + 16u * lane) = cur[m];
      flush();
      issue(cur, rr + 2u);
      if constexpr (PATCH == 9) {  // (variant 342, timing only: loads + the LDS transpose, written and read back)
        uint32_t a = r;
#pragma unroll
        for (uint32_t i = 0; i < 8; ++i) {
          const u32x4 q = *reinterpret_cast<const u32x4*>(tr + rb + 16u * ((i + rot) & 7u));
          a ^= q[0] ^ q[1] ^ q[2] ^ q[3];
        }
        r = a;
        return;
      }
      // the lane's whole line in one LDS round trip (both halves)
      u32x4 ql[8];
#pragma unroll
      for (uint32_t i = 0; i < 8; ++i) ql[i] = *reinterpret_cast<const u32x4*>(tr + rb + 16u * ((i + rot) & 7u));
#pragma unroll
      for (uint32_t h = 0; h < 2; ++h) {
        const u32x4* q = ql + 4 * h;
        const uint32_t P = Sk + 128u * rr + 64u * h;
        const uint32_t rel = x - P;
        const bool in = rel < 64u;
        if (__builtin_amdgcn_ballot_w64(x1 - P < 64u) != 0) {
          // two or more boundaries in some lane's half (frames under 64
          // bytes): byte by byte, the bytes re-read from the staged line (a
          // rolled loop: this path is rare and must not bloat the fast one)
#pragma nounroll
          for (uint32_t b = 0; b < 64u; ++b) {
            const uint32_t pi = 4u * h + (b >> 4);
            const uint32_t w = s_lds(tr, rb + 16u * ((pi + rot) & 7u) + (b & 12u));
            const uint32_t pos = P + b;
            while (__builtin_amdgcn_ballot_w64(x == pos) != 0) {
              const bool ev = x == pos;
              end_at(ev, r, x, 2);
              r = ev ? 0xFFFFFFFFu : r;
              advance(ev);
            }
            r = s_z1<FOLD>(lds, r ^ ((w >> (8u * (b & 3u))) & 0xFFu), b0);  // (one byte: Z_1 shifts r, not w)
          }
          continue;
        }
        const uint32_t kb = in ? rel >> 2 : 99u, c = rel & 3u;
        const uint32_t lm = in ? (uint32_t)((1ull << (8u * c)) - 1ull) : 0u;
        const uint32_t Kc = c == 0u ? 0xFFFFFFFFu : c == 1u ? kK1 : c == 2u ? kK2 : kK3;
        uint32_t ecap = 0;
        if constexpr (DEFER) {
          // no boundary selects in the fold: the plain fold, one capture of r
          // per 8-byte unit, and the boundary's effect added after the half
          // (r_true = r_plain ^ Z_{64 - 4d}(e ^ K_c))
          uint32_t rc = 0;
          const uint32_t ub = kb >> 1;
#pragma unroll
          for (uint32_t u = 0; u < 8; ++u) {
            const uint32_t w0 = q[u >> 1][(2u * u) & 3u], w1 = q[u >> 1][(2u * u + 1u) & 3u];
            rc = ub == u ? r : rc;
            r = s_z8half(lds, r ^ w0, z8, 0) ^ s_z8half(lds, w1, z8, 1);
          }
          if (__builtin_amdgcn_ballot_w64(in) != 0) {
            // the boundary unit's two words, from the staged line
            const uint32_t u = (kb >> 1) & 7u;
            const uint2 wp = *reinterpret_cast<const uint2*>(tr + rb + 16u * ((4u * h + (u >> 1) + rot) & 7u) +
                                                             8u * (u & 1u));
            const bool odd = kb & 1u;
            const uint32_t z4 = s_z8half(lds, rc ^ wp.x, z8, 1);  // the state before w1
            const uint32_t rd = odd ? z4 : rc;
            ecap = rd ^ ((odd ? wp.y : wp.x) & lm);
            // Z_{4m}(ecap ^ K_c), m = 16 - kb dwords, by binary powers: Z_4, Z_8
            // (the fold's tables), Z_16 / Z_32 / Z_64 (the shared tables)
            const uint32_t m = 16u - (kb & 15u);
            uint32_t z = ecap ^ Kc;
            z = (m & 1u) ? s_z8half(lds, z, z8, 1) : z;
            z = (m & 2u) ? s_z8half(lds, z, z8, 0) : z;
#pragma unroll
            for (uint32_t t = 0; t < 3; ++t) {
              const uint32_t* zt = reinterpret_cast<const uint32_t*>(lds + LY::kZx) + 1024u * t;
              const uint32_t zz = __builtin_amdgcn_bitop3_b32(zt[z & 0xFFu], zt[256u + ((z >> 8) & 0xFFu)],
                                                              zt[512u + ((z >> 16) & 0xFFu)], 0x96) ^
                                  zt[768u + (z >> 24)];
              z = (m & (4u << t)) ? zz : z;
            }
            r = in ? r ^ z : r;
          }
        } else if constexpr (PATCH == 2) {
          // the patched boundary word, and the half as two chains of four
          // units: A from r, B from 0 (independent: two LDS round trips in
          // flight per lane); after the half r = Z_32(A) ^ B, or B alone when
          // the boundary lies in B.  A boundary in B captured B's local state:
          // the true one adds Z_{8(u-4)}(A), read with Z_32(A) in one round
          // trip from the shared Z_8 / Z_16 / Z_24 / Z_32 tables
          const uint32_t ub = (kb >> 1) & 7u;
          const bool odd = (kb & 1u) != 0u;
          const uint2 wp = *reinterpret_cast<const uint2*>(tr + rb + 16u * ((4u * h + (ub >> 1) + rot) & 7u) +
                                                           8u * (ub & 1u));
          const uint32_t wb = __builtin_amdgcn_bitop3_b32(odd ? wp.y : wp.x, lm, Kc, 0x9A);
          const uint32_t wb0 = odd ? 0u : wb;
          const uint32_t kbu = kb >> 1;  // (49 in a lane without a boundary)
          uint32_t ra = r, rbv = 0, rc = 0;
#pragma unroll
          for (uint32_t u = 0; u < 4; ++u) {
            const uint32_t w0 = q[u >> 1][(2u * u) & 3u], w1 = q[u >> 1][(2u * u + 1u) & 3u];
            const uint32_t x0 = q[2 + (u >> 1)][(2u * u) & 3u], x1w = q[2 + (u >> 1)][(2u * u + 1u) & 3u];
            const bool au = kbu == u, a1 = au && odd;
            const bool bu = kbu == u + 4u, b1 = bu && odd;
            rc = au ? ra : bu ? rbv : rc;
            ra = s_z8unit(lds, au ? wb0 : ra ^ w0, a1 ? wb : w1, z8);
            rbv = s_z8unit(lds, bu ? wb0 : rbv ^ x0, b1 ? wb : x1w, z8);
          }
          const bool inb = kbu - 4u < 4u;
          const uint32_t* zy = reinterpret_cast<const uint32_t*>(lds + LY::kZx);
          const uint32_t zsel = 1024u * ((kbu - 5u) & 3u);  // Z_{8(u-4)} for u = 5..7
          uint32_t a32[4], ac[4];
#pragma unroll
          for (uint32_t k = 0; k < 4; ++k) {
            const uint32_t e = (ra >> (8u * k)) & 0xFFu;
            a32[k] = zy[3u * 1024u + 256u * k + e];
            ac[k] = zy[zsel + 256u * k + e];
          }
          const uint32_t z32 = __builtin_amdgcn_bitop3_b32(a32[0], a32[1], a32[2], 0x96) ^ a32[3];
          const uint32_t zc = __builtin_amdgcn_bitop3_b32(ac[0], ac[1], ac[2], 0x96) ^ ac[3];
          r = inb ? rbv : z32 ^ rbv;
          const uint32_t rct = inb ? rc ^ (kbu == 4u ? ra : zc) : rc;
          const uint32_t z4t = s_z8half(lds, rct ^ wp.x, z8, 1);
          ecap = odd ? z4t ^ (wp.y & lm) : rct ^ (wp.x & lm);
        } else if constexpr (PATCH == 1 || PATCH >= 3) {
          // the boundary word patched once per half, read back from the staged
          // line: (w & ~lm) ^ K_c; the boundary unit u = kb >> 1 then enters
          // (patch, w1) for a boundary in w0 and (0, patch) for one in w1 (Z_8(0)
          // = 0 drops r), so a unit costs one compare and two selects
          const uint32_t ub = (kb >> 1) & 7u;
          const bool odd = (kb & 1u) != 0u;
          const uint2 wp = *reinterpret_cast<const uint2*>(tr + rb + 16u * ((4u * h + (ub >> 1) + rot) & 7u) +
                                                           8u * (ub & 1u));
          const uint32_t wb = __builtin_amdgcn_bitop3_b32(odd ? wp.y : wp.x, lm, Kc, 0x9A);
          const uint32_t wb0 = odd ? 0u : wb;
          const uint32_t kbu = kb >> 1;  // (49 in a lane without a boundary)
          uint32_t rc = 0;
#pragma unroll
          for (uint32_t u = 0; u < 8; ++u) {
            const uint32_t w0 = q[u >> 1][(2u * u) & 3u], w1 = q[u >> 1][(2u * u + 1u) & 3u];
            const bool au = kbu == u, a1 = au && odd;
            rc = au ? r : rc;
            if constexpr (PATCH == 5)  // (variant 330, timing only: a two-op stand-in for the unit's lookups)
              r = __builtin_amdgcn_alignbit(au ? wb0 : r ^ w0, a1 ? wb : w1, 7) ^ (a1 ? wb : w1);
            else
              r = s_z8unit(lds, au ? wb0 : r ^ w0, a1 ? wb : w1, z8);
          }
          // (variant 332, timing only: the ending frame's capture and Z_c skipped)
          const uint32_t z4t = PATCH == 6 ? rc : s_z8half(lds, rc ^ wp.x, z8, 1);
          ecap = odd ? z4t ^ (wp.y & lm) : rc ^ (wp.x & lm);
        } else if constexpr (FOLD == 8) {
          // 8-byte units; the unit holding the boundary captures (r, w0, w1)
          uint32_t rc = 0, w0c = 0, w1c = 0;
#pragma unroll
          for (uint32_t u = 0; u < 8; ++u) {
            const uint32_t w0 = q[u >> 1][(2u * u) & 3u], w1 = q[u >> 1][(2u * u + 1u) & 3u];
            const bool a0 = 2u * u == kb, a1 = 2u * u + 1u == kb, au = a0 || a1;
            rc = au ? r : rc, w0c = au ? w0 : w0c, w1c = au ? w1 : w1c;
            const uint32_t v0 = a0 ? __builtin_amdgcn_bitop3_b32(w0, lm, Kc, 0x9A) : r ^ w0;
            const uint32_t v1 = a1 ? __builtin_amdgcn_bitop3_b32(w1, lm, Kc, 0x9A) : w1;
            const uint32_t yw = s_z8half(lds, v1, z8, 1);  // Z_4(v1): off the chain
            const uint32_t yr = s_z8half(lds, v0, z8, 0);
            r = (a1 ? 0u : yr) ^ yw;  // a new frame in w1 owes nothing to r
          }
          // the ending frame's state before Z_c: in w0, r ^ (w0 & lm); in w1,
          // Z_4(r ^ w0) ^ (w1 & lm) (Z_4 = the T8_4..7 half)
          const uint32_t z4t = s_z8half(lds, rc ^ w0c, z8, 1);
          ecap = (kb & 1u) ? z4t ^ (w1c & lm) : rc ^ (w0c & lm);
        } else {
#pragma unroll
          for (uint32_t d = 0; d < 16; ++d) {
            const uint32_t w = q[d >> 2][d & 3u];
            const bool at = d == kb;
            ecap = at ? __builtin_amdgcn_bitop3_b32(r, w, lm, 0x78) : ecap;    // r ^ (w & lm)
            const uint32_t vr = __builtin_amdgcn_bitop3_b32(w, lm, Kc, 0x9A);  // (w & ~lm) ^ Kc
            const uint32_t v = at ? vr : r ^ w;
            r = s_z4<FOLD>(lds, v, b0, zl);
          }
        }
        if (__builtin_amdgcn_ballot_w64(in) != 0) {
          uint32_t S = ecap;  // Z_c(e), c = 0..3
          if constexpr (PATCH == 6) {
          } else if constexpr (FOLD == 8) {
            // Z_c(e) = (e >> 8c) ^ XOR_{i<c} Z_{c-i}(byte i of e) = ... T8_{8-c+i}[byte i]
            uint32_t y[3];
#pragma unroll
            for (uint32_t i = 0; i < 3; ++i)
              y[i] = s_lds(lds, kSTab + __builtin_amdgcn_perm(ecap, b0, 0x0c020400u + (i << 8)) +
                                    (((8u - c + i) & 7u) << 5));
            const uint32_t sh = c == 0u ? ecap : ecap >> (8u * c);
            S = __builtin_amdgcn_bitop3_b32(sh, c > 0u ? y[0] : 0u, c > 1u ? y[1] : 0u, 0x96) ^ (c > 2u ? y[2] : 0u);
          } else if constexpr (FOLD == 4) {
            // one round trip: Z_c(e) = (e >> 8c) ^ XOR_{i<c} Z_{c-i}(byte i of e),
            // Z_m(b) = Z_4(b << 8 (4 - m)) = table 4 - m's entry b
            uint32_t y[3];
#pragma unroll
            for (uint32_t i = 0; i < 3; ++i)
              y[i] = s_lds(lds, kSTab + __builtin_amdgcn_perm(ecap, b0, 0x0c020400u + (i << 8)) +
                                    (((4u - c + i) & 3u) << 6));
            const uint32_t sh = c == 0u ? ecap : ecap >> (8u * c);
            S = __builtin_amdgcn_bitop3_b32(sh, c > 0u ? y[0] : 0u, c > 1u ? y[1] : 0u, 0x96) ^ (c > 2u ? y[2] : 0u);
          } else {
#pragma unroll
            for (uint32_t s = 0; s < 3; ++s) {
              const uint32_t z = s_z1<FOLD>(lds, S, b0);
              S = s < c ? z : S;
            }
          }
          end_at(in, S, x, (int)h);
          advance(in);
        }
      }
    };
    for (uint32_t rr = 0; rr < rounds; rr += 2) {
      round_step(buf0, rr);
      if (rr + 1u < rounds) round_step(buf1, rr + 1u);
    }
    flush();
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(buf0[0]), "+v"(buf0[1]), "+v"(buf0[2]), "+v"(buf0[3]), "+v"(buf0[4]),
                 "+v"(buf0[5]), "+v"(buf0[6]), "+v"(buf0[7]));
    if constexpr (PF) asm volatile("" : "+v"(pre[0]), "+v"(pre[1]), "+v"(pre[2]), "+v"(pre[3]), "+v"(pre[4]), "+v"(pre[5]));
    asm volatile("" : "+v"(buf1[0]), "+v"(buf1[1]), "+v"(buf1[2]), "+v"(buf1[3]), "+v"(buf1[4]), "+v"(buf1[5]),
                 "+v"(buf1[6]), "+v"(buf1[7]));
    if constexpr (PATCH == 7) {  // (variant 334, timing only: no carries)
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    // ---- carries: the true register at each stretch's start
    const uint32_t E1 = r;
    const bool hb = j > jstart;  // this stretch holds a boundary
    const uint32_t up = ((lane + 63u) & 63u) << 2;
    const uint32_t Ep = (uint32_t)__builtin_amdgcn_ds_bpermute((int)up, (int)E1);
    // (evaluated by every lane: under `lane == 0 || ...` hipcc runs the
    // bpermute with lane 0 masked off, and a read from an inactive lane
    // returns 0, so lane 1 saw "no boundary" in lane 0)
    const int hbv = __builtin_amdgcn_ds_bpermute((int)up, (int)hb);
    const bool hbp = (lane == 0) | (hbv != 0);
    uint32_t Pk = Ep;
    if (__builtin_amdgcn_ballot_w64(rec && !hbp) != 0) {
      // a frame longer than a stretch: P_k = Z_Q(P_{k-1}) ^ E_{k-1} through
      // stretches without a boundary (Jacobi sweeps until nothing changes)
      for (uint32_t it = 0; it < 64u; ++it) {
        const uint32_t Pp = (uint32_t)__builtin_amdgcn_ds_bpermute((int)up, (int)Pk);
        const uint32_t zq = s_zd<LY>(lds, image, hbp ? 0u : Q, Pp);
        const uint32_t Pn = hbp ? Ep : zq ^ Ep;
        const bool ch = Pn != Pk;
        Pk = Pn;
        if (__builtin_amdgcn_ballot_w64(ch) == 0) break;
      }
    }
    if (__builtin_amdgcn_ballot_w64(rec) != 0) {
      const uint32_t S = rec_S ^ s_zd<LY>(lds, image, rec ? rec_d : 0u, Pk);
      const uint32_t crc = ~S;
      const uint32_t fr = (uint32_t)f0r + rec_j - 1u;
      if constexpr (MODE == StageMode::kCrc) {
        __builtin_amdgcn_raw_buffer_store_b32(crc, out_rsrc, rec ? fr * 4u : kSOOB, 0, 0);
      } else {
        const uint32_t xa = list[rec_j > 0 ? rec_j - 1u : 0u], xe = list[rec_j];
        const uint32_t ok = (xe - xa >= 4u && crc == 0x2144DF1Cu) ? 1u : 0u;
        __builtin_amdgcn_raw_buffer_store_b8((uint8_t)ok, out_rsrc, rec ? fr : kSOOB, 0, 0);
      }
    }
    __builtin_amdgcn_wave_barrier();  // the list is rewritten by the next block
  }
}

hipError_t launch_crc32_stage_research(const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out, bool verify,
                              int fold, int waves, const void* image, int num_cus, hipStream_t stream,
                              bool big_blocks) {
  if (n == 0) return hipSuccess;
  const uint64_t bfl = big_blocks ? kStageBFBig : fold == 12 ? kStageBFSmall : fold == 13 ? kStageBFMid
                                                                            : fold == 15 ? kStageBF510 : kStageBF;
  uint64_t grid = (n + bfl - 1) / bfl;
  if (grid > (uint64_t)num_cus) grid = (uint64_t)num_cus;
  const uint64_t per = (n + grid - 1) / grid;
  const uint32_t* img = static_cast<const uint32_t*>(image);
#define LNX_STAGE(M, F, W, ...)                                                                             \
  hipLaunchKernelGGL((crc32_stage_rs_kernel<M, F, W, ##__VA_ARGS__>), dim3((unsigned)grid), dim3(W * 64), 0, stream, \
                     bytes, off, n, per, img, out)
  // variants 300-303, 308, 309: both folds, 382- or 766-frame blocks
  // (10 waves per workgroup, variants 304-307, measured no faster in round 4
  // and no longer fit its registers once the whole line is read at once)
  if (fold >= 17 && fold <= 22) {  // timing-only diagnostics of the product form (wrong results)
    if (fold == 17) LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 4);
    else if (fold == 18) LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 5);
    else if (fold == 19) LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 6);
    else if (fold == 21) LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 8);
    else if (fold == 22) LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 9);
    else LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 7);
    return hipGetLastError();
  }
  if (fold == 16) {  // the product form with 6 waves (1.5 per SIMD): how much the second wave per SIMD buys
    if (big_blocks) return hipErrorInvalidValue;
    if (verify) LNX_STAGE(StageMode::kVerify, 8, 6, kStageBF, false, 1);
    else LNX_STAGE(StageMode::kCrc, 8, 6, kStageBF, false, 1);
    return hipGetLastError();
  }
  if (waves != 8) return hipErrorInvalidValue;
#define LNX_STAGE_W(M, F) LNX_STAGE(M, F, 8)
  if (fold == 15) {  // the product form with 510-frame blocks
    if (big_blocks) return hipErrorInvalidValue;
    if (verify) LNX_STAGE(StageMode::kVerify, 8, 8, kStageBF510, false, 1);
    else LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF510, false, 1);
  } else if (fold == 14) {  // the product form with the next block's offsets loaded ahead
    if (big_blocks) return hipErrorInvalidValue;
    if (verify) LNX_STAGE(StageMode::kVerify, 8, 8, kStageBF, false, 3);
    else LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 3);
  } else if (fold == 12 || fold == 13) {  // the product form (patched boundary word) with 190- / 254-frame blocks
    if (big_blocks) return hipErrorInvalidValue;
    if (fold == 12) {
      if (verify) LNX_STAGE(StageMode::kVerify, 8, 8, kStageBFSmall, false, 1);
      else LNX_STAGE(StageMode::kCrc, 8, 8, kStageBFSmall, false, 1);
    } else {
      if (verify) LNX_STAGE(StageMode::kVerify, 8, 8, kStageBFMid, false, 1);
      else LNX_STAGE(StageMode::kCrc, 8, 8, kStageBFMid, false, 1);
    }
  } else if (fold == 10 || fold == 11) {  // the slicing-by-8 fold with the boundary word patched once per half (11: two chains per half)
    if (big_blocks) return hipErrorInvalidValue;
    if (fold == 11) {
      if (verify) LNX_STAGE(StageMode::kVerify, 8, 8, kStageBF, false, 2);
      else LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 2);
    } else {
      if (verify) LNX_STAGE(StageMode::kVerify, 8, 8, kStageBF, false, 1);
      else LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, false, 1);
    }
  } else if (fold == 9) {  // the slicing-by-8 fold with the deferred boundary correction
    if (big_blocks) return hipErrorInvalidValue;
    if (verify) LNX_STAGE(StageMode::kVerify, 8, 8, kStageBF, true); else LNX_STAGE(StageMode::kCrc, 8, 8, kStageBF, true);
  } else if (fold == 8) {
    if (big_blocks) return hipErrorInvalidValue;
    if (verify) LNX_STAGE(StageMode::kVerify, 8, 8); else LNX_STAGE(StageMode::kCrc, 8, 8);
  } else if (big_blocks) {
    if (fold != 4 || waves != 8) return hipErrorInvalidValue;
    if (verify) LNX_STAGE(StageMode::kVerify, 4, 8, kStageBFBig); else LNX_STAGE(StageMode::kCrc, 4, 8, kStageBFBig);
  } else if (fold == 4) {
    if (verify) { LNX_STAGE_W(StageMode::kVerify, 4); } else { LNX_STAGE_W(StageMode::kCrc, 4); }
  } else {
    if (verify) { LNX_STAGE_W(StageMode::kVerify, 2); } else { LNX_STAGE_W(StageMode::kCrc, 2); }
  }
#undef LNX_STAGE_W
#undef LNX_STAGE
  return hipGetLastError();
}

}  // namespace rs
}  // namespace lnx
#endif  // LNX_RESEARCH
