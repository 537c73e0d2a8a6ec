// search_kernel.hip — batched ethernet.CRC32Search, gfx950.
//
// Reference: ethernet.CRC32Search(data, minOffCRC) (lneto ethernet/crc.go:28-47)
// returns the first off in [max(minOff, 0), len-4] with
//     CRC32(data[:off]) == LE32(data[off:off+4])
// or -1 (also when len < minOff + 4).  The Go code extends the CRC one byte at a
// time; here every prefix state of a capture is computed at once.  The test is
// the residue form of the same equality: CRC32(M || LE32(CRC32(M))) is the
// constant 0x2144DF1C for every M, and the 4-byte step is a bijection of the
// register, so the equality holds exactly when the register after data[:off+4]
// is ~0x2144DF1C = 0xDEBB20E3.
//
// One wave per capture, 256 bytes per block: lane j takes word j of the block;
// the carried register (0xFFFFFFFF at the start: the CRC init) is XOR-ed into
// word 0 for the scan (exact after whole words; the byte states inside word 0
// start from the carry itself), so with init 0
//   a_j = Z_4(w_j)                       (register contribution of word j)
//   inclusive scan over j with (A, B) -> Z_{|B|}(A) ^ B, |B| = 4*2^k bytes
// gives the register after every word; four byte steps from the state before
// the word give the register after every byte.  Z_{4*2^k} (k = 0..5) are byte
// tables in LDS (shared; lookups here are rare next to the frame CRC path).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdlib>
#include "gf2.hpp"

namespace lnx {

[[maybe_unused]] constexpr int kSearchBlock = 256;
[[maybe_unused]] constexpr uint32_t kSearchTabBytes = 1024 + 6 * 4096;  // byte-step table + 6 x 4 byte tables
constexpr uint32_t kResidueRegister = 0xDEBB20E3u;     // ~0x2144DF1C

// Z_{4*2^k}(x) through the four byte tables of level k
__device__ __forceinline__ uint32_t zlevel(const uint32_t* lds, int k, uint32_t x) {
  const uint32_t* z = lds + 256 + k * 1024;
  return z[x & 0xFFu] ^ z[256 + ((x >> 8) & 0xFFu)] ^ z[512 + ((x >> 16) & 0xFFu)] ^ z[768 + (x >> 24)];
}


// ------------------------------------------------------------------ segment lanes (r1g)
// One wave per capture, blocks of 64 x SEG bytes: lane j owns the SEG bytes
// at block offset SEG*j and folds them twice with the byte-step table
// (lane-private bank column, conflict-free):
//   pass A, from 0, a word at a time (Z_4 tables): its local contribution
//          l_j (lane 0 also folds in Z_SEG of the register carried in);
//   scan:  P_j = XOR_{i<=j} Z_{SEG*(j-i)}(l_i) in six steps with the
//          Z_{SEG*2^k} byte tables, so P_{j-1} is the register entering j;
//   pass B, from P_{j-1}: the register after every byte, tested against the
//          residue register as above.
// About two table lookups per byte plus 28 per lane per block, against ten
// per byte for the word-lane kernel above; bytes come from aligned dword loads
// realigned with v_alignbyte (a dword holding a capture byte never crosses a
// page, so loads stop at the capture end).
constexpr uint32_t kSearchSeg = 24;  // 1536-byte blocks: a 1500-B capture keeps 63 of 64 lanes busy
constexpr uint32_t kSegTabOff = 256 + 6 * 1024;                  // after the word-lane kernel's tables
constexpr uint32_t kSegTabDwords = 8192 + 7 * 1024;              // replicated byte table + 6 levels + Z_4
constexpr int kSegBlock = 1024;  // 2 blocks per CU (57 KiB LDS each): 8 waves per SIMD

__device__ __forceinline__ uint32_t zseg(const uint32_t* z, uint32_t x) {  // four byte tables at z
  return z[x & 0xFFu] ^ z[256 + ((x >> 8) & 0xFFu)] ^ z[512 + ((x >> 16) & 0xFFu)] ^ z[768 + (x >> 24)];
}
// zseg(z, x) ^ y with the five-way XOR in two v_bitop3
__device__ __forceinline__ uint32_t zseg_xor(const uint32_t* z, uint32_t x, uint32_t y) {
  const uint32_t t = __builtin_amdgcn_bitop3_b32(z[x & 0xFFu], z[256 + ((x >> 8) & 0xFFu)], z[512 + ((x >> 16) & 0xFFu)], 0x96);
  return __builtin_amdgcn_bitop3_b32(t, z[768 + (x >> 24)], y, 0x96);
}

// kBallot: pass B tests each byte with one compare into a wave mask and keeps
// the first (lane, byte) hit in scalar registers (a residue hit is rare: the
// branch is taken about once per capture); otherwise a per-lane hit bitmask
// kZWords: pass A folds its first kZWords words through the shared Z_4 tables
// (fewer VALU, bank conflicts) and the rest byte by byte through the
// conflict-free byte column (more VALU, no conflicts); 2 of 6 balances the two
// (r1h: 0.798 ms against 0.834 for 6, 0.804 for 3, 0.811 for 1, 0.814 for 0)
[[maybe_unused]] constexpr int kSearchZWords = 2;

template <bool kBallot, int kZWords>
__global__ void __launch_bounds__(kSegBlock) __attribute__((amdgpu_waves_per_eu(8)))  // <= 64 VGPRs: 2 blocks per CU
crc32_search_seg_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                        const int64_t* __restrict__ min_off, uint64_t n, const uint32_t* __restrict__ tables,
                        int64_t* __restrict__ result) {
  constexpr uint32_t SEG = kSearchSeg, NW = SEG / 4;
  __shared__ uint32_t lds[kSegTabDwords];
  for (uint32_t i = threadIdx.x; i < kSegTabDwords; i += kSegBlock) lds[i] = tables[kSegTabOff + i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, col = lane & 31u;
  const uint32_t* bt = lds + col;       // byte table, this lane's column: entry e at bt[32 e]
  const uint32_t* zt = lds + 8192;      // level k at zt + 1024 k
  auto bstep = [&](uint32_t r, uint32_t b) -> uint32_t { return bt[((r ^ b) & 0xFFu) << 5] ^ (r >> 8); };
  const uint64_t nwaves = (uint64_t)gridDim.x * (kSegBlock / 64);
  for (uint64_t c = (uint64_t)blockIdx.x * (kSegBlock / 64) + (threadIdx.x >> 6); c < n; c += nwaves) {
    const uint64_t s = off[c], e = off[c + 1];
    const int64_t L = e > s ? (int64_t)(e - s) : 0;
    int64_t m = min_off ? min_off[c] : 0;
    if (m < 0) m = 0;
    int64_t found = -1;
    if (L >= m + 4) {
      const uint8_t* d = bytes + s;
      uint32_t carry = 0xFFFFFFFFu;  // register entering the block (CRC init)
      for (int64_t B = 0; B < L && found < 0; B += 64 * SEG) {
        const int64_t base = B + (int64_t)(SEG * lane);
        // the lane's SEG bytes: NW + 1 aligned dwords (only those holding a
        // capture byte), realigned; bytes past the capture end read as junk
        // and only feed states past it
        const uintptr_t a = reinterpret_cast<uintptr_t>(d + base);
        const uint32_t sh = (uint32_t)(a & 3u);
        const uint32_t* wp = reinterpret_cast<const uint32_t*>(a - sh);
        const int64_t lim = (int64_t)(reinterpret_cast<uintptr_t>(d) + (uint64_t)L);  // first byte past the capture
        // dwords of the lane window that hold a capture byte (a 32-bit count,
        // so each load's guard is one 32-bit compare)
        const int64_t nd64 = (lim - (int64_t)(a - sh) + 3) >> 2;
        const int32_t nd = nd64 < 0 ? 0 : (nd64 > (int64_t)(NW + 1) ? (int32_t)(NW + 1) : (int32_t)nd64);
        uint32_t v[NW + 1];
#pragma unroll
        for (uint32_t i = 0; i <= NW; ++i) v[i] = (int32_t)i < nd ? wp[i] : 0u;
        uint32_t u[NW];
#pragma unroll
        for (uint32_t i = 0; i < NW; ++i) u[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], sh);
        // pass A: only the segment's end state is needed, so whole words
        // (slicing-by-4: Z_4 of register ^ word, shared tables)
        uint32_t l = 0;
#pragma unroll
        for (uint32_t i = 0; i < NW; ++i) {
          if ((int)i < kZWords) {
            l = zseg(zt + 6 * 1024, l ^ u[i]);
          } else {  // the same map through the conflict-free byte column
#pragma unroll
            for (uint32_t q = 0; q < 4; ++q) l = bstep(l, u[i] >> (8 * q));
          }
        }
        if (lane == 0) l ^= zseg(zt, carry);
        // scan: P holds lanes (lane - 2^k, lane] after step k
        uint32_t P = l;
#pragma unroll
        for (int k = 0; k < 6; ++k) {
          const uint32_t dd = 1u << k;
          const uint32_t prev = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - dd) * 4u), (int)P);
          P ^= lane >= dd ? zseg(zt + 1024 * k, prev) : 0u;
        }
        uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - 1u) * 4u), (int)P);
        r = lane == 0 ? carry : r;
        // pass B: the register after every byte. The state after byte i is the
        // CRC32Search candidate off = base + i + 1 - 4, valid for
        // base + i + 1 in [m + 4, L]
        if (kBallot) {
          uint32_t best_lane = 64, best_i = 0;  // wave-uniform
#pragma unroll
          for (uint32_t i = 0; i < SEG; ++i) {
            r = bstep(r, u[i >> 2] >> (8 * (i & 3)));
            if (__builtin_amdgcn_ballot_w64(r == kResidueRegister)) {
              const int64_t k = base + (int64_t)i + 1;
              const uint64_t ok = __builtin_amdgcn_ballot_w64(r == kResidueRegister && k >= m + 4 && k <= L);
              if (ok) {
                const uint32_t ln = (uint32_t)__builtin_ctzll(ok);
                if (ln < best_lane) best_lane = ln, best_i = i;
              }
            }
          }
          if (best_lane < 64) found = B + (int64_t)(SEG * best_lane + best_i) + 1 - 4;
        } else {
          // bit i of hm marks a residue after byte i, then the first bit whose
          // offset is in range
          uint32_t hm = 0;
#pragma unroll
          for (uint32_t i = 0; i < SEG; ++i) {
            r = bstep(r, u[i >> 2] >> (8 * (i & 3)));
            hm |= r == kResidueRegister ? (1u << i) : 0u;
          }
          const int64_t ilo = m + 3 - base, ihi = L - 1 - base;  // valid i range (inclusive)
          if (ilo > 0) hm = ilo >= 32 ? 0u : hm & (0xFFFFFFFFu << ilo);
          if (ihi < 31) hm = ihi < 0 ? 0u : hm & (0xFFFFFFFFu >> (31 - ihi));
          const int64_t best = hm ? base + (int64_t)__builtin_ctz(hm) + 1 - 4 : -1;
          const uint64_t hits = __builtin_amdgcn_ballot_w64(best >= 0);
          if (hits) {
            const uint32_t first = (uint32_t)__builtin_ctzll(hits);
            found = (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)best, first)) |
                              ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)((uint64_t)best >> 32), first) << 32));
          }
        }
        carry = (uint32_t)__builtin_amdgcn_readlane((int)P, 63);
      }
    }
    if (lane == 0) result[c] = found;
  }
}


// Two captures per wave (r2 product): each 32-lane half folds its own capture
// in blocks of 32 x 48 bytes (1536 bytes: a 1500-B capture is still one block)
// with the same three phases; the scan spans the half's 32 lanes in five
// levels of Z_{48*2^k}.  Per byte that is 0.42 scan lookups (shared tables,
// bank-conflicting) against 1.0 with 24-byte segments over 64 lanes.
constexpr uint32_t kHalfSeg = 48;
constexpr uint32_t kHalfTabOff = kSegTabOff + kSegTabDwords;  // Z_{48*2^k}, k = 0..4, in the host tables
constexpr uint32_t kHalfLdsDwords = 8192 + 5 * 1024 + 1024;    // byte table (32 columns), 5 levels, Z_4
constexpr uint32_t kHalfNibOff = kHalfTabOff + 5 * 1024;         // Z_4 nibble tables in 32 columns (4096 dwords)
//
// Pass B by word checks (WB, the r2 product): the register after k = 1..4
// bytes of a word entered with register r is Z_k(r ^ (w & lo_k)), lo_k the
// low k bytes, and Z_k is a bijection of the register, so it equals the
// residue register exactly when r ^ (w & lo_k) == Z_{-k}(0xDEBB20E3).  A word
// then costs four compares against constants and one Z_4 step to the next word
// (kBZ words through the shared Z_4 tables, the rest as four byte steps through
// the lane's conflict-free column) instead of four dependent byte steps each
// followed by a compare (tests/test_search_algebra.py restates both).
constexpr uint32_t kResBack1 = zshift_bytes(kResidueRegister, -1);
constexpr uint32_t kResBack2 = zshift_bytes(kResidueRegister, -2);
constexpr uint32_t kResBack3 = zshift_bytes(kResidueRegister, -3);
constexpr uint32_t kResBack4 = zshift_bytes(kResidueRegister, -4);
static_assert(kResBack4 == 0xFFFFFFFFu && kResBack1 == 0x00BE26EDu, "residue back-shifts");
// UL (crc32_search_u_kernel, r2 product): the four Z_4 byte tables in 32
// lane-private bank columns (the CRC kernel's U layout, 128 KiB), so every Z_4
// step of pass A and pass B is four conflict-free lookups addressed by v_perm;
// one 16-wave workgroup per CU.  With pass B by word checks the dependent chain
// is one Z_4 step per word (four independent lookups), not four byte steps, so
// four waves per SIMD are enough (r2y: the byte-chain pass B was latency-bound
// in this layout).
constexpr uint32_t kULdsDwords = 32768 + 6 * 1024;  // U (Z_4, 32 columns), Z_{48*2^k} for k = 0..4, Z_24
constexpr uint32_t kZ24Off = kHalfNibOff + 4096;     // Z_24 byte tables in the host tables
__device__ __forceinline__ uint32_t ulds(const uint32_t* lds, uint32_t byte_addr) {
  return *reinterpret_cast<const uint32_t*>(reinterpret_cast<const char*>(lds) + byte_addr);
}
// Z_4(x) ^ y through the U layout: byte k of x is byte 1 of the address (v_perm
// with the lane's column base), tables m = 1, 3 ride in the +128 immediate
__device__ __forceinline__ uint32_t ustep_xor(const uint32_t* lds, uint32_t x, uint32_t y, uint32_t b0, uint32_t b1) {
  const uint32_t a0 = __builtin_amdgcn_perm(x, b0, 0x0c020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(x, b0, 0x0c020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(x, b1, 0x0c020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(x, b1, 0x0c020700u);
  const uint32_t t = __builtin_amdgcn_bitop3_b32(ulds(lds, a0), ulds(lds, a1 + 128), ulds(lds, a2), 0x96);
  return __builtin_amdgcn_bitop3_b32(t, ulds(lds, a3 + 128), y, 0x96);
}

template <int kZWords, bool WB, int kBZ, bool UL>
__device__ __forceinline__ void search_half_body(uint32_t* lds, const uint8_t* __restrict__ bytes,
                                                 const uint64_t* __restrict__ off, const int64_t* __restrict__ min_off,
                                                 uint64_t n, const uint32_t* __restrict__ tables,
                                                 int64_t* __restrict__ result) {
  constexpr uint32_t SEG = kHalfSeg, NW = SEG / 4;
  constexpr uint32_t kNib = kBZ < 0 ? 4096u : 0u;  // pass B's Z_4 by lane-private nibble tables
  constexpr uint32_t kZt = UL ? 32768u : 8192u;     // the scan tables
  if constexpr (UL) {
    // thread t expands Z_4 value t (table t >> 8, entry t & 255) into its 32 bank replicas
    static_assert(kSegBlock == 1024, "one U value per thread");
    const uint32_t t = threadIdx.x, v = tables[kSegTabOff + 8192 + 6 * 1024 + t];
    const uint32_t ua = ((t >> 9) << 16) | ((t & 255u) << 8) | (((t >> 8) & 1u) << 7);
    uint4* row = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + ua);
    const uint4 v4 = {v, v, v, v};
#pragma unroll
    for (int i = 0; i < 8; ++i) row[(i + t) & 7u] = v4;
  } else {
    for (uint32_t i = threadIdx.x; i < kNib; i += kSegBlock) lds[kHalfLdsDwords + i] = tables[kHalfNibOff + i];
    for (uint32_t i = threadIdx.x; i < 8192; i += kSegBlock) lds[i] = tables[kSegTabOff + i];
    for (uint32_t i = threadIdx.x; i < 1024; i += kSegBlock) lds[8192 + 5 * 1024 + i] = tables[kSegTabOff + 8192 + 6 * 1024 + i];
  }
  for (uint32_t i = threadIdx.x; i < 5 * 1024; i += kSegBlock) lds[kZt + i] = tables[kHalfTabOff + i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, col = lane & 31u, hl = lane & 31u, half = lane >> 5;
  const uint32_t* bt = lds + col;               // byte table, this lane's column: entry e at bt[32 e]
  const uint32_t* zt = lds + kZt;               // level k at zt + 1024 k
  const uint32_t* z4 = lds + 8192 + 5 * 1024;   // Z_4 (shared tables; not in the UL layout)
  const uint32_t ub0 = col << 2, ub1 = ub0 | 65536u;  // UL: the lane's U column bases
  auto bstep = [&](uint32_t r, uint32_t b) -> uint32_t { return bt[((r ^ b) & 0xFFu) << 5] ^ (r >> 8); };
  const uint64_t nwaves = (uint64_t)gridDim.x * (kSegBlock / 64);
  for (uint64_t q = (uint64_t)blockIdx.x * (kSegBlock / 64) + (threadIdx.x >> 6); q * 2 < n; q += nwaves) {
    const uint64_t c = q * 2 + half;
    const bool live = c < n;
    const uint64_t s = live ? off[c] : 0, e = live ? off[c + 1] : 0;
    const int64_t L = e > s ? (int64_t)(e - s) : 0;
    int64_t m = live && min_off ? min_off[c] : 0;
    if (m < 0) m = 0;
    int64_t found = -1;
    bool act = live && L >= m + 4;  // this half still searching
    const uint8_t* d = bytes + s;
    uint32_t carry = 0xFFFFFFFFu;  // register entering the block (CRC init)
    for (int64_t B = 0; __builtin_amdgcn_ballot_w64(act) != 0; B += 32 * SEG) {
      const int64_t base = B + (int64_t)(SEG * hl);
      const uintptr_t a = reinterpret_cast<uintptr_t>(d + base);
      const uint32_t sh = (uint32_t)(a & 3u);
      const uint32_t* wp = reinterpret_cast<const uint32_t*>(d + base - sh);  // global, not flat (see search_u_body)
      const int64_t lim = (int64_t)(reinterpret_cast<uintptr_t>(d) + (uint64_t)L);  // first byte past the capture
      const int64_t nd64 = act ? (lim - (int64_t)(a - sh) + 3) >> 2 : 0;
      const int32_t nd = nd64 < 0 ? 0 : (nd64 > (int64_t)(NW + 1) ? (int32_t)(NW + 1) : (int32_t)nd64);
      uint32_t v[NW + 1];
#pragma unroll
      for (uint32_t i = 0; i <= NW; ++i) v[i] = (int32_t)i < nd ? wp[i] : 0u;
      uint32_t u[NW];
#pragma unroll
      for (uint32_t i = 0; i < NW; ++i) u[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], sh);
      // pass A: the segment's end state from 0 (kZWords words by Z_4, the rest byte by byte)
      uint32_t l = 0;
      if constexpr (UL) {
        uint32_t x = u[0];
#pragma unroll
        for (uint32_t i = 0; i + 1 < NW; ++i) x = ustep_xor(lds, x, u[i + 1], ub0, ub1);
        l = ustep_xor(lds, x, 0u, ub0, ub1);
      } else if constexpr (kZWords == (int)NW && WB) {  // every word by Z_4: the next word rides in the second v_bitop3
        uint32_t x = u[0];
#pragma unroll
        for (uint32_t i = 0; i + 1 < NW; ++i) x = zseg_xor(z4, x, u[i + 1]);
        l = zseg_xor(z4, x, 0u);
      }
#pragma unroll
      for (uint32_t i = 0; i < ((kZWords == (int)NW && WB) || UL ? 0u : NW); ++i) {
        if ((int)i < kZWords) {
          l = zseg(z4, l ^ u[i]);
        } else {
#pragma unroll
          for (uint32_t qq = 0; qq < 4; ++qq) l = bstep(l, u[i] >> (8 * qq));
        }
      }
      if (hl == 0) l ^= zseg(zt, carry);
      // scan within the half: P holds lanes (hl - 2^k, hl] after step k
      uint32_t P = l;
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const uint32_t dd = 1u << k;
        const uint32_t prev = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - dd) * 4u), (int)P);
        if constexpr (WB) {
          if (hl >= dd) P = zseg_xor(zt + 1024 * k, prev, P);
        } else {
          P ^= hl >= dd ? zseg(zt + 1024 * k, prev) : 0u;
        }
      }
      uint32_t r = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - 1u) * 4u), (int)P);
      r = hl == 0 ? carry : r;
      // pass B: the register after every byte; the first valid residue per half
      uint32_t bl0 = 32, bi0 = 0, bl1 = 32, bi1 = 0;  // wave-uniform
      if constexpr (WB) {
        // byte index bi of the segment is a valid candidate when base + bi + 1 is in [m + 4, L]
        const int64_t lo64 = m + 3 - base, hi64 = L - 1 - base;
        const int32_t vlo = lo64 < 0 ? 0 : (lo64 > 64 ? 64 : (int32_t)lo64);
        const int32_t vhi = hi64 < 0 ? -1 : (hi64 > 64 ? 64 : (int32_t)hi64);
        const uint64_t actm = __builtin_amdgcn_ballot_w64(act);
#pragma unroll
        for (uint32_t i = 0; i < NW; ++i) {
          const uint32_t w = u[i];
          const bool h1 = (r ^ (w & 0xFFu)) == kResBack1, h2 = (r ^ (w & 0xFFFFu)) == kResBack2;
          const bool h3 = (r ^ (w & 0xFFFFFFu)) == kResBack3;
          uint32_t x = r ^ w;
          const bool h4 = x == kResBack4;
          const uint64_t any = (__builtin_amdgcn_ballot_w64(h1) | __builtin_amdgcn_ballot_w64(h2) |
                                __builtin_amdgcn_ballot_w64(h3) | __builtin_amdgcn_ballot_w64(h4)) & actm;
          if (any) {
            const bool hk[4] = {h1, h2, h3, h4};
#pragma unroll
            for (uint32_t kk = 0; kk < 4; ++kk) {
              const int32_t bi = (int32_t)(4 * i + kk);
              const uint64_t ok = __builtin_amdgcn_ballot_w64(hk[kk] && bi >= vlo && bi <= vhi) & actm;
              const uint32_t o0 = (uint32_t)ok, o1 = (uint32_t)(ok >> 32);
              if (o0) {
                const uint32_t ln = (uint32_t)__builtin_ctz(o0);
                if (ln < bl0) bl0 = ln, bi0 = 4 * i + kk;
              }
              if (o1) {
                const uint32_t ln = (uint32_t)__builtin_ctz(o1);
                if (ln < bl1) bl1 = ln, bi1 = 4 * i + kk;
              }
            }
          }
          if (i + 1 < NW) {
            if constexpr (UL) {
              r = ustep_xor(lds, x, 0u, ub0, ub1);
            } else if constexpr (kBZ < 0) {
              const uint32_t* nb = lds + kHalfLdsDwords + col;  // (i, v) at nb[32 (16 i + v)]
              uint32_t y[8];
#pragma unroll
              for (uint32_t q = 0; q < 8; ++q) y[q] = nb[(16u * q + ((x >> (4 * q)) & 15u)) << 5];
              r = (y[0] ^ y[1] ^ y[2]) ^ (y[3] ^ y[4] ^ y[5]) ^ (y[6] ^ y[7]);
            } else if ((int)i < kBZ) {
              r = zseg(z4, x);
            } else {
              // Z_4(x) as four byte steps on the pre-XOR-ed word (conflict-free column)
#pragma unroll
              for (uint32_t qq = 0; qq < 4; ++qq) x = bt[(x & 0xFFu) << 5] ^ (x >> 8);
              r = x;
            }
          }
        }
      }
#pragma unroll
      for (uint32_t i = 0; i < (WB ? 0u : SEG); ++i) {
        r = bstep(r, u[i >> 2] >> (8 * (i & 3)));
        if (__builtin_amdgcn_ballot_w64(act && r == kResidueRegister)) {
          const int64_t k = base + (int64_t)i + 1;
          const uint64_t ok = __builtin_amdgcn_ballot_w64(act && r == kResidueRegister && k >= m + 4 && k <= L);
          const uint32_t o0 = (uint32_t)ok, o1 = (uint32_t)(ok >> 32);
          if (o0) {
            const uint32_t ln = (uint32_t)__builtin_ctz(o0);
            if (ln < bl0) bl0 = ln, bi0 = i;
          }
          if (o1) {
            const uint32_t ln = (uint32_t)__builtin_ctz(o1);
            if (ln < bl1) bl1 = ln, bi1 = i;
          }
        }
      }
      const uint32_t bl = half ? bl1 : bl0, bi = half ? bi1 : bi0;
      if (act && bl < 32) found = B + (int64_t)(SEG * bl + bi) + 1 - 4;
      const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)P, 31);
      const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)P, 63);
      carry = half ? c1 : c0;
      act = act && found < 0 && B + (int64_t)(32 * SEG) < L;
    }
    if (live && hl == 0) result[c] = found;
  }
}

template <int kZWords, bool WB = false, int kBZ = 12>
__global__ void __launch_bounds__(kSegBlock) __attribute__((amdgpu_waves_per_eu(8)))  // <= 64 VGPRs: 2 blocks per CU
crc32_search_half_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                         const int64_t* __restrict__ min_off, uint64_t n, const uint32_t* __restrict__ tables,
                         int64_t* __restrict__ result) {
  __shared__ uint32_t lds[kHalfLdsDwords + (kBZ < 0 ? 4096u : 0u)];
  search_half_body<kZWords, WB, kBZ, false>(lds, bytes, off, min_off, n, tables, result);
}

// The UL product body: NC captures per half-wave folded side by side, so each
// lane carries NC independent Z_4 chains through pass A and pass B (one 16-wave
// block per CU leaves four waves per SIMD to hide the LDS latency; r2s2e: one
// capture per half ran 0.666 ms against 0.624 for the two-block form).
template <int NC, bool SPLIT = false, int GLD = 1>
__device__ __forceinline__ void search_u_body(uint32_t* lds, const uint8_t* __restrict__ bytes,
                                              const uint64_t* __restrict__ off, const int64_t* __restrict__ min_off,
                                              uint64_t n, const uint32_t* __restrict__ tables,
                                              int64_t* __restrict__ result) {
  constexpr uint32_t SEG = kHalfSeg, NW = SEG / 4;
  {
    static_assert(kSegBlock == 1024, "one U value per thread");
    const uint32_t t = threadIdx.x, v = tables[kSegTabOff + 8192 + 6 * 1024 + t];
    const uint32_t ua = ((t >> 9) << 16) | ((t & 255u) << 8) | (((t >> 8) & 1u) << 7);
    uint4* row = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + ua);
    const uint4 v4 = {v, v, v, v};
#pragma unroll
    for (int i = 0; i < 8; ++i) row[(i + t) & 7u] = v4;
  }
  for (uint32_t i = threadIdx.x; i < 5 * 1024; i += kSegBlock) lds[32768 + i] = tables[kHalfTabOff + i];
  if constexpr (SPLIT) lds[32768 + 5 * 1024 + threadIdx.x] = tables[kZ24Off + threadIdx.x];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, col = lane & 31u, hl = lane & 31u, half = lane >> 5;
  const uint32_t* zt = lds + 32768;  // Z_{48*2^k} at zt + 1024 k (shared)
  const uint32_t* z24 = lds + 32768 + 5 * 1024;  // SPLIT: Z_24 (shared)
  const uint32_t ub0 = col << 2, ub1 = ub0 | 65536u;
  const uint64_t nwaves = (uint64_t)gridDim.x * (kSegBlock / 64);
  constexpr uint64_t CPW = 2 * NC;  // captures per wave: capture 2j + half of the group in half `half`
  struct Grp {
    uint64_t s[NC], e[NC];
    int64_t m[NC];
  };
  auto load_grp = [&](uint64_t qq, Grp& g) {
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const uint64_t cc = qq * CPW + 2 * j + half;
      const bool lv = cc < n;
      g.s[j] = lv ? off[cc] : 0;
      g.e[j] = lv ? off[cc + 1] : 0;
      g.m[j] = lv && min_off ? min_off[cc] : 0;
    }
  };
  // the words of block B of each capture of a group (only dwords holding a capture byte).
  // Packed groups (every capture of the group inside [off[first], off[last + 1]),
  // under 2 GiB) load through one buffer descriptor over the group's bytes
  // instead: one per-lane offset, the word index in the immediate, no guard
  // (words past a capture's end are the next capture's bytes and only feed
  // states past its end; past the group the range check returns 0).
  __amdgpu_buffer_rsrc_t grsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(bytes), (short)0, 0, 0x00020000);
  uint64_t gbase = 0;
  bool gfast = false;
  auto load_words = [&](const Grp& g, int64_t B, const bool (&ac)[NC], uint32_t (&v)[NC][NW + 1]) {
    const int64_t base = B + (int64_t)(SEG * hl);
    if (gfast) {
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const uint64_t a = g.s[j] + (uint64_t)base;  // byte offset of the lane's segment in `bytes`
        const uint32_t vo = ac[j] ? (uint32_t)((a & ~3ull) - gbase) : 0x80000000u;
        // GLD 2: alternate the nt bit so hipcc cannot merge neighbours into
        // 16-byte loads (GLD 1 lets it)
#pragma unroll
        for (uint32_t i = 0; i <= NW; ++i)
          v[j][i] = GLD == 2 && (i & 1) ? __builtin_amdgcn_raw_buffer_load_b32(grsrc, vo + 4 * i, 0, 2)
                                        : __builtin_amdgcn_raw_buffer_load_b32(grsrc, vo + 4 * i, 0, 0);
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const uint8_t* dj = bytes + g.s[j];
      const int64_t Lj = g.e[j] > g.s[j] ? (int64_t)(g.e[j] - g.s[j]) : 0;
      const uintptr_t a = reinterpret_cast<uintptr_t>(dj + base);
      const uint32_t sh = (uint32_t)(a & 3u);
      // pointer arithmetic on the kernel argument (not an integer cast), so the
      // loads are global_load (vmcnt only): flat loads also count in lgkmcnt,
      // and every wait for an LDS lookup would then wait for them too
      const uint32_t* wp = reinterpret_cast<const uint32_t*>(dj + base - sh);
      const int64_t lim = (int64_t)(reinterpret_cast<uintptr_t>(dj) + (uint64_t)Lj);
      const int64_t nd64 = ac[j] ? (lim - (int64_t)(a - sh) + 3) >> 2 : 0;
      const int32_t nd = nd64 < 0 ? 0 : (nd64 > (int64_t)(NW + 1) ? (int32_t)(NW + 1) : (int32_t)nd64);
      // one dword per lane per load (16-byte loads measured slower, r2s2i)
#pragma unroll
      for (uint32_t i = 0; i <= NW; ++i) v[j][i] = (int32_t)i < nd ? wp[i] : 0u;
    }
  };
  const uint64_t q0 = (uint64_t)blockIdx.x * (kSegBlock / 64) + (threadIdx.x >> 6);
  for (uint64_t q = q0; q * CPW < n; q += nwaves) {
    uint64_t c[NC];
    bool live[NC], act[NC];
    int64_t L[NC], m[NC], found[NC];
    const uint8_t* d[NC];
    uint32_t carry[NC];
    Grp gc;
    load_grp(q, gc);
    {
      // the group's byte range (wave-uniform: off[] of the group's first and one-past-last capture)
      const uint64_t ga = q * CPW, gb = ga + CPW < n ? ga + CPW : n;
      const uint64_t gs = off[ga], ge = off[gb];
      bool inside = ge >= gs && ge - (gs & ~3ull) + 3 < (1ull << 31);
#pragma unroll
      for (int j = 0; j < NC; ++j)
        inside = inside && (gc.e[j] <= gc.s[j] || (gc.s[j] >= gs && gc.e[j] <= ge));
      gfast = GLD != 0 && __builtin_amdgcn_ballot_w64(!inside) == 0;
      // gs / ge are wave-uniform (one group per wave): move them to SGPRs, or
      // hipcc wraps every buffer load in a waterfall loop over the descriptor
      auto uni64 = [](uint64_t x) -> uint64_t {
        return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x) |
               ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32);
      };
      gbase = uni64(gs) & ~3ull;
      const uint64_t geu = uni64(ge);
      grsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(bytes + gbase), (short)0,
                                                // rounded up to whole dwords: the range check drops a dword
                                                // that straddles the end, and the one holding the group's
                                                // last byte never crosses a page
                                                gfast ? (int)((geu - gbase + 3) & ~3ull) : 0, 0x00020000);
    }
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      c[j] = q * CPW + 2 * j + half;
      live[j] = c[j] < n;
      const uint64_t s_ = gc.s[j], e_ = gc.e[j];
      L[j] = e_ > s_ ? (int64_t)(e_ - s_) : 0;
      m[j] = gc.m[j];
      if (m[j] < 0) m[j] = 0;
      found[j] = -1;
      act[j] = live[j] && L[j] >= m[j] + 4;
      d[j] = bytes + s_;
      carry[j] = 0xFFFFFFFFu;
    }
    auto any_act = [&]() {
      bool a = false;
#pragma unroll
      for (int j = 0; j < NC; ++j) a = a || act[j];
      return __builtin_amdgcn_ballot_w64(a) != 0;
    };
    for (int64_t B = 0; any_act(); B += 32 * SEG) {
      const int64_t base = B + (int64_t)(SEG * hl);
      uint32_t u[NC][NW];
      {
        uint32_t v[NC][NW + 1];
        load_words(gc, B, act, v);
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const uint32_t sh = (uint32_t)((reinterpret_cast<uintptr_t>(d[j]) + (uint64_t)base) & 3u);
#pragma unroll
          for (uint32_t i = 0; i < NW; ++i) u[j][i] = __builtin_amdgcn_alignbyte(v[j][i + 1], v[j][i], sh);
        }
      }
      // pass A: each segment's end state from 0, the NC chains side by side.
      // SPLIT: each segment as two independent 24-byte chains, joined by Z_24
      // (la: words 0..5, kept for pass B's second chain)
      constexpr uint32_t NH = SPLIT ? NW / 2 : NW;
      uint32_t x[NC], xb[NC], la[NC];
#pragma unroll
      for (int j = 0; j < NC; ++j) x[j] = u[j][0], xb[j] = u[j][NH % NW];
#pragma unroll
      for (uint32_t i = 0; i + 1 < NH; ++i)
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          x[j] = ustep_xor(lds, x[j], u[j][i + 1], ub0, ub1);
          if constexpr (SPLIT) xb[j] = ustep_xor(lds, xb[j], u[j][NH + i + 1], ub0, ub1);
        }
      uint32_t P[NC];
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        if constexpr (SPLIT) {
          la[j] = ustep_xor(lds, x[j], 0u, ub0, ub1);
          P[j] = zseg_xor(z24, la[j], ustep_xor(lds, xb[j], 0u, ub0, ub1));
        } else {
          P[j] = ustep_xor(lds, x[j], 0u, ub0, ub1);
        }
        if (hl == 0) P[j] ^= zseg(zt, carry[j]);
      }
      // scan within the half
#pragma unroll
      for (int k = 0; k < 5; ++k) {
        const uint32_t dd = 1u << k;
#pragma unroll
        for (int j = 0; j < NC; ++j) {
          const uint32_t prev = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - dd) * 4u), (int)P[j]);
          if (hl >= dd) P[j] = zseg_xor(zt + 1024 * k, prev, P[j]);
        }
      }
      uint32_t r[NC], rb[NC];
      int32_t vlo[NC], vhi[NC];
      uint64_t actm[NC];
      uint32_t bl0[NC], bi0[NC], bl1[NC], bi1[NC];  // wave-uniform
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const uint32_t pr = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - 1u) * 4u), (int)P[j]);
        r[j] = hl == 0 ? carry[j] : pr;
        if constexpr (SPLIT) rb[j] = zseg_xor(z24, r[j], la[j]);  // the register entering word NH
        const int64_t lo64 = m[j] + 3 - base, hi64 = L[j] - 1 - base;
        vlo[j] = lo64 < 0 ? 0 : (lo64 > 64 ? 64 : (int32_t)lo64);
        vhi[j] = hi64 < 0 ? -1 : (hi64 > 64 ? 64 : (int32_t)hi64);
        actm[j] = __builtin_amdgcn_ballot_w64(act[j]);
        bl0[j] = 32, bi0[j] = 0, bl1[j] = 32, bi1[j] = 0;
      }
      // pass B by word checks (see crc32_search_half_kernel), the chains side by side
      // (SPLIT: word i of the first half and word NH + i of the second together)
      constexpr int NCH = SPLIT ? 2 : 1;
#pragma unroll
      for (uint32_t ii = 0; ii < NH; ++ii) {
#pragma unroll
        for (int jh = 0; jh < NC * NCH; ++jh) {
          const int j = jh % NC, h = jh / NC;
          const uint32_t i = ii + (uint32_t)h * NH;
          const uint32_t w = u[j][i], rr = h ? rb[j] : r[j];
          const bool h1 = (rr ^ (w & 0xFFu)) == kResBack1, h2 = (rr ^ (w & 0xFFFFu)) == kResBack2;
          const bool h3 = (rr ^ (w & 0xFFFFFFu)) == kResBack3;
          const uint32_t xx = rr ^ w;
          const bool h4 = xx == kResBack4;
          const uint64_t any = (__builtin_amdgcn_ballot_w64(h1) | __builtin_amdgcn_ballot_w64(h2) |
                                __builtin_amdgcn_ballot_w64(h3) | __builtin_amdgcn_ballot_w64(h4)) & actm[j];
          if (any) {
            const bool hk[4] = {h1, h2, h3, h4};
#pragma unroll
            for (uint32_t kk = 0; kk < 4; ++kk) {
              const int32_t bi = (int32_t)(4 * i + kk);
              const uint64_t ok = __builtin_amdgcn_ballot_w64(hk[kk] && bi >= vlo[j] && bi <= vhi[j]) & actm[j];
              const uint32_t o0 = (uint32_t)ok, o1 = (uint32_t)(ok >> 32);
              // hits arrive in byte order within a chain; with two chains a lane's
              // later-half hit can come first, so ties keep the smaller byte
              if (o0) {
                const uint32_t ln = (uint32_t)__builtin_ctz(o0);
                if (ln < bl0[j] || (SPLIT && ln == bl0[j] && 4 * i + kk < bi0[j])) bl0[j] = ln, bi0[j] = 4 * i + kk;
              }
              if (o1) {
                const uint32_t ln = (uint32_t)__builtin_ctz(o1);
                if (ln < bl1[j] || (SPLIT && ln == bl1[j] && 4 * i + kk < bi1[j])) bl1[j] = ln, bi1[j] = 4 * i + kk;
              }
            }
          }
          if (ii + 1 < NH) {
            if (h)
              rb[j] = ustep_xor(lds, xx, 0u, ub0, ub1);
            else
              r[j] = ustep_xor(lds, xx, 0u, ub0, ub1);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NC; ++j) {
        const uint32_t bl = half ? bl1[j] : bl0[j], bi = half ? bi1[j] : bi0[j];
        if (act[j] && bl < 32) found[j] = B + (int64_t)(SEG * bl + bi) + 1 - 4;
        const uint32_t c0 = (uint32_t)__builtin_amdgcn_readlane((int)P[j], 31);
        const uint32_t c1 = (uint32_t)__builtin_amdgcn_readlane((int)P[j], 63);
        carry[j] = half ? c1 : c0;
        act[j] = act[j] && found[j] < 0 && B + (int64_t)(32 * SEG) < L[j];
      }
    }
#pragma unroll
    for (int j = 0; j < NC; ++j)
      if (live[j] && hl == 0) result[c[j]] = found[j];
  }
}

template <int NC, bool SPLIT = false, int GLD = 1>
__global__ void __launch_bounds__(kSegBlock, 1)
crc32_search_u_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                      const int64_t* __restrict__ min_off, uint64_t n, const uint32_t* __restrict__ tables,
                      int64_t* __restrict__ result) {
  __shared__ __attribute__((aligned(16))) uint32_t lds[kULdsDwords];
  if constexpr (NC == 0)
    search_half_body<12, true, 0, true>(lds, bytes, off, min_off, n, tables, result);
  else
    search_u_body<NC, SPLIT, GLD>(lds, bytes, off, min_off, n, tables, result);
}

// Octet segments (round 4; LNX_PROF_SEARCH=o in the research library).  The
// shared-table lookups (the scan, 5 levels over 32 lanes, 0.5 lookups per byte
// with about 2.6x bank conflicts) were 22 % of the product's LDS cycles.  Here
// 8 lanes take a capture's 1536-byte block, 192 bytes each, so a wave folds 8
// captures and the scan has 3 levels over 8 lanes (0.06 shared lookups per
// byte).  Each lane's 192 bytes are four 48-byte chains folded side by side
// (the same dependent-chain length as the product's 12 words):
//   pass A   la_c = chain c folded from 0 (U layout, conflict-free)
//            l = Z48(Z48(Z48(la_0) ^ la_1) ^ la_2) ^ la_3   (Horner)
//   scan     Z_{192*2^k}, k = 0..2, shared byte tables (lane 0 folds Z_192(carry))
//   entries  r_0 = register entering the segment, r_{c+1} = Z48(r_c) ^ la_c
//   pass B   word checks on the four chains side by side
// Z48 goes through lane-private nibble tables (8 conflict-free lookups, 16 KiB
// in 32 bank columns).  A lane keeps its smallest valid hit byte; the first
// lane of its octet with a hit gives the capture's answer (lanes are in byte
// order).  tests/test_search_algebra.py::oct_search restates the schedule.
constexpr uint32_t kOctNibOff = kZ24Off + 1024;          // host tables: Z_48 nibble tables, 32 columns
[[maybe_unused]] constexpr uint32_t kOctLevOff = kOctNibOff + 4096;  // host tables: Z_{192*2^k}, k = 0..2 (copied with the nibbles)
constexpr uint32_t kOctLdsDwords = 32768 + 4096 + 3 * 1024;
static_assert(kOctLdsDwords * 4 <= 163840, "octet LDS");

__global__ void __launch_bounds__(kSegBlock, 1)
crc32_search_o_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off,
                      const int64_t* __restrict__ min_off, uint64_t n, const uint32_t* __restrict__ tables,
                      int64_t* __restrict__ result) {
  constexpr uint32_t LPC = 8, SEG = 1536 / LPC, NW = SEG / 4, CW = 12, NCH = NW / CW;
  static_assert(NCH == 4, "four 48-byte chains");
  __shared__ __attribute__((aligned(16))) uint32_t lds[kOctLdsDwords];
  {
    static_assert(kSegBlock == 1024, "one U value per thread");
    const uint32_t t = threadIdx.x, v = tables[kSegTabOff + 8192 + 6 * 1024 + t];
    const uint32_t ua = ((t >> 9) << 16) | ((t & 255u) << 8) | (((t >> 8) & 1u) << 7);
    uint4* row = reinterpret_cast<uint4*>(reinterpret_cast<char*>(lds) + ua);
    const uint4 v4 = {v, v, v, v};
#pragma unroll
    for (int i = 0; i < 8; ++i) row[(i + t) & 7u] = v4;
  }
  for (uint32_t i = threadIdx.x; i < 4096u + 3u * 1024u; i += kSegBlock) lds[32768 + i] = tables[kOctNibOff + i];
  __syncthreads();
  const uint32_t lane = threadIdx.x & 63u, col = lane & 31u, hl = lane & (LPC - 1), oct = lane / LPC;
  const uint32_t* zt = lds + 32768 + 4096;  // Z_{192*2^k} at zt + 1024 k (shared)
  const uint32_t ub0 = col << 2, ub1 = ub0 | 65536u;
  // Z48 through the lane-private nibble tables: (i, v) at byte ((16 i + v) << 7) + 4 col
  const char* nib = reinterpret_cast<const char*>(lds + 32768) + ub0;
  auto z48 = [&](uint32_t x) -> uint32_t {
    uint32_t y[8];
#pragma unroll
    for (uint32_t i = 0; i < 8; ++i)
      y[i] = *reinterpret_cast<const uint32_t*>(nib + ((16u * i + __builtin_amdgcn_ubfe(x, 4 * i, 4)) << 7));
    return __builtin_amdgcn_bitop3_b32(__builtin_amdgcn_bitop3_b32(y[0], y[1], y[2], 0x96),
                                       __builtin_amdgcn_bitop3_b32(y[3], y[4], y[5], 0x96), y[6] ^ y[7], 0x96);
  };
  const uint64_t nwaves = (uint64_t)gridDim.x * (kSegBlock / 64);
  for (uint64_t q = (uint64_t)blockIdx.x * (kSegBlock / 64) + (threadIdx.x >> 6); q * (64 / LPC) < n; q += nwaves) {
    const uint64_t ga = q * (64 / LPC);
    const uint64_t c = ga + oct;
    const bool live = c < n;
    const uint64_t s = live ? off[c] : 0, e = live ? off[c + 1] : 0;
    const int64_t L = e > s ? (int64_t)(e - s) : 0;
    int64_t m = live && min_off ? min_off[c] : 0;
    if (m < 0) m = 0;
    int64_t found = -1;
    bool act = live && L >= m + 4;
    uint32_t carry = 0xFFFFFFFFu;
    // the group's bytes through one descriptor when every capture lies inside [off[ga], off[gb])
    const uint64_t gb = ga + 64 / LPC < n ? ga + 64 / LPC : n;
    auto uni64 = [](uint64_t x) -> uint64_t {
      return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)x) |
             ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(x >> 32)) << 32);
    };
    const uint64_t gs = uni64(off[ga]), ge = uni64(off[gb]);
    const bool inside = ge >= gs && ge - (gs & ~3ull) + 3 < (1ull << 31) && (e <= s || (s >= gs && e <= ge));
    const bool gfast = __builtin_amdgcn_ballot_w64(!inside) == 0;
    const uint64_t gbase = gs & ~3ull;
    const __amdgpu_buffer_rsrc_t grsrc = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<uint8_t*>(bytes + gbase), (short)0, gfast ? (int)((ge - gbase + 3) & ~3ull) : 0, 0x00020000);
    for (int64_t B = 0; __builtin_amdgcn_ballot_w64(act) != 0; B += LPC * SEG) {
      const int64_t base = B + (int64_t)(SEG * hl);
      const uint32_t sh = (uint32_t)((s + (uint64_t)base) & 3u);
      uint32_t u[NW];
      {
        uint32_t v[NW + 1];
        if (gfast) {
          const uint32_t vo = act ? (uint32_t)(((s + (uint64_t)base) & ~3ull) - gbase) : 0x80000000u;
#pragma unroll
          for (uint32_t i = 0; i <= NW; ++i) v[i] = __builtin_amdgcn_raw_buffer_load_b32(grsrc, vo + 4 * i, 0, 0);
        } else {
          const uint8_t* dj = bytes + s;
          const uint32_t* wp = reinterpret_cast<const uint32_t*>(dj + base - sh);
          const int64_t nd64 = act ? (L - base + (int64_t)sh + 3) >> 2 : 0;
          const int32_t nd = nd64 < 0 ? 0 : (nd64 > (int64_t)(NW + 1) ? (int32_t)(NW + 1) : (int32_t)nd64);
#pragma unroll
          for (uint32_t i = 0; i <= NW; ++i) v[i] = (int32_t)i < nd ? wp[i] : 0u;
        }
#pragma unroll
        for (uint32_t i = 0; i < NW; ++i) u[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], sh);
      }
      // pass A: the four chains side by side
      uint32_t x[NCH], la[NCH];
#pragma unroll
      for (uint32_t ch = 0; ch < NCH; ++ch) x[ch] = u[CW * ch];
#pragma unroll
      for (uint32_t i = 0; i + 1 < CW; ++i)
#pragma unroll
        for (uint32_t ch = 0; ch < NCH; ++ch) x[ch] = ustep_xor(lds, x[ch], u[CW * ch + i + 1], ub0, ub1);
#pragma unroll
      for (uint32_t ch = 0; ch < NCH; ++ch) la[ch] = ustep_xor(lds, x[ch], 0u, ub0, ub1);
      uint32_t P = la[0];
#pragma unroll
      for (uint32_t ch = 1; ch < NCH; ++ch) P = z48(P) ^ la[ch];
      if (hl == 0) P ^= zseg(zt, carry);
      // scan within the octet
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        const uint32_t dd = 1u << k;
        const uint32_t prev = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - dd) * 4u), (int)P);
        if (hl >= dd) P = zseg_xor(zt + 1024 * k, prev, P);
      }
      uint32_t r[NCH];
      {
        const uint32_t pr = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane - 1u) * 4u), (int)P);
        r[0] = hl == 0 ? carry : pr;
      }
#pragma unroll
      for (uint32_t ch = 1; ch < NCH; ++ch) r[ch] = z48(r[ch - 1]) ^ la[ch - 1];
      // pass B: word checks; a valid hit at byte bi of the segment means base + bi + 1 in [m + 4, L]
      const int64_t lo64 = m + 3 - base, hi64 = L - 1 - base;
      const int32_t vlo = lo64 < 0 ? 0 : (lo64 > (int64_t)SEG ? (int32_t)SEG : (int32_t)lo64);
      const int32_t vhi = hi64 < 0 ? -1 : (hi64 > (int64_t)SEG ? (int32_t)SEG : (int32_t)hi64);
      const uint64_t actm = __builtin_amdgcn_ballot_w64(act);
      uint32_t best = 0xFFu;  // the lane's smallest valid hit byte (0xFF: none)
#pragma unroll
      for (uint32_t i = 0; i < CW; ++i) {
#pragma unroll
        for (uint32_t ch = 0; ch < NCH; ++ch) {
          const uint32_t j = CW * ch + i, w = u[j], rr = r[ch];
          const bool h1 = (rr ^ (w & 0xFFu)) == kResBack1, h2 = (rr ^ (w & 0xFFFFu)) == kResBack2;
          const bool h3 = (rr ^ (w & 0xFFFFFFu)) == kResBack3;
          const uint32_t xx = rr ^ w;
          const bool h4 = xx == kResBack4;
          const uint64_t any = (__builtin_amdgcn_ballot_w64(h1) | __builtin_amdgcn_ballot_w64(h2) |
                                __builtin_amdgcn_ballot_w64(h3) | __builtin_amdgcn_ballot_w64(h4)) & actm;
          if (any) {
            const bool hk[4] = {h1, h2, h3, h4};
#pragma unroll
            for (uint32_t kk = 0; kk < 4; ++kk) {
              const int32_t bi = (int32_t)(4 * j + kk);
              if (hk[kk] && bi >= vlo && bi <= vhi && (uint32_t)bi < best) best = (uint32_t)bi;
            }
          }
          if (i + 1 < CW) r[ch] = ustep_xor(lds, xx, 0u, ub0, ub1);
        }
      }
      const uint64_t hitm = __builtin_amdgcn_ballot_w64(best != 0xFFu) & actm;
      if (hitm) {
        const uint32_t om = (uint32_t)(hitm >> (LPC * oct)) & ((1u << LPC) - 1u);
        const uint32_t fl = LPC * oct + (om ? (uint32_t)__builtin_ctz(om) : 0u);
        const uint32_t fb = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(fl * 4u), (int)best);
        if (act && om) found = B + (int64_t)(SEG * (fl - LPC * oct) + fb) + 1 - 4;
      }
      carry = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((lane | (LPC - 1)) * 4u), (int)P);
      act = act && found < 0 && B + (int64_t)(LPC * SEG) < L;
    }
    if (live && hl == 0) result[c] = found;
  }
}

#ifdef LNX_RESEARCH
#include "research/search_research.inc"
#endif

hipError_t launch_crc32_search(const uint8_t* bytes, const uint64_t* off, const int64_t* min_off, uint64_t n,
                               const uint32_t* tables, int64_t* result, int num_cus, hipStream_t stream) {
  if (n == 0) return hipSuccess;
  auto launch_octets = [&]() {
    uint64_t g1 = ((n + 7) / 8 + kSegBlock / 64 - 1) / (kSegBlock / 64);
    if (g1 > (uint64_t)num_cus) g1 = (uint64_t)num_cus;
    hipLaunchKernelGGL(crc32_search_o_kernel, dim3((unsigned)g1), dim3(kSegBlock), 0, stream, bytes, off, min_off, n,
                       tables, result);
  };
#ifndef LNX_RESEARCH
  // product: octet segments, 8 captures per wave (r4)
  launch_octets();
  return hipGetLastError();
#else
  (void)launch_octets;
  return launch_crc32_search_research(bytes, off, min_off, n, tables, result, num_cus, stream);
#endif
}

}  // namespace lnx
