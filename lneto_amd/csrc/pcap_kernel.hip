// pcap_kernel.hip — pcap's checksum re-verification over a batch, gfx950
// (the verify callers; the capture tool's variant).
//
// For every Ethernet frame, the status lneto's packet-capture breakdown records
// about its checksums (PacketBreakdown.CaptureEthernet / CaptureIPv4 /
// CaptureIPv6, internet/pcap/capture.go:67-277), which differs from the
// receive path's (ingress_kernel.hip):
//   - a bad IPv4 header sum is recorded and the transport check still runs
//     (:229-231);
//   - on IPv4 the TCP / UDP checks run only when tcp / udp.NewFrame accept the
//     payload, and their size checks end the capture (:241-266); a UDP
//     checksum of 0 is not checked (:259); ICMPv4 is always summed, with no
//     pseudo-header (:267-273);
//   - IPv6 sums TCP over the payload and UDP / UDPLite over the UDP length
//     (:179-199), the pseudo-header from CRCWritePseudo (ipv6/frame.go:104-108).
// status = bit 0 IPv4 header sum bad, bit 1 transport sum bad, bits 2-7 the
// errGeneric code (errors.go:6-28) of a size check that ends the capture on the
// way to the transport check (IPv6 UDP: the one recorded in its place).
//
// Layout: four frames per wave, one per 16-lane row, frames grid-strided,
// every check per lane in the vector unit (no scalar work per frame).  A row
// loads its frame's first 1536 bytes at once (six 16-byte blocks per lane,
// from the block holding byte 0), realigns the first 128 into frame-aligned
// dwords across the row (ds_bpermute + v_alignbyte) and reads each header
// field with one ds_bpermute; the checks are selects in capture order.  The
// same registers (and, past 1536 bytes, further 16-byte loads) then sum the
// header [14, 34) and the transport bytes (pseudo-header addresses + segment)
// at once: two (E, O) pairs of v_dot4_u32_u8 sums of the bytes at even / odd
// frame offsets (every segment starts at an even offset, so its sum of
// big-endian words is 256 E + O, as in sum16_kernel.hip), reduced within the
// row.  A block holding one of the frame's bytes lies in that byte's page, so
// the loads never fault.
#include <hip/hip_runtime.h>
#include <cstdint>

namespace lnx {

constexpr int kPcapBlock = 256;
constexpr uint32_t kPcapErrInvalidLengthField = 15, kPcapErrTruncatedFrame = 18;

__device__ __forceinline__ uint32_t pcap_keep_from(int32_t lo) {
  lo = lo < 0 ? 0 : (lo > 4 ? 4 : lo);
  return (uint32_t)(0xFFFFFFFFull << (8 * lo));
}
// byte mask of the frame offsets [a, b) inside the dword whose byte 0 is at o
__device__ __forceinline__ uint32_t pcap_range(int32_t o, int32_t a, int32_t b) {
  return pcap_keep_from(a - o) & ~pcap_keep_from(b - o);
}

__device__ __forceinline__ uint32_t pcap_fold(uint32_t sum) {  // crc.go:17-21
  sum = (sum & 0xffffu) + (sum >> 16);
  return (uint16_t)~(uint16_t)(sum + (sum >> 16));
}

// the sums' contributions of one 16-byte block at frame offset o
__device__ __forceinline__ void pcap_block(const uint4& v, int32_t o, int32_t hA, int32_t hB, int32_t a1, int32_t b1,
                                           int32_t a2, int32_t b2, uint32_t& hE, uint32_t& hO, uint32_t& tE,
                                           uint32_t& tO) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int32_t oj = o + 4 * j;
    const uint32_t xh = w[j] & pcap_range(oj, hA, hB);
    const uint32_t xt = w[j] & (pcap_range(oj, a1, b1) | pcap_range(oj, a2, b2));
    hE = __builtin_amdgcn_udot4(xh, 0x00010001u, hE, false);
    hO = __builtin_amdgcn_udot4(xh, 0x01000100u, hO, false);
    tE = __builtin_amdgcn_udot4(xt, 0x00010001u, tE, false);
    tO = __builtin_amdgcn_udot4(xt, 0x01000100u, tO, false);
  }
}

// The row form: four frames per wave, one per 16-lane row, every check per
// lane in the vector unit (no scalar work per frame).  A row's window is
// kPcapSlots 16-byte blocks per lane (block b of the frame's window in lane
// b % 16, slot b / 16); the header's frame-aligned dwords 0..31 are H0 / H1 of
// the row's lanes (dword k in lane k % 16), realigned by ds_bpermute within
// the row; a field is one ds_bpermute from the lane holding its dword.
constexpr int kPcapSlots = 6;                       // 1536-byte window a row
constexpr int32_t kPcapRowWin = 16 * 16 * kPcapSlots;

__device__ __forceinline__ uint32_t pcap_bperm(uint32_t lane_idx, uint32_t v) {
  return (uint32_t)__builtin_amdgcn_ds_bpermute((int)(lane_idx << 2), (int)v);
}

__global__ void __launch_bounds__(kPcapBlock)
pcap_rows_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t n,
                 uint8_t* __restrict__ status) {
  const uint32_t lane = threadIdx.x & 63u, rl = lane & 15u, rbase = lane & 48u;
  const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t stride = (uint64_t)gridDim.x * (kPcapBlock / 64);
  for (uint64_t g = (uint64_t)blockIdx.x * (kPcapBlock / 64) + wave; g * 4 < n; g += stride) {
    const uint64_t f = g * 4 + (lane >> 4);
    const bool valid = f < n;
    const uint64_t s = valid ? off[f] : 0, e = valid ? off[f + 1] : 0;
    const uint64_t L = e > s ? e - s : 0;  // an end below its start: an empty frame
    const uint8_t* p = bytes + s;
    const uint32_t q = (uint32_t)((uintptr_t)p & 15u);
    const uint64_t nb64 = L == 0 ? 0 : ((uint64_t)q + L + 15) >> 4;
    const uint32_t nb = nb64 < (uint64_t)(16 * kPcapSlots) ? (uint32_t)nb64 : 16u * kPcapSlots;
    const uint32_t nbmax = max(max((uint32_t)__builtin_amdgcn_readlane((int)nb, 0), (uint32_t)__builtin_amdgcn_readlane((int)nb, 16)),
                               max((uint32_t)__builtin_amdgcn_readlane((int)nb, 32), (uint32_t)__builtin_amdgcn_readlane((int)nb, 48)));
    uint4 w[kPcapSlots];
#pragma unroll
    for (int k = 0; k < kPcapSlots; ++k) {
      const uint32_t b = 16u * k + rl;
      w[k] = uint4{0u, 0u, 0u, 0u};
      if (b < nb) w[k] = *reinterpret_cast<const uint4*>(p - q + 16 * b);
    }
    // frame-aligned header dwords: H0 = dword rl, H1 = dword rl + 16 of the frame
    auto realign = [&](uint32_t k) -> uint32_t {
      const uint32_t dw = (q >> 2) + k, src = rbase + (dw >> 2);  // (dw >> 2) <= 8: slot 0
      const uint32_t c0 = pcap_bperm(src, w[0].x), c1 = pcap_bperm(src, w[0].y);
      const uint32_t c2 = pcap_bperm(src, w[0].z), c3 = pcap_bperm(src, w[0].w);
      const uint32_t n0 = pcap_bperm(src + 1, w[0].x);
      const uint32_t sel = dw & 3u;
      const uint32_t lo = sel == 0 ? c0 : sel == 1 ? c1 : sel == 2 ? c2 : c3;
      const uint32_t hi = sel == 0 ? c1 : sel == 1 ? c2 : sel == 2 ? c3 : n0;
      return __builtin_amdgcn_alignbyte(hi, lo, q & 3u);
    };
    const uint32_t H0 = realign(rl), H1 = realign(rl + 16);
    auto D = [&](uint32_t k) -> uint32_t {  // frame dword k < 32 of this lane's row
      const uint32_t a = pcap_bperm(rbase + (k & 15u), H0), b = pcap_bperm(rbase + (k & 15u), H1);
      return k < 16 ? a : b;
    };
    auto Bk = [](uint32_t dword, uint32_t k) -> uint32_t { return (dword >> (8 * (k & 3u))) & 0xFFu; };
    auto BE16 = [&](uint32_t dword, uint32_t k) -> uint32_t { return (Bk(dword, k) << 8) | Bk(dword, k + 1); };
    // every field up front (offsets < 128 whatever the header holds), the
    // checks as selects in capture order, first error kept (the bytes read
    // past L never decide anything: each is used only behind its length check)
    const uint32_t d3 = pcap_bperm(rbase + 3, H0), d4 = pcap_bperm(rbase + 4, H0);
    const uint32_t d5 = pcap_bperm(rbase + 5, H0), d14 = pcap_bperm(rbase + 14, H0);
    const uint32_t Lc = L < 0x100000u ? (uint32_t)L : 0x100000u;
    const uint32_t il = Lc - 14;
    const uint32_t et = BE16(d3, 12);
    const uint32_t ce = Lc < 14 ? kPcapErrTruncatedFrame
                        : (et <= 1500 && Lc < et) ? kPcapErrInvalidLengthField
                        : (et == 0x8100 && Lc < 18) ? kPcapErrTruncatedFrame : 0u;
    const uint32_t tl = BE16(d4, 16), ihl = Bk(d3, 14) & 15u, hl = ihl * 4, proto4 = Bk(d5, 23);
    const uint32_t p0 = 14 + hl, plen = tl - hl;
    const uint32_t c4 = il < 20 ? kPcapErrTruncatedFrame : tl < 20 ? kPcapErrInvalidLengthField
                        : tl > il ? kPcapErrTruncatedFrame : (ihl < 5 || hl > tl) ? kPcapErrInvalidLengthField : 0u;
    // p0 = 2 mod 4: the UDP length at bytes 2-3 of dword (p0 + 4) / 4, its
    // checksum at bytes 0-1 of the next, the TCP data offset at byte 2 of (p0 + 12) / 4
    const uint32_t du = D((p0 + 4) >> 2), dc = D((p0 + 6) >> 2), dt = D((p0 + 12) >> 2);
    const uint32_t doff = (Bk(dt, p0 + 12) >> 4) * 4, ul4 = BE16(du, p0 + 4), ck4 = BE16(dc, p0 + 6);
    const bool tcp4 = proto4 == 6 && plen >= 20, udp4 = proto4 == 17 && plen >= 8, icmp4 = proto4 == 1 && plen >= 8;
    const uint32_t ct4 = tcp4 ? (doff < 20 ? kPcapErrInvalidLengthField : doff > plen ? kPcapErrTruncatedFrame : 0u)
                         : udp4 ? (ul4 < 8 ? kPcapErrInvalidLengthField : ul4 > plen ? kPcapErrTruncatedFrame : 0u) : 0u;
    const bool t4 = ct4 == 0 && (tcp4 || (udp4 && ck4 != 0) || icmp4);
    const uint32_t pl = BE16(d4, 18), proto6 = Bk(d5, 20), ul6 = BE16(d14, 58);
    const uint32_t c6 = il < 40 ? kPcapErrTruncatedFrame : pl + 40 > il ? kPcapErrInvalidLengthField : 0u;
    const bool tcp6 = proto6 == 6, udp6 = proto6 == 17 || proto6 == 136;
    const uint32_t ct6 = udp6 ? (pl < 8 ? kPcapErrTruncatedFrame : ul6 < 8 ? kPcapErrInvalidLengthField
                                 : ul6 > pl ? kPcapErrTruncatedFrame : 0u) : 0u;
    const bool is4 = ce == 0 && et == 0x0800 && c4 == 0, is6 = ce == 0 && et == 0x86DD && c6 == 0;
    const uint32_t code = ce ? ce : et == 0x0800 ? (c4 ? c4 : ct4) : et == 0x86DD ? (c6 ? c6 : ct6) : 0u;
    const bool sum_h = is4, sum_t = (is4 && t4) || (is6 && ct6 == 0 && (tcp6 || udp6));
    const int32_t a1 = sum_t ? (is4 ? (icmp4 ? 0 : 26) : 22) : 0;
    const int32_t b1 = sum_t ? (is4 ? (icmp4 ? 0 : 34) : (int32_t)(54 + (tcp6 ? pl : ul6))) : 0;
    const int32_t a2 = sum_t && is4 ? (int32_t)p0 : 0;
    const int32_t b2 = sum_t && is4 ? (int32_t)(p0 + (udp4 ? ul4 : plen)) : 0;
    const uint32_t seed = is4 ? (tcp4 ? plen + 6 : udp4 ? ul4 + 17 : 0u) : pl + proto6;
    const int32_t hA = sum_h ? 14 : 0, hB = sum_h ? 34 : 0;
    const int32_t hi = sum_t ? (b2 > a2 ? b2 : b1) : 34;
    uint32_t hE = 0, hO = 0, tE = 0, tO = 0;
#pragma unroll
    for (int k = 0; k < kPcapSlots; ++k)  // (a slot no row's frame reaches holds zeros: skipped)
      if (k == 0 || 16u * k < nbmax)
        pcap_block(w[k], 16 * (int32_t)(16 * k + rl) - (int32_t)q, hA, hB, a1, b1, a2, b2, hE, hO, tE, tO);
    if (sum_t)  // past the window (frames over ~1.5 KiB)
      for (int32_t o = kPcapRowWin - (int32_t)q + 16 * (int32_t)rl; o < hi; o += 256)
        pcap_block(*reinterpret_cast<const uint4*>(p + o), o, hA, hB, a1, b1, a2, b2, hE, hO, tE, tO);
    uint32_t hs = (q & 1) ? (hO << 8) + hE : (hE << 8) + hO;
    uint32_t ts = (q & 1) ? (tO << 8) + tE : (tE << 8) + tO;
#pragma unroll
    for (int sft = 1; sft < 16; sft <<= 1) {  // within the row
      hs += (uint32_t)__shfl_xor((int)hs, sft, 16);
      ts += (uint32_t)__shfl_xor((int)ts, sft, 16);
    }
    uint32_t st = code << 2;
    if (sum_h && pcap_fold(hs) != 0) st |= 1u;
    if (sum_t && pcap_fold(ts + seed) != 0) st |= 2u;
    if (valid && rl == 0) status[f] = (uint8_t)st;
  }
}

hipError_t launch_pcap_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint8_t* status, int num_cus,
                              hipStream_t stream) {
  if (n == 0) return hipSuccess;
  constexpr uint64_t frames_per_block = kPcapBlock / 16;  // four frames a wave
  uint64_t grid = (n + frames_per_block - 1) / frames_per_block;
  const uint64_t cap = (uint64_t)num_cus * 64;
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL(pcap_rows_kernel, dim3((unsigned)grid), dim3(kPcapBlock), 0, stream, bytes, off, n, status);
  return hipGetLastError();
}

}  // namespace lnx
