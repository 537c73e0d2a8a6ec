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
// Layout: one wave per frame, frames grid-strided.  The wave loads the frame's
// first 2 KiB at once (two 16-byte blocks per lane, from the block holding
// byte 0); the header's first 128 bytes are realigned across lanes into
// frame-aligned dwords (ds_bpermute + v_alignbyte) and every header field is
// a v_readlane of one of them, so the whole decision is scalar and costs no
// second round trip.  The same
// registers (and, past 2 KiB, further 16-byte loads) then sum the header
// [14, 34) and the transport bytes (pseudo-header addresses + segment) at once:
// two (E, O) pairs of v_dot4_u32_u8 sums of the bytes at even / odd frame
// offsets (every segment starts at an even offset, so its sum of big-endian
// words is 256 E + O, as in sum16_kernel.hip).  A block holding one of the
// frame's bytes lies in that byte's page, so the loads never fault.
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

// a frame's first kPcapWin bytes come in with two 16-byte loads per lane
// issued before the header is parsed (the window's blocks: lane and lane + 64)
constexpr int32_t kPcapWin = 2048;

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

__global__ void __launch_bounds__(kPcapBlock)
pcap_verify_kernel(const uint8_t* __restrict__ bytes, const uint64_t* __restrict__ off, uint64_t n,
                   uint8_t* __restrict__ status) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t stride = (uint64_t)gridDim.x * (kPcapBlock / 64);
  // the window of frame [s, e): 16-byte blocks from the one holding byte 0,
  // those holding frame bytes up to the window's 128
  auto window = [&](uint64_t s, uint64_t e, uint4& v0, uint4& v1) {
    const uint64_t L = e > s ? e - s : 0;
    const uint8_t* p = bytes + s;
    const uint32_t q = (uint32_t)((uintptr_t)p & 15u);
    const uint64_t nb64 = L == 0 ? 0 : ((uint64_t)q + L + 15) >> 4;
    const uint32_t nb = nb64 < 128 ? (uint32_t)nb64 : 128u;
    // a buffer descriptor of nb blocks: the range check returns 0 for the
    // blocks past them, so every lane issues both loads (no branch around
    // them, and the wait before this frame's use counts the next frame's
    // loads instead of draining them); an empty frame touches no memory
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p - q), 0, (int)(16 * nb), 0x00020000);
    const auto r0 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * lane, 0, 0);
    const auto r1 = __builtin_amdgcn_raw_buffer_load_b128(rsrc, 16 * (lane + 64), 0, 0);
    v0 = uint4{r0[0], r0[1], r0[2], r0[3]};
    v1 = uint4{r1[0], r1[1], r1[2], r1[3]};
  };
  // the status of frame f = [s, e) from its window v0, v1
  auto check = [&](uint64_t f, uint64_t s, uint64_t e, const uint4& v0, const uint4& v1) {
    const uint64_t L = e > s ? e - s : 0;  // an end below its start: an empty frame
    const uint8_t* p = bytes + s;
    const int32_t q = (int32_t)((uintptr_t)p & 15u);
    // The header as frame-aligned dwords: lane l < 32 holds frame bytes
    // [4l, 4l + 4), window dwords j + l and j + l + 1 (j = q / 4) joined by
    // v_alignbyte at q % 4; the window dwords come from their lanes by
    // ds_bpermute (the four of lane (j + l) / 4 and the first of the next).
    // Then a header byte is one v_readlane at a wave-uniform lane index.
    // Every byte the checks below use lies inside the frame (each is read
    // after the length check that covers it), so bytes past L need no masking
    const uint32_t dw = ((uint32_t)q >> 2) + lane, src = (dw >> 2) << 2;
    const uint32_t c0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)v0.x);
    const uint32_t c1 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)v0.y);
    const uint32_t c2 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)v0.z);
    const uint32_t c3 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src, (int)v0.w);
    const uint32_t n0 = (uint32_t)__builtin_amdgcn_ds_bpermute((int)src + 4, (int)v0.x);
    const uint32_t sel = dw & 3u;
    const uint32_t lo = sel == 0 ? c0 : sel == 1 ? c1 : sel == 2 ? c2 : c3;
    const uint32_t hi = sel == 0 ? c1 : sel == 1 ? c2 : sel == 2 ? c3 : n0;
    const uint32_t H = __builtin_amdgcn_alignbyte(hi, lo, (uint32_t)q & 3u);
    auto B = [&](uint32_t k) -> uint32_t {  // frame byte k < 128, k wave-uniform
      return ((uint32_t)__builtin_amdgcn_readlane((int)H, (int)(k >> 2)) >> (8 * (k & 3u))) & 0xFFu;
    };
    auto BE16 = [&](uint32_t k) -> uint32_t { return (B(k) << 8) | B(k + 1); };

    uint32_t code = 0, seed = 0;
    bool sum_h = false, sum_t = false;
    int32_t a1 = 0, b1 = 0, a2 = 0, b2 = 0;  // transport ranges: pseudo-header addresses, segment
    if (L < 14) {
      code = kPcapErrTruncatedFrame;                       // ethernet.NewFrame (:74-77)
    } else {
      const uint32_t et = BE16(12);
      if (et <= 1500 && L < et) {
        code = kPcapErrInvalidLengthField;                 // ValidateSize (ethernet/frame.go:119-127)
      } else if (et == 0x8100 && L < 18) {
        code = kPcapErrTruncatedFrame;
      } else if (et == 0x0800) {                           // CaptureIPv4 (:203-277)
        const uint64_t il = L - 14;
        const uint32_t tl = BE16(16), ihl = B(14) & 15u;
        if (il < 20) code = kPcapErrTruncatedFrame;        // ipv4.NewFrame
        else if (tl < 20) code = kPcapErrInvalidLengthField;  // ValidateSize, first error kept
        else if (tl > il) code = kPcapErrTruncatedFrame;
        else if (ihl < 5 || ihl * 4 > tl) code = kPcapErrInvalidLengthField;
        else {
          sum_h = true;                                    // CalculateHeaderCRC: bytes [14, 34)
          const uint32_t proto = B(23), p0 = 14 + ihl * 4, plen = tl - ihl * 4;
          if (proto == 6 && plen >= 20) {                  // tcp.NewFrame accepts the payload
            const uint32_t doff = (B(p0 + 12) >> 4) * 4;   // tcp ValidateSize ends the capture
            if (doff < 20) code = kPcapErrInvalidLengthField;
            else if (doff > plen) code = kPcapErrTruncatedFrame;
            else { sum_t = true; a1 = 26; b1 = 34; a2 = p0; b2 = p0 + plen; seed = plen + 6; }
          } else if (proto == 17 && plen >= 8) {           // udp.NewFrame accepts the payload
            const uint32_t ul = BE16(p0 + 4);
            if (ul < 8) code = kPcapErrInvalidLengthField;
            else if (ul > plen) code = kPcapErrTruncatedFrame;
            else if (BE16(p0 + 6) != 0) { sum_t = true; a1 = 26; b1 = 34; a2 = p0; b2 = p0 + ul; seed = ul + 17; }
          } else if (proto == 1 && plen >= 8) {            // icmpv4.NewFrame; no pseudo-header
            sum_t = true; a2 = p0; b2 = p0 + plen;
          }
        }
      } else if (et == 0x86DD) {                           // CaptureIPv6 (:159-201)
        const uint64_t il = L - 14;
        const uint32_t pl = BE16(18), proto = B(20);
        if (il < 40) code = kPcapErrTruncatedFrame;        // ipv6.NewFrame
        else if (pl + 40 > il) code = kPcapErrInvalidLengthField;  // ValidateSize
        else if (proto == 6) { sum_t = true; a1 = 22; b1 = 54 + pl; seed = pl + 6; }
        else if (proto == 17 || proto == 136) {
          if (pl < 8) code = kPcapErrTruncatedFrame;       // udp.NewFrame on the payload
          else {
            const uint32_t ul = BE16(58);
            if (ul < 8) code = kPcapErrInvalidLengthField;
            else if (ul > pl) code = kPcapErrTruncatedFrame;
            else { sum_t = true; a1 = 22; b1 = 54 + ul; seed = pl + proto; }
          }
        }
      }
    }

    uint32_t st = code << 2;
    if (sum_h || sum_t) {
      const int32_t hi = sum_t ? (b2 > a2 ? b2 : b1) : 34;
      const int32_t hA = sum_h ? 14 : 0, hB = sum_h ? 34 : 0;
      uint32_t hE = 0, hO = 0, tE = 0, tO = 0;
      // the window's blocks from registers (ranges outside [0, L) never reach
      // them: every range ends at or below L), then past the window from memory
      pcap_block(v0, 16 * (int32_t)lane - q, hA, hB, a1, b1, a2, b2, hE, hO, tE, tO);
      pcap_block(v1, 16 * (int32_t)(lane + 64) - q, hA, hB, a1, b1, a2, b2, hE, hO, tE, tO);
      for (int32_t o = kPcapWin - q + 16 * (int32_t)lane; o < hi; o += 1024)
        pcap_block(*reinterpret_cast<const uint4*>(p + o), o, hA, hB, a1, b1, a2, b2, hE, hO, tE, tO);
      // byte 0 of every dword sits at an even frame offset iff the frame starts at an even address
      uint32_t hs = (q & 1) ? (hO << 8) + hE : (hE << 8) + hO;
      uint32_t ts = (q & 1) ? (tO << 8) + tE : (tE << 8) + tO;
#pragma unroll
      for (int sft = 1; sft < 64; sft <<= 1) {
        hs += (uint32_t)__shfl_xor((int)hs, sft);
        ts += (uint32_t)__shfl_xor((int)ts, sft);
      }
      if (sum_h && pcap_fold(hs) != 0) st |= 1u;
      if (sum_t && pcap_fold(ts + seed) != 0) st |= 2u;
    }
    if (lane == 0) status[f] = (uint8_t)st;
  };
  // two frames in flight per wave: the next one's offsets and window load
  // while this one is checked; the roles alternate (A, B) so that no register
  // copy waits for a window early
  uint64_t f = (uint64_t)blockIdx.x * (kPcapBlock / 64) + wave;
  if (f >= n) return;
  uint64_t sA = off[f], eA = off[f + 1], sB = 0, eB = 0;
  uint4 xa0, xa1, xb0, xb1;
  window(sA, eA, xa0, xa1);
  // (the next window's loads are issued unconditionally, an empty one past
  // the wave's last frame: a load skipped on one path would make the compiler
  // wait for every load before this frame's first use)
  for (;;) {
    uint64_t fn = f + stride;
    bool more = fn < n;
    sB = off[more ? fn : f];
    eB = more ? off[fn + 1] : sB;
    window(sB, eB, xb0, xb1);
    check(f, sA, eA, xa0, xa1);
    if (!more) break;
    f = fn;
    fn = f + stride;
    more = fn < n;
    sA = off[more ? fn : f];
    eA = more ? off[fn + 1] : sA;
    window(sA, eA, xa0, xa1);
    check(f, sB, eB, xb0, xb1);
    if (!more) break;
    f = fn;
  }
}

hipError_t launch_pcap_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint8_t* status, int num_cus,
                              hipStream_t stream) {
  if (n == 0) return hipSuccess;
  constexpr uint64_t frames_per_block = kPcapBlock / 64;
  uint64_t grid = (n + frames_per_block - 1) / frames_per_block;
  const uint64_t cap = (uint64_t)num_cus * 64;  // 16 waves per SIMD's worth of blocks, then grid-stride
  if (grid > cap) grid = cap;
  hipLaunchKernelGGL(pcap_verify_kernel, dim3((unsigned)grid), dim3(kPcapBlock), 0, stream, bytes, off, n, status);
  return hipGetLastError();
}

}  // namespace lnx
