// api.cpp — C-ABI of the batched HIP path: per-device context (the LDS table
// image), argument checks, host-memory and multi-GPU conveniences.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>
#include "../../include/lneto_amd.h"
#include "gf2.hpp"
#include "lds_layout.hpp"
#include "rx_filter.hpp"
#include "dispatch.hpp"

namespace lnx {
hipError_t launch_crc32_frames(const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out,
                               bool verify, const void* image, int num_cus, hipStream_t stream, uint32_t policy,
                               uint32_t* stage_flag, uint32_t epoch);
hipError_t launch_crc32_stage(const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out, bool verify,
                              uint32_t policy, const void* image, uint32_t* scratch, int num_cus, hipStream_t stream,
                              const uint32_t* stage_flag, uint32_t epoch);
#ifdef LNX_RESEARCH
namespace rs {
hipError_t launch_crc32_stage_research(const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out, bool verify,
                                       int fold, int waves, const void* image, int num_cus, hipStream_t stream,
                                       bool big_blocks = false);
}
hipError_t launch_crc32_variant(int var, const uint8_t* bytes, const uint64_t* off, uint64_t n, void* out,
                                const void* image, int num_cus, hipStream_t stream, uint64_t* timeline);
uint64_t crc32_launch_waves(uint64_t n, int num_cus);
hipError_t launch_fcs_scatter(uint8_t* bytes, const uint64_t* start, uint32_t* len, const uint32_t* crc, uint64_t n,
                              uint32_t capacity, uint8_t* status, int num_cus, hipStream_t stream);
#endif
hipError_t launch_rx_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t flags, bool fcs,
                            uint8_t* ok, uint8_t* verdict, const uint32_t* seg_len, const RxFilter* filter,
                            const uint32_t* image, int num_cus, hipStream_t stream, bool host = false,
                            const uint32_t* gate = nullptr, uint32_t epoch = 0);
hipError_t launch_pcap_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint8_t* status, int num_cus,
                              hipStream_t stream);
hipError_t launch_ingress_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t flags,
                                 uint8_t* verdict, int num_cus, hipStream_t stream, const uint32_t* seg_len,
                                 uint32_t trim, const RxFilter* filter, uint32_t* gate = nullptr, uint32_t epoch = 0,
                                 uint64_t short_mean = 0);
hipError_t launch_crc32_search(const uint8_t* bytes, const uint64_t* off, const int64_t* min_off, uint64_t n,
                               const uint32_t* tables, int64_t* result, int num_cus, hipStream_t stream);
hipError_t launch_crc32_segments(const uint8_t* bytes, const uint64_t* start, const uint32_t* len, uint64_t n,
                                 void* out, const void* images, int num_cus, hipStream_t stream);
hipError_t launch_fcs_append(uint8_t* bytes, const uint64_t* start, uint32_t* len, uint64_t n, uint32_t capacity,
                             uint8_t* status, const void* images, int num_cus, hipStream_t stream, int var = 0);
hipError_t launch_tx_checksum(uint8_t* bytes, const uint64_t* start, const uint32_t* len, uint64_t n,
                              uint8_t* status, int num_cus, hipStream_t stream, uint32_t* gate = nullptr,
                              uint32_t epoch = 0, uint64_t short_mean = 0);
hipError_t launch_tx_finish(uint8_t* bytes, const uint64_t* start, uint32_t* len, uint64_t n, uint32_t capacity,
                            uint32_t flags, uint8_t* st_ck, uint8_t* st_ap, const uint32_t* image, int num_cus,
                            hipStream_t stream, bool host, const uint32_t* gate = nullptr, uint32_t epoch = 0);
hipError_t launch_sum16_segments(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                                 const uint32_t* seed, uint64_t n, uint16_t* out, int num_cus,
                                 hipStream_t stream, int var = 0);

// The 160 KiB LDS image of row width rl (lds_layout.hpp), built once on the host.
std::vector<uint32_t> build_lds_image(uint32_t rl) {
  std::vector<uint32_t> img(kLdsDwords, 0);
  const int64_t sb = 4 * (int64_t)rl;
  for (uint32_t m = 0; m < 4; ++m) {
    for (uint32_t e = 0; e < 256; ++e) {
      const uint32_t v = zshift_bytes(e << (8 * m), sb);  // U_m[e] = Z_SB(e << 8m)
      for (uint32_t c = 0; c < 32; ++c) img[u_addr(m, e, c) / 4] = v;
    }
  }
  for (uint32_t c = 0; c < 32; ++c) {
    const int64_t p = c % rl;
    for (uint32_t i = 0; i < 8; ++i)
      for (uint32_t v = 0; v < 16; ++v)
        img[f_addr(c, i, v) / 4] = zshift_bytes(v << (4 * i), -4 * p);  // F_p = Z_{-4p}
    const uint32_t q0 = (uint32_t)p & 7u;
    for (uint32_t h = 0; h < 2; ++h)
      for (uint32_t t = 1; t < 4; ++t)
        for (uint32_t v = 0; v < 16; ++v)
          img[t_addr(c, h, t, v) / 4] = zshift_bytes(v << (4 * (q0 + 4 * h)), -(int64_t)t);  // Z_{-t}
  }
  return img;
}

#ifdef LNX_RESEARCH
// The LDS image of the streaming rows (stream_rows.hpp) with row steps of SB
// bytes (128: 8-lane rows, 64: 4-lane rows): U = Z_4 (the chain's dword step),
// F column n = Z_{-4n} (n = 0..31), then the Z_{SB-12} byte tables (the skip
// over the other lanes' pieces, at kSZ116), Z_c (c = 0..3) and Z_{SB-4k}
// (k = 0..4) nibble tables by row lane, the constants Z_{SB-j}(0xFFFFFFFF) and
// the Z_1 byte table.
std::vector<uint32_t> build_stream_image(int64_t sb) {
  std::vector<uint32_t> img(kLdsDwords, 0);
  for (uint32_t m = 0; m < 4; ++m)
    for (uint32_t e = 0; e < 256; ++e) {
      const uint32_t v = zshift_bytes(e << (8 * m), 4);
      for (uint32_t c = 0; c < 32; ++c) img[u_addr(m, e, c) / 4] = v;
    }
  for (uint32_t c = 0; c < 32; ++c)
    for (uint32_t i = 0; i < 8; ++i)
      for (uint32_t v = 0; v < 16; ++v) img[f_addr(c, i, v) / 4] = zshift_bytes(v << (4 * i), -4 * (int64_t)c);
  for (uint32_t m = 0; m < 4; ++m)
    for (uint32_t e = 0; e < 256; ++e) img[(kSZ116 + 1024 * m + 4 * e) / 4] = zshift_bytes(e << (8 * m), sb - 12);
  for (uint32_t c = 0; c < 4; ++c)
    for (uint32_t p = 0; p < 8; ++p)
      for (uint32_t v = 0; v < 16; ++v) img[kSTc / 4 + (c * 8 + p) * 16 + v] = zshift_bytes(v << (4 * p), c);
  for (uint32_t k = 0; k < 5; ++k)
    for (uint32_t p = 0; p < 8; ++p)
      for (uint32_t v = 0; v < 16; ++v)
        img[kSG / 4 + (k * 8 + p) * 16 + v] = zshift_bytes(v << (4 * p), sb - 4 * (int64_t)k);
  for (uint32_t j = 0; j < 16; ++j) img[kSK / 4 + j] = zshift_bytes(0xFFFFFFFFu, sb - (int64_t)j);
  for (uint32_t e = 0; e < 256; ++e) img[kST1 / 4 + e] = zshift_bytes(e, 1);
  return img;
}

// The LDS image of the lane streams (stream_lanes.hpp): U = Z_4, then the
// Z_c byte tables (c = 1..3), the Z_{64-4k} nibble tables (k = 0..15) and
// the constants Z_{64-j}(0xFFFFFFFF) (lds_layout.hpp kLZc, kLZd, kLK).
std::vector<uint32_t> build_lanes_image() {
  std::vector<uint32_t> img(kLdsDwords, 0);
  for (uint32_t m = 0; m < 4; ++m)
    for (uint32_t e = 0; e < 256; ++e) {
      const uint32_t v = zshift_bytes(e << (8 * m), 4);
      for (uint32_t c = 0; c < 32; ++c) img[u_addr(m, e, c) / 4] = v;
    }
  for (uint32_t c = 1; c < 4; ++c)
    for (uint32_t m = 0; m < 4; ++m)
      for (uint32_t e = 0; e < 256; ++e) img[kLZc / 4 + (c - 1) * 1024 + 256 * m + e] = zshift_bytes(e << (8 * m), c);
  for (uint32_t k = 0; k < 16; ++k)
    for (uint32_t i = 0; i < 8; ++i)
      for (uint32_t v = 0; v < 16; ++v)
        img[kLZd / 4 + 128 * k + 16 * i + v] = zshift_bytes(v << (4 * i), 64 - 4 * (int64_t)k);
  for (uint32_t j = 0; j < 64; ++j) img[kLK / 4 + j] = zshift_bytes(0xFFFFFFFFu, 64 - (int64_t)j);
  return img;
}
#endif  // LNX_RESEARCH

// The staged lane streams' image (stage_kernel.hip): the slicing-by-2 byte
// tables A[e] = Z_2(e), B[e] = Z_1(e), then Z_{2^m} as eight nibble tables
// for m = 0..30, entry (m, i, v) at dword 512 + 128 m + 16 i + v.
std::vector<uint32_t> build_stage_image() {
  std::vector<uint32_t> t(512 + 31 * 128 + 1024 + 2048 + 3 * 1024 + 4 * 1024 + 9 * 128);
  for (uint32_t e = 0; e < 256; ++e) t[e] = zshift_bytes(e, 2), t[256 + e] = zshift_bytes(e, 1);
  for (uint32_t m = 0; m < 31; ++m)
    for (uint32_t i = 0; i < 8; ++i)
      for (uint32_t v = 0; v < 16; ++v) t[512 + 128 * m + 16 * i + v] = zshift_bytes_fast(v << (4 * i), 1ull << m);
  for (uint32_t k = 0; k < 4; ++k)  // Z_4 byte tables (the FOLD 4 variants)
    for (uint32_t e = 0; e < 256; ++e) t[512 + 31 * 128 + 256 * k + e] = zshift_bytes(e << (8 * k), 4);
  for (uint32_t k = 0; k < 8; ++k)  // slicing-by-8 byte tables T8_k[e] = Z_{8-k}(e) (the FOLD 8 variants)
    for (uint32_t e = 0; e < 256; ++e) t[512 + 31 * 128 + 1024 + 256 * k + e] = zshift_bytes(e, 8 - (int)k);
  for (uint32_t z = 0; z < 3; ++z)  // Z_16, Z_32, Z_64 byte tables (the deferred-correction variants)
    for (uint32_t k = 0; k < 4; ++k)
      for (uint32_t e = 0; e < 256; ++e)
        t[512 + 31 * 128 + 1024 + 2048 + 1024 * z + 256 * k + e] = zshift_bytes(e << (8 * k), 16 << z);
  for (uint32_t z = 0; z < 4; ++z)  // Z_8, Z_16, Z_24, Z_32 byte tables (two chains per half)
    for (uint32_t k = 0; k < 4; ++k)
      for (uint32_t e = 0; e < 256; ++e)
        t[512 + 31 * 128 + 1024 + 2048 + 3 * 1024 + 1024 * z + 256 * k + e] = zshift_bytes(e << (8 * k), 8 * (z + 1));
  for (uint32_t m = 31; m < 40; ++m)  // Z_{2^m} nibble tables for m = 31..39 (giant frames' Z_d, stage_kernel.hip)
    for (uint32_t i = 0; i < 8; ++i)
      for (uint32_t v = 0; v < 16; ++v)
        t[512 + 31 * 128 + 1024 + 2048 + 3 * 1024 + 4 * 1024 + 128 * (m - 31) + 16 * i + v] =
            zshift_bytes_fast(v << (4 * i), 1ull << m);
  return t;
}

// The fused receive kernel's image (rx_verify_kernel.hip): the slicing tables
// T_k[e] = Z_128(e << 8k), T_{4+k}[e] = Z_124(e << 8k) (k < 4), then the nibble
// tables of Z_{-8q} (q < 32) and Z_{-b} (b < 8), entry (t, i, v) at 128 t + 16 i + v.
std::vector<uint32_t> build_rx_image() {
  std::vector<uint32_t> t(2048 + 56 * 128);
  for (uint32_t k = 0; k < 4; ++k)
    for (uint32_t e = 0; e < 256; ++e) {
      t[256 * k + e] = zshift_bytes(e << (8 * k), 128);
      t[256 * (4 + k) + e] = zshift_bytes(e << (8 * k), 124);
    }
  for (uint32_t q = 0; q < 40; ++q)
    for (uint32_t i = 0; i < 8; ++i)
      for (uint32_t v = 0; v < 16; ++v)
        t[2048 + 128 * q + 16 * i + v] = zshift_bytes(v << (4 * i), q < 32 ? -8 * (int64_t)q : -(int64_t)(q - 32));
  // then Z_{2^m}, m < 16: the transmit kernel's CRC corrections for the fields it writes
  for (uint32_t m = 0; m < 16; ++m)
    for (uint32_t i = 0; i < 8; ++i)
      for (uint32_t v = 0; v < 16; ++v) t[2048 + 40 * 128 + 128 * m + 16 * i + v] = zshift_bytes(v << (4 * i), 1ll << m);
  return t;
}

// Tables of crc32_search_kernel: the byte-step table, then Z_{4*2^k} as four
// byte tables for k = 0..5 (search_kernel.hip).
// Then the tables of crc32_search_seg_kernel (24-byte lane segments): the
// byte-step table replicated in 32 bank columns (entry e, column c at 32e + c),
// Z_{24*2^k} as four byte tables for k = 0..5, and Z_4 as four byte tables;
// then Z_{48*2^k} for k = 0..4 (crc32_search_half_kernel, 48-byte segments).
std::vector<uint32_t> build_search_tables() {
  constexpr uint32_t kOld = 256 + 6 * 1024, kSeg = 24;  // = kSearchSeg
  std::vector<uint32_t> t(kOld + 8192 + 7 * 1024 + 5 * 1024 + 4096 + 1024 + 4096 + 3 * 1024);
  for (uint32_t e = 0; e < 256; ++e) t[e] = zshift_bytes(e, 1);
  for (uint32_t k = 0; k < 6; ++k)
    for (uint32_t m = 0; m < 4; ++m)
      for (uint32_t e = 0; e < 256; ++e) t[256 + k * 1024 + m * 256 + e] = zshift_bytes(e << (8 * m), 4 << k);
  for (uint32_t e = 0; e < 256; ++e)
    for (uint32_t c = 0; c < 32; ++c) t[kOld + 32 * e + c] = t[e];
  for (uint32_t k = 0; k < 6; ++k)
    for (uint32_t m = 0; m < 4; ++m)
      for (uint32_t e = 0; e < 256; ++e)
        t[kOld + 8192 + k * 1024 + m * 256 + e] = zshift_bytes_fast(e << (8 * m), (uint64_t)kSeg << k);
  for (uint32_t m = 0; m < 4; ++m)  // Z_4 (slicing-by-4) for the segment folds
    for (uint32_t e = 0; e < 256; ++e) t[kOld + 8192 + 6 * 1024 + m * 256 + e] = zshift_bytes(e << (8 * m), 4);
  // crc32_search_half_kernel (48-byte segments): Z_{48*2^k} for k = 0..4
  for (uint32_t k = 0; k < 5; ++k)
    for (uint32_t m = 0; m < 4; ++m)
      for (uint32_t e = 0; e < 256; ++e)
        t[kOld + 8192 + 7 * 1024 + k * 1024 + m * 256 + e] = zshift_bytes_fast(e << (8 * m), (uint64_t)48 << k);
  // Z_4 as eight nibble tables, each entry in 32 bank columns: (i, v, c) at (16 i + v) * 32 + c
  for (uint32_t i = 0; i < 8; ++i)
    for (uint32_t v = 0; v < 16; ++v)
      for (uint32_t c = 0; c < 32; ++c)
        t[kOld + 8192 + 12 * 1024 + (16 * i + v) * 32 + c] = zshift_bytes(v << (4 * i), 4);
  // Z_24 as four byte tables (crc32_search_u_kernel's split chains: half a 48-byte segment)
  for (uint32_t m = 0; m < 4; ++m)
    for (uint32_t e = 0; e < 256; ++e) t[kOld + 8192 + 12 * 1024 + 4096 + m * 256 + e] = zshift_bytes(e << (8 * m), 24);
  // octet segments (crc32_search_o_kernel): Z_48 as eight nibble tables in 32
  // bank columns, (i, v, c) at (16 i + v) * 32 + c, then Z_{192*2^k}, k = 0..2
  constexpr uint32_t kOct = kOld + 8192 + 12 * 1024 + 4096 + 1024;
  for (uint32_t i = 0; i < 8; ++i)
    for (uint32_t v = 0; v < 16; ++v)
      for (uint32_t c = 0; c < 32; ++c) t[kOct + (16 * i + v) * 32 + c] = zshift_bytes_fast(v << (4 * i), 48);
  for (uint32_t k = 0; k < 3; ++k)
    for (uint32_t m = 0; m < 4; ++m)
      for (uint32_t e = 0; e < 256; ++e)
        t[kOct + 4096 + k * 1024 + m * 256 + e] = zshift_bytes_fast(e << (8 * m), (uint64_t)192 << k);
  return t;
}

namespace {

thread_local std::string g_last_error;

int hip_fail(hipError_t e, const char* what) {
  g_last_error = std::string(what) + ": " + hipGetErrorString(e);
  return LNX_EHIP;
}

struct DeviceCtx {
  std::mutex mu;                   // serializes initialization
  std::atomic<bool> ready{false};  // set once every field below is valid
  void* d_image = nullptr;
  int num_cus = 0;
  uint32_t* d_search = nullptr;  // crc32_search_kernel tables
  uint32_t* d_stage = nullptr;   // crc32_stage_kernel image
  uint32_t* d_rx = nullptr;      // rx_verify_kernel image
  // Per stream: the staged kernel's giant-slice slots (stage_kernel.hip
  // giant_pieces; zero between launches).  Launches on one stream run in
  // order, so each stream owns one set; streams never share one.
  // hipStreamPerThread names a different stream in every thread, so it is
  // keyed by thread too.  At most kGiantStreams sets live per device; the
  // least recently used one is freed (after a device sync) to make room.
  struct GiantScratch {
    hipStream_t stream;
    std::thread::id thread;
    uint32_t* p;
    uint64_t used;   // use counter at the last call
    uint32_t epoch;  // the last call's epoch (the staged launch's flag word, kStageFlag)
  };
  std::mutex giant_mu;
  std::vector<GiantScratch> giant;
  uint64_t giant_clock = 0;
#ifdef LNX_RESEARCH
  // Per-stream scratch of the two-launch TX append (the CRCs between its
  // launches): calls on one stream run in order, so each stream reuses its
  // buffer; it grows, after a sync of that stream, when a batch outgrows it.
  struct Scratch {
    hipStream_t stream;
    void* p;
    size_t cap;
  };
  std::mutex scratch_mu;
  std::vector<Scratch> scratch;
#endif
};

constexpr int kMaxDevices = 64;
DeviceCtx g_ctx[kMaxDevices];

// Compact form of an image (lds_layout.hpp kCompactDwords): the U values once,
// then the F/T tail verbatim.
std::vector<uint32_t> compact_image(const std::vector<uint32_t>& full) {
  std::vector<uint32_t> c(kCompactDwords);
  for (uint32_t m = 0; m < 4; ++m)
    for (uint32_t e = 0; e < 256; ++e) c[256 * m + e] = full[u_addr(m, e, 0) / 4];
  std::copy(full.begin() + kFBase / 4, full.end(), c.begin() + kCompactUDwords);
  return c;
}

// The compact images back to back: [RL = 16][RL = 4][RL = 32][stream][stream64][lanes] (lds_layout.hpp image_index).
const std::vector<uint32_t>& host_image() {
  static const std::vector<uint32_t> img = [] {
    std::vector<uint32_t> all;
#ifdef LNX_RESEARCH
    for (uint32_t rl : {16u, 4u, 32u, 8u, 9u, 10u}) {  // 8, 9: the stream images (128- and 64-byte row steps); 10: lanes
      const std::vector<uint32_t> im = compact_image(rl == 8    ? build_stream_image(128)
                                                     : rl == 9  ? build_stream_image(64)
                                                     : rl == 10 ? build_lanes_image()
                                                                : build_lds_image(rl));
      all.insert(all.end(), im.begin(), im.end());
    }
#else
    for (uint32_t rl : {16u, 4u, 32u}) {  // the product's row widths (image_index 0..2)
      const std::vector<uint32_t> im = compact_image(build_lds_image(rl));
      all.insert(all.end(), im.begin(), im.end());
    }
#endif
    return all;
  }();
  return img;
}

// Context of the calling thread's current device (created on first use).  A
// failed initialization (e.g. hipMalloc out of memory) frees what it had
// allocated and leaves the context uninitialized, so a later call retries.
int init_ctx(DeviceCtx& c, int dev) {
  auto fail = [&](hipError_t err, const char* what) {
    (void)hipFree(c.d_image);
    (void)hipFree(c.d_search);
    (void)hipFree(c.d_stage);
    (void)hipFree(c.d_rx);
    c.d_image = nullptr;
    c.d_search = nullptr;
    c.d_stage = nullptr;
    c.d_rx = nullptr;
    return hip_fail(err, what);
  };
  hipError_t err = hipDeviceGetAttribute(&c.num_cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (err != hipSuccess) return fail(err, "hipDeviceGetAttribute");
  const auto& img = host_image();
  if ((err = hipMalloc(&c.d_image, img.size() * 4)) != hipSuccess) return fail(err, "hipMalloc(image)");
  if ((err = hipMemcpy(c.d_image, img.data(), img.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
    return fail(err, "hipMemcpy(image)");
  const std::vector<uint32_t> st = build_search_tables();
  if ((err = hipMalloc(reinterpret_cast<void**>(&c.d_search), st.size() * 4)) != hipSuccess)
    return fail(err, "hipMalloc(search tables)");
  if ((err = hipMemcpy(c.d_search, st.data(), st.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
    return fail(err, "hipMemcpy(search tables)");
  const std::vector<uint32_t> sg = build_stage_image();
  if ((err = hipMalloc(reinterpret_cast<void**>(&c.d_stage), sg.size() * 4)) != hipSuccess)
    return fail(err, "hipMalloc(stage image)");
  if ((err = hipMemcpy(c.d_stage, sg.data(), sg.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
    return fail(err, "hipMemcpy(stage image)");
  const std::vector<uint32_t> rx = build_rx_image();
  if ((err = hipMalloc(reinterpret_cast<void**>(&c.d_rx), rx.size() * 4)) != hipSuccess)
    return fail(err, "hipMalloc(rx image)");
  if ((err = hipMemcpy(c.d_rx, rx.data(), rx.size() * 4, hipMemcpyHostToDevice)) != hipSuccess)
    return fail(err, "hipMemcpy(rx image)");
  return LNX_OK;
}

int get_ctx(DeviceCtx** out) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return hip_fail(e, "hipGetDevice");
  if (dev < 0 || dev >= kMaxDevices) return LNX_ENODEV;
  DeviceCtx& c = g_ctx[dev];
  if (!c.ready.load(std::memory_order_acquire)) {
    std::lock_guard<std::mutex> lk(c.mu);
    if (!c.ready.load(std::memory_order_relaxed)) {
      const int st = init_ctx(c, dev);
      if (st != LNX_OK) return st;
      c.ready.store(true, std::memory_order_release);
    }
  }
  *out = &c;
  return LNX_OK;
}

// Slots of the giant slices: acc[kGiantSlots] then cnt[kGiantSlots]
// (stage_kernel.hip: at most 2^20 pieces plus one per slice), then the flag
// word through which the rows launch tells the staged launch it has work
// (the call's epoch: nonzero, new every call on the stream, so the word needs
// no reset)
constexpr size_t kGiantSlots = (1u << 20) + 4096u;
constexpr size_t kStageFlag = 2 * kGiantSlots;
constexpr size_t kIngressGate = kStageFlag + 1;  // lnx_ingress_verify_batch's second launch (the same epoch rule)
constexpr size_t kTxChecksumGate = kStageFlag + 2;  // lnx_tx_checksum_batch's
constexpr size_t kScratchWords = kStageFlag + 16;
// the mean frame length from which the ingress rows beat the receive check
// without its CRC (tools/prof/ingress_vs_rv.py)
constexpr uint64_t kIngressShortMean = 1280;
// ... and the generate rows against tx_finish's checksum step (sampled mean)
constexpr uint64_t kTxChecksumShortMean = 896;

// The calling device's giant-slice scratch for `stream`, zeroed on that
// stream when made (stream order puts the zeroing before the first launch).
constexpr size_t kGiantStreams = 32;
int giant_scratch(DeviceCtx* c, hipStream_t stream, uint32_t** out, uint32_t* epoch) {
  std::lock_guard<std::mutex> lk(c->giant_mu);
  const std::thread::id tid = stream == hipStreamPerThread ? std::this_thread::get_id() : std::thread::id();
  ++c->giant_clock;
  for (auto& g : c->giant)
    if (g.stream == stream && g.thread == tid) {
      g.used = c->giant_clock;
      g.epoch = g.epoch + 1u == 0u ? 1u : g.epoch + 1u;
      *out = g.p;
      *epoch = g.epoch;
      return LNX_OK;
    }
  hipError_t e;
  if (c->giant.size() >= kGiantStreams) {
    // its stream may still run a launch on it (or be gone): wait for the device
    auto lru = std::min_element(c->giant.begin(), c->giant.end(),
                                [](const DeviceCtx::GiantScratch& a, const DeviceCtx::GiantScratch& b) {
                                  return a.used < b.used;
                                });
    if ((e = hipDeviceSynchronize()) != hipSuccess) return hip_fail(e, "hipDeviceSynchronize(giant-slice scratch)");
    (void)hipFree(lru->p);
    c->giant.erase(lru);
  }
  uint32_t* p = nullptr;
  e = hipMalloc(reinterpret_cast<void**>(&p), kScratchWords * sizeof(uint32_t));
  if (e != hipSuccess) return hip_fail(e, "hipMalloc(giant-slice scratch)");
  if ((e = hipMemsetAsync(p, 0, kScratchWords * sizeof(uint32_t), stream)) != hipSuccess) {
    (void)hipFree(p);
    return hip_fail(e, "hipMemsetAsync(giant-slice scratch)");
  }
  c->giant.push_back({stream, tid, p, c->giant_clock, 1u});
  *out = p;
  *epoch = 1u;
  return LNX_OK;
}

}  // namespace

// CRC-32 / FCS verify of an offsets batch: the rows kernel,
// then the staged kernel, over the same slices; each workgroup folds its slice
// only if dispatch.hpp's slice_kind() gives it to its kernel, and the staged
// launch folds the giant slices.  policy kPolicyShort (LNX_BATCH_SHORT_FRAMES)
// gives every slice that fits to the staged kernel, so the rows launch is
// skipped.  Also the receive ring's entry (rx_ring.hip).
int crc_offsets(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, void* d_out, bool verify, uint32_t policy,
                hipStream_t stream) {
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  uint32_t* scratch = nullptr;
  uint32_t epoch = 0;
  if ((st = giant_scratch(c, stream, &scratch, &epoch)) != LNX_OK) return st;
  hipError_t e = hipSuccess;
  // auto: the rows launch stores the epoch in the flag word when a slice is
  // not its own, and the staged launch behind it exits at once otherwise
  uint32_t* flag = policy == kPolicyAuto ? scratch + kStageFlag : nullptr;
  if (policy == kPolicyAuto)
    e = launch_crc32_frames(d_bytes, d_off, n, d_out, verify, c->d_image, c->num_cus, stream, policy, flag, epoch);
  if (e != hipSuccess) return hip_fail(e, "crc32_rows_kernel launch");
  e = launch_crc32_stage(d_bytes, d_off, n, d_out, verify, policy, c->d_stage, scratch, c->num_cus, stream, flag,
                         epoch);
  if (e != hipSuccess) return hip_fail(e, "crc32_stage_kernel launch");
  return LNX_OK;
}

namespace {
int crc_common(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, void* d_out, bool verify,
               uint32_t flags, void* stream) {
  if (flags & ~LNX_BATCH_SHORT_FRAMES) return LNX_EINVAL;
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_off || !d_out) return LNX_EINVAL;
  return crc_offsets(d_bytes, d_off, n, d_out, verify, (flags & LNX_BATCH_SHORT_FRAMES) ? kPolicyShort : kPolicyAuto,
                     static_cast<hipStream_t>(stream));
}
}  // namespace

// For the other translation units (rx_ring.hip): the current device's LDS
// image and CU count, and the thread's lnx_last_error.
int device_resources(const void** image, int* num_cus, const void** stage_image, const void** rx_image) {
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  *image = c->d_image;
  *num_cus = c->num_cus;
  if (stage_image) *stage_image = c->d_stage;
  if (rx_image) *rx_image = c->d_rx;
  return LNX_OK;
}
int hip_error(hipError_t e, const char* what) { return hip_fail(e, what); }

}  // namespace lnx

using namespace lnx;

extern "C" {

int lnx_crc32_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t* d_crc,
                    void* stream) {
  return crc_common(d_bytes, d_off, n, d_crc, false, 0, stream);
}

int lnx_fcs_verify_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint8_t* d_ok,
                         void* stream) {
  return crc_common(d_bytes, d_off, n, d_ok, true, 0, stream);
}

int lnx_crc32_batch_ex(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t* d_crc, uint32_t flags,
                       void* stream) {
  return crc_common(d_bytes, d_off, n, d_crc, false, flags, stream);
}

int lnx_fcs_verify_batch_ex(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint8_t* d_ok,
                            uint32_t flags, void* stream) {
  return crc_common(d_bytes, d_off, n, d_ok, true, flags, stream);
}

int lnx_sum16_batch(const uint8_t* d_bytes, const uint64_t* d_off, const uint32_t* d_len,
                    const uint32_t* d_seed, uint64_t n, uint16_t* d_out, void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_off || !d_len || !d_out) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  hipError_t e = launch_sum16_segments(d_bytes, d_off, d_len, d_seed, n, d_out, c->num_cus,
                                       static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "sum16_segments_kernel launch");
  return LNX_OK;
}

#ifdef LNX_RESEARCH
// The calling device's scratch for `stream`, at least `bytes` long.  The
// caller holds c->scratch_mu until its launches on the scratch are enqueued,
// so a concurrent grow (which syncs the stream, then frees) cannot free it
// under a launch that is not yet in the stream.
static int stream_scratch(DeviceCtx* c, hipStream_t stream, size_t bytes, void** out) {
  DeviceCtx::Scratch* sc = nullptr;
  for (auto& x : c->scratch)
    if (x.stream == stream) sc = &x;
  if (!sc) {
    c->scratch.push_back({stream, nullptr, 0});
    sc = &c->scratch.back();
  }
  if (sc->cap < bytes) {
    hipError_t e;
    if (sc->p) {  // the stream's earlier launches may still read the old buffer
      if ((e = hipStreamSynchronize(stream)) != hipSuccess) return hip_fail(e, "hipStreamSynchronize(scratch)");
      (void)hipFree(sc->p);
      sc->p = nullptr, sc->cap = 0;
    }
    const size_t want = bytes < (1u << 20) ? (1u << 20) : bytes + bytes / 4;
    if ((e = hipMalloc(&sc->p, want)) != hipSuccess) return hip_fail(e, "hipMalloc(scratch)");
    sc->cap = want;
  }
  *out = sc->p;
  return LNX_OK;
}
#endif  // LNX_RESEARCH

int lnx_crc32_segments(const uint8_t* d_bytes, const uint64_t* d_start, const uint32_t* d_len, uint64_t n,
                       uint32_t* d_crc, void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_start || !d_len || !d_crc) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  hipError_t e = launch_crc32_segments(d_bytes, d_start, d_len, n, d_crc, c->d_image, c->num_cus,
                                       static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "crc32_rows_kernel (segments) launch");
  return LNX_OK;
}

int lnx_fcs_append_batch(uint8_t* d_bytes, const uint64_t* d_start, uint32_t* d_len, uint64_t n, uint32_t capacity,
                         uint8_t* d_status, void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_start || !d_len || !d_status) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  // one launch of the CRC kernel in its append mode: no scratch, no allocation
  // (a compact CRC array plus a scatter launch measured the same, 0.331 ms:
  // lnx__fcs_append_variant 200)
  const hipError_t e = launch_fcs_append(d_bytes, d_start, d_len, n, capacity, d_status, c->d_image, c->num_cus,
                                         static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "crc32_rows_kernel (append) launch");
  return LNX_OK;
}

#ifdef LNX_RESEARCH
// TX append in two launches (A/B, lnx__fcs_append_variant 200): the segment-mode
// CRC kernel into a compact per-stream scratch, then fcs_scatter_kernel.
static int fcs_append_two_launch(DeviceCtx* c, uint8_t* d_bytes, const uint64_t* d_start, uint32_t* d_len, uint64_t n,
                                 uint32_t capacity, uint8_t* d_status, hipStream_t s) {
  std::lock_guard<std::mutex> lk(c->scratch_mu);  // held until both launches are enqueued
  uint32_t* scr = nullptr;
  int st = stream_scratch(c, s, n * sizeof(uint32_t), reinterpret_cast<void**>(&scr));
  if (st != LNX_OK) return st;
  hipError_t e = launch_crc32_segments(d_bytes, d_start, d_len, n, scr, c->d_image, c->num_cus, s);
  if (e != hipSuccess) return hip_fail(e, "crc32_rows_kernel (append: segments) launch");
  e = launch_fcs_scatter(d_bytes, d_start, d_len, scr, n, capacity, d_status, c->num_cus, s);
  if (e != hipSuccess) return hip_fail(e, "fcs_scatter_kernel launch");
  return LNX_OK;
}
#endif  // LNX_RESEARCH

int lnx_tx_checksum_batch(uint8_t* d_bytes, const uint64_t* d_start, const uint32_t* d_len, uint64_t n,
                          uint8_t* d_status, void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_start || !d_len || !d_status) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  // two launches, one of which works (as lnx_ingress_verify_batch): the
  // generate rows, or for a batch whose sampled mean frame is under
  // kTxChecksumShortMean bytes tx_finish with the checksum step only
  const hipStream_t hs = static_cast<hipStream_t>(stream);
  uint32_t* scratch = nullptr;
  uint32_t epoch = 0;
  if ((st = giant_scratch(c, hs, &scratch, &epoch)) != LNX_OK) return st;
  uint32_t* gate = scratch + kTxChecksumGate;
  hipError_t e = launch_tx_checksum(d_bytes, d_start, d_len, n, d_status, c->num_cus, hs, gate, epoch,
                                    kTxChecksumShortMean);
  if (e != hipSuccess) return hip_fail(e, "tx checksum (ingress_verify_kernel<GEN>) launch");
  e = launch_tx_finish(d_bytes, d_start, const_cast<uint32_t*>(d_len), n, 0, LNX_TX_CHECKSUM, d_status, d_status,
                       c->d_rx, c->num_cus, hs, false, gate, epoch);
  if (e != hipSuccess) return hip_fail(e, "tx_finish_kernel launch");
  return LNX_OK;
}

int lnx_tx_finish_batch(uint8_t* d_bytes, const uint64_t* d_start, uint32_t* d_len, uint64_t n, uint32_t capacity,
                        uint32_t flags, uint8_t* d_status, void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_start || !d_len || !d_status) return LNX_EINVAL;
  if ((flags & ~(uint32_t)(LNX_TX_CHECKSUM | LNX_TX_FCS)) != 0) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  const hipError_t e = launch_tx_finish(d_bytes, d_start, d_len, n, capacity, flags, d_status, d_status, c->d_rx,
                                        c->num_cus, static_cast<hipStream_t>(stream), false);
  if (e != hipSuccess) return hip_fail(e, "tx_finish_kernel launch");
  return LNX_OK;
}

int lnx_crc32_search_batch(const uint8_t* d_bytes, const uint64_t* d_off, const int64_t* d_min_off, uint64_t n,
                           int64_t* d_result, void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_off || !d_result) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  hipError_t e = launch_crc32_search(d_bytes, d_off, d_min_off, n, c->d_search, d_result, c->num_cus,
                                     static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "crc32_search_kernel launch");
  return LNX_OK;
}

int lnx_ingress_verify_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t flags,
                             uint8_t* d_verdict, void* stream) {
  return lnx_ingress_verify_batch_filtered(d_bytes, d_off, n, flags, nullptr, d_verdict, stream);
}

int lnx_ingress_verify_batch_filtered(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t flags,
                                      const lnx_rx_filter* filter, uint8_t* d_verdict, void* stream) {
  RxFilter filt;
  if (!rx_filter_of(filter, &filt)) return LNX_EINVAL;
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_off || !d_verdict) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  // two launches, one of which works (the mean frame length is device-resident):
  // the ingress rows for a batch whose mean frame is >= kIngressShortMean
  // bytes, else the receive check without its CRC (rx_verify_kernel: the same
  // verdicts, no ok output), gated by a word of the stream's scratch
  const hipStream_t hs = static_cast<hipStream_t>(stream);
  uint32_t* scratch = nullptr;
  uint32_t epoch = 0;
  if ((st = giant_scratch(c, hs, &scratch, &epoch)) != LNX_OK) return st;
  uint32_t* gate = scratch + kIngressGate;
  const uint32_t vf = flags & (LNX_VERIFY_EVIL_BIT | LNX_VERIFY_ICMP);
  hipError_t e = launch_ingress_verify(d_bytes, d_off, n, vf, d_verdict, c->num_cus, hs, nullptr, 0, &filt, gate, epoch,
                                       kIngressShortMean);
  if (e != hipSuccess) return hip_fail(e, "ingress_verify_kernel launch");
  e = launch_rx_verify(d_bytes, d_off, n, vf, false, nullptr, d_verdict, nullptr, &filt, c->d_rx, c->num_cus, hs, false,
                       gate, epoch);
  if (e != hipSuccess) return hip_fail(e, "rx_verify_kernel launch");
  return LNX_OK;
}

int lnx_rx_verify_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t flags,
                        const lnx_rx_filter* filter, uint8_t* d_fcs_ok, uint8_t* d_verdict, void* stream) {
  RxFilter filt;
  if (!rx_filter_of(filter, &filt)) return LNX_EINVAL;
  if (flags & ~(uint32_t)(LNX_VERIFY_EVIL_BIT | LNX_VERIFY_ICMP | LNX_RX_NO_FCS)) return LNX_EINVAL;
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_off || !d_fcs_ok || !d_verdict) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  const hipError_t e = launch_rx_verify(d_bytes, d_off, n, flags & (LNX_VERIFY_EVIL_BIT | LNX_VERIFY_ICMP),
                                        !(flags & LNX_RX_NO_FCS), d_fcs_ok, d_verdict, nullptr, &filt, c->d_rx,
                                        c->num_cus, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "rx_verify_kernel launch");
  return LNX_OK;
}

int lnx_pcap_verify_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint8_t* d_status,
                          void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_off || !d_status) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  const hipError_t e = launch_pcap_verify(d_bytes, d_off, n, d_status, c->num_cus, static_cast<hipStream_t>(stream));
  if (e != hipSuccess) return hip_fail(e, "pcap_verify_kernel launch");
  return LNX_OK;
}

int lnx_crc32_batch_host(const uint8_t* h_bytes, uint64_t nbytes, const uint64_t* h_off, uint64_t n,
                         uint32_t* h_crc, int device) {
  if (n == 0) return LNX_OK;
  if (!h_bytes || !h_off || !h_crc) return LNX_EINVAL;
  for (uint64_t i = 0; i <= n; ++i)
    if (h_off[i] > nbytes) return LNX_EINVAL;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_fail(e, "hipSetDevice");
  uint8_t* d_bytes = nullptr;
  uint64_t* d_off = nullptr;
  uint32_t* d_crc = nullptr;
  int rc = LNX_OK;
  hipStream_t s = nullptr;
  if ((e = hipStreamCreateWithFlags(&s, hipStreamNonBlocking)) != hipSuccess) return hip_fail(e, "hipStreamCreate");
  if ((e = hipMallocAsync(reinterpret_cast<void**>(&d_bytes), nbytes ? nbytes : 4, s)) != hipSuccess ||
      (e = hipMallocAsync(reinterpret_cast<void**>(&d_off), (n + 1) * 8, s)) != hipSuccess ||
      (e = hipMallocAsync(reinterpret_cast<void**>(&d_crc), n * 4, s)) != hipSuccess) {
    rc = hip_fail(e, "hipMallocAsync");
  }
  if (rc == LNX_OK) {
    if ((e = hipMemcpyAsync(d_bytes, h_bytes, nbytes, hipMemcpyHostToDevice, s)) != hipSuccess ||
        (e = hipMemcpyAsync(d_off, h_off, (n + 1) * 8, hipMemcpyHostToDevice, s)) != hipSuccess)
      rc = hip_fail(e, "hipMemcpyAsync H2D");
  }
  // (the plain entry: each slice's kernel is picked on the device)
  if (rc == LNX_OK) rc = lnx_crc32_batch(d_bytes, d_off, n, d_crc, s);
  if (rc == LNX_OK && (e = hipMemcpyAsync(h_crc, d_crc, n * 4, hipMemcpyDeviceToHost, s)) != hipSuccess)
    rc = hip_fail(e, "hipMemcpyAsync D2H");
  if (d_bytes) (void)hipFreeAsync(d_bytes, s);
  if (d_off) (void)hipFreeAsync(d_off, s);
  if (d_crc) (void)hipFreeAsync(d_crc, s);
  if ((e = hipStreamSynchronize(s)) != hipSuccess && rc == LNX_OK) rc = hip_fail(e, "hipStreamSynchronize");
  (void)hipStreamDestroy(s);
  return rc;
}

int lnx_crc32_batch_multi(int ngpu, const int* devices, const uint8_t* const* d_bytes_per_gpu,
                          const uint64_t* const* d_off_per_gpu, const uint64_t* n_per_gpu,
                          uint32_t* const* d_crc_per_gpu) {
  if (ngpu <= 0 || !devices || !d_bytes_per_gpu || !d_off_per_gpu || !n_per_gpu || !d_crc_per_gpu)
    return LNX_EINVAL;
  std::vector<int> rcs(ngpu, LNX_OK);
  std::vector<std::string> errs(ngpu);
  std::vector<std::thread> th;
  for (int g = 0; g < ngpu; ++g) {
    th.emplace_back([&, g] {
      hipError_t e = hipSetDevice(devices[g]);
      if (e != hipSuccess) { rcs[g] = hip_fail(e, "hipSetDevice"); errs[g] = g_last_error; return; }
      int rc = lnx_crc32_batch(d_bytes_per_gpu[g], d_off_per_gpu[g], n_per_gpu[g], d_crc_per_gpu[g], nullptr);
      if (rc == LNX_OK && (e = hipDeviceSynchronize()) != hipSuccess) rc = hip_fail(e, "hipDeviceSynchronize");
      rcs[g] = rc;
      if (rc != LNX_OK) errs[g] = g_last_error;
    });
  }
  for (auto& t : th) t.join();
  for (int g = 0; g < ngpu; ++g)
    if (rcs[g] != LNX_OK) { g_last_error = errs[g]; return rcs[g]; }
  return LNX_OK;
}

#ifdef LNX_RESEARCH
// Profiling hooks of the research library (liblneto_amd_research.so, not in
// include/lneto_amd.h): kernel variants of DESIGN.md §4.
int lnx__crc32_variant(int var, const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t* d_crc,
                       void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_off || !d_crc) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  // 300 / 301: the staged lane streams (stage_kernel.hip), CRC / FCS verify,
  // slicing-by-2 fold; 302 / 303: the same with the 16-column Z_4 fold;
  // 304-307: 300-303 with 10 waves per workgroup instead of 8 (retired);
  // 308 / 309: 302 / 303 with 766-frame blocks; 310 / 311: the slicing-by-8 fold;
  // 312 / 313: the slicing-by-8 fold with the boundary correction deferred;
  // 314 / 315: the slicing-by-8 fold with the boundary word patched per half;
  // 316 / 317: 314 / 315 with each half folded as two chains of four units;
  // 318 / 319 and 320 / 321: 314 / 315 with 190- and 254-frame blocks;
  // 322 / 323: 314 / 315 with the next block's offsets loaded ahead;
  // 324 / 325: 314 / 315 with 510-frame blocks; 326 / 327: 314 / 315 with 6 waves;
  // 328 / 330: timing only (wrong results): 314 without the transpose writes,
  // 314 with a two-op stand-in for the lookups; 332: 314 without the ending
  // frames' capture and Z_c; 334: 314 without the carries; 340: the ring's
  // loads alone; 342: loads + the LDS transpose (round 5)
  // (all in stage_research.hip, the round-4 kernel; the product staged kernel
  // with its round-5 dispatch is lnx_crc32_batch_ex(LNX_BATCH_SHORT_FRAMES))
  hipError_t e = (var >= 300 && var <= 327) || var == 328 || var == 330 || var == 332 || var == 334 || var == 340 ||
                         var == 342
                     ? rs::launch_crc32_stage_research(d_bytes, d_off, n, d_crc, var & 1,
                                          var == 342 ? 22 : var == 340 ? 21 : var == 334 ? 20 : var == 332 ? 19 : var == 330 ? 18 : var == 328 ? 17 : var >= 326 ? 16 : var >= 324 ? 15 : var >= 322 ? 14 : var >= 320 ? 13 : var >= 318 ? 12 : var >= 316 ? 11 : var >= 314 ? 10 : var >= 312 ? 9 : var >= 310 ? 8 : (var & 2) || var >= 308 ? 4 : 2,
                                          var >= 304 && var < 308 ? 10 : 8, c->d_stage, c->num_cus,
                                          static_cast<hipStream_t>(stream), var == 308 || var == 309)
                     : launch_crc32_variant(var, d_bytes, d_off, n, d_crc, c->d_image, c->num_cus,
                                            static_cast<hipStream_t>(stream), nullptr);
  if (e != hipSuccess) return hip_fail(e, "crc32 variant launch");
  return LNX_OK;
}

// Profiling hook: TX FCS append variants (0 = the product, results held and
// flushed; 4 = FCS, length and status stored as each frame finishes).
int lnx__fcs_append_variant(int var, uint8_t* d_bytes, const uint64_t* d_start, uint32_t* d_len, uint64_t n,
                            uint32_t capacity, uint8_t* d_status, void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_start || !d_len || !d_status) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  if (var == 200)  // two launches: CRCs into a compact scratch, then the scatter kernel
    return fcs_append_two_launch(c, d_bytes, d_start, d_len, n, capacity, d_status, static_cast<hipStream_t>(stream));
  // 100 (= 0): the one-launch append mode, the product; 4 / 7: its A/B forms
  // (store at once / with the 64-byte sector)
  const hipError_t e = launch_fcs_append(d_bytes, d_start, d_len, n, capacity, d_status, c->d_image, c->num_cus,
                                         static_cast<hipStream_t>(stream), var == 100 ? 0 : var);
  if (e != hipSuccess) return hip_fail(e, "fcs append variant launch");
  return LNX_OK;
}

// Profiling hook: sum16 kernel variants (0 = line rows, the product; 1 = the
// r1c half-line rows).
int lnx__sum16_variant(int var, const uint8_t* d_bytes, const uint64_t* d_off, const uint32_t* d_len,
                       const uint32_t* d_seed, uint64_t n, uint16_t* d_out, void* stream) {
  if (n == 0) return LNX_OK;
  if (!d_bytes || !d_off || !d_len || !d_out) return LNX_EINVAL;
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  hipError_t e = launch_sum16_segments(d_bytes, d_off, d_len, d_seed, n, d_out, c->num_cus,
                                       static_cast<hipStream_t>(stream), var);
  if (e != hipSuccess) return hip_fail(e, "sum16 variant launch");
  return LNX_OK;
}

// Profiling hook: the variant with a per-wave timeline (3 x uint64 per wave:
// entry, image copied, exit; 100 MHz clock).  Returns the wave count when
// d_timeline is NULL.
int64_t lnx__crc32_timeline(int var, const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t* d_crc,
                            uint64_t* d_timeline, void* stream) {
  DeviceCtx* c = nullptr;
  int st = get_ctx(&c);
  if (st != LNX_OK) return st;
  if (!d_timeline) return (int64_t)crc32_launch_waves(n, c->num_cus);
  if (n == 0 || !d_bytes || !d_off || !d_crc) return LNX_EINVAL;
  hipError_t e = launch_crc32_variant(var, d_bytes, d_off, n, d_crc, c->d_image, c->num_cus,
                                      static_cast<hipStream_t>(stream), d_timeline);
  if (e != hipSuccess) return hip_fail(e, "crc32 timeline launch");
  return LNX_OK;
}
#endif  // LNX_RESEARCH

int lnx_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char* lnx_last_error(void) { return g_last_error.c_str(); }

const char* lnx_version(void) {
  return "lneto_amd 0.12 gfx950: crc32 rows (32-lane whole-line rows from 4096 B mean: 24-line items; one-word "
         "16-lane rows 1600-4096 B: 1 slot x 24 steps, 4-frame chunks; lean two-word line rows 640-1600 B, offsets "
         "and segment mode: one 13-line frame per row per slot; whole-line rows load a frame's first and last lines "
         "at the default cache policy, the rest nt; 4-lane rows: 2 slots x 16 steps, 32-frame chunks, held results; "
         "narrow rows load only the 4-step runs an item has; TX FCS append in the same launch: pad, FCS, length, "
         "status; segment slices out of address order folded frame by frame) + sum16 16-lane line rows + ingress "
         "verdicts (qword rows, end mask on the last qword, ICMP clients' checks) and TX checksum generate (the same "
         "rows, GEN) + rx ring (ingress and egress packets) + CRC32Search (eight captures per wave, 192-byte lane "
         "segments as four 48-byte chains joined by lane-private Z_48 nibble tables, 3-level scan, Z_4 in the "
         "lane-private U layout, pass B by word checks, group-descriptor loads) + staged lane streams for "
         "short-frame batches (slicing-by-8 fold, LDS transposed whole-line loads; out-of-order blocks by lane and "
         "by whole waves) and slice dispatch on the device (staged launch gated by the rows launch's flag word; "
         "giant slices by span, mean or 8x skew, out-of-order giant slices frame by frame) + rx_verify (FCS and "
         "verdicts in one read: 16-lane rows, 56-frame groups, the next pass loaded ahead, units no frame reaches "
         "skipped) + tx_finish (checksums, padding and FCS in one read, CRC corrected by linearity; 16 waves, "
         "48-frame groups) + zero copy through the ring's pinned slots";
}

}  // extern "C"
