// rx_ring.hip — pinned receive ring and the batched ingress pipeline.
//
// Reference: netdev.Stack.IngressPackets(bufs [][]byte, offset int) error
// (x/netdev/interface.go:82-89), implemented by xnet.Netstack
// (x/xnet/netstack.go:103-111) as one StackEthernet.Demux per buffer
// (internet/stack-ethernet.go:139-165) with buf[offset:] as the frame.  The
// buffers come from netdev's bufferSelect slot pool (x/netdev/buffer.go:25-37:
// fixed slots of a fixed capacity, a length per slot).  lneto never checks the
// FCS (the PHY is trusted, x/netdev/interface.go:34-40); here the ring checks
// it before the stack sees the frame, and computes the receive path's
// checksum-stage verdict of the stripped frame in the same pass.
//
// The ring owns `nslots` slots of `slot_cap` bytes in pinned host memory
// (hipHostMalloc) plus a pinned length per slot, so a producer (tap / NIC
// queue) writes frames where the GPU can DMA them.  lnx_rx_ring_ingress runs a
// slot range through `depth` stages, each on its own HIP stream with its own
// device buffers; batch k uses stage k % depth:
//     H2D  slots [b0, b0 + nb) (one contiguous copy) and their lengths
//     ring_segments_kernel   start = i*cap + offset, len = min(len, cap) - offset
//     crc32_rows_kernel      segment mode, FCS residue verify  -> ok[i]
//     ingress_verify_kernel  segment mode, FCS stripped       -> verdict[i]
//     D2H  ok / verdict into pinned result arrays
// so the copy of batch k+1 overlaps the kernels of batch k: the pipeline runs
// at the PCIe rate, the kernels are ~100x faster than the link.
//
// Zero copy (round 5, the default): the slots are mapped into the GPU's
// address space, so the receive kernel reads each frame straight from the
// pinned slot over PCIe (only the frame's bytes cross the link, whatever the
// slot fill) and no host thread copies a frame.  A batch then costs the H2D of
// its lengths (4 B per frame), ring_segments_kernel, rx_verify_kernel and the
// D2H of 2 B of results per frame.  lnx_ingress_packets / lnx_egress_packets
// take the same path when the caller's buffers are the ring's slots (netdev's
// RunnerConfig.Buffers, x/netdev/runner.go:92-94, can be exactly those: see
// INTEGRATION.md); the transmit kernels then patch the frames in place in host
// memory.  Buffers elsewhere (pageable memory) are gathered back to back into
// pinned staging (n + 1 offsets, so PCIe carries the frame bytes plus 8 bytes
// per frame) and, for egress, scattered back.  lnx_rx_ring_set_zero_copy(0)
// selects the copying forms for every batch (the round-4 path: whole slots when
// they are at least 90 % full, else packed).
//
// Stack configuration (lnx_rx_ring_set_filter) and FCS-less devices
// (LNX_RX_NO_FCS) follow the reference's receive path exactly
// (ingress_kernel.hip, rx_filter.hpp).
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>
#include "../../include/lneto_amd.h"
#include "rx_filter.hpp"

namespace lnx {

int device_resources(const void** image, int* num_cus, const void** stage_image, const void** rx_image);
hipError_t launch_rx_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t flags, bool fcs,
                            uint8_t* ok, uint8_t* verdict, const uint32_t* seg_len, const RxFilter* filter,
                            const uint32_t* image, int num_cus, hipStream_t stream, bool host = false,
                            const uint32_t* gate = nullptr, uint32_t epoch = 0);
int hip_error(hipError_t e, const char* what);
// host_path.cpp: the per-frame host forms (batches below the ring's host threshold)
uint8_t host_verdict(const uint8_t* fr, size_t L, uint32_t flags, const RxFilter& f);
uint8_t host_tx_checksum(uint8_t* f, size_t L);
uint8_t host_fcs_append(uint8_t* f, uint32_t* len, uint32_t capacity);
uint8_t host_fcs_ok(const uint8_t* f, size_t L);
hipError_t launch_fcs_verify_segments(const uint8_t* bytes, const uint64_t* start, const uint32_t* len, uint64_t n,
                                      uint8_t* ok, const void* images, int num_cus, hipStream_t stream);
hipError_t launch_ingress_verify(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t flags,
                                 uint8_t* verdict, int num_cus, hipStream_t stream, const uint32_t* seg_len,
                                 uint32_t trim, const RxFilter* filter, uint32_t* gate = nullptr, uint32_t epoch = 0,
                                 uint64_t short_mean = 0);
hipError_t launch_tx_checksum(uint8_t* bytes, const uint64_t* start, const uint32_t* len, uint64_t n,
                              uint8_t* status, int num_cus, hipStream_t stream, uint32_t* gate = nullptr,
                              uint32_t epoch = 0, uint64_t short_mean = 0);
hipError_t launch_fcs_append(uint8_t* bytes, const uint64_t* start, uint32_t* len, uint64_t n, uint32_t capacity,
                             uint8_t* status, const void* images, int num_cus, hipStream_t stream, int var = 0);
hipError_t launch_tx_finish(uint8_t* bytes, const uint64_t* start, uint32_t* len, uint64_t n, uint32_t capacity,
                            uint32_t flags, uint8_t* st_ck, uint8_t* st_ap, const uint32_t* image, int num_cus,
                            hipStream_t stream, bool host, const uint32_t* gate = nullptr, uint32_t epoch = 0);

// Slot i of the batch: frame = slot[offset : min(len, cap)].
__global__ void __launch_bounds__(256)
ring_segments_kernel(uint64_t* __restrict__ start, uint32_t* __restrict__ len, uint32_t n, uint32_t cap,
                     uint32_t offset) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const uint32_t l = len[i] < cap ? len[i] : cap;
    start[i] = (uint64_t)i * cap + offset;
    len[i] = l > offset ? l - offset : 0u;
  }
}

}  // namespace lnx

using namespace lnx;

struct lnx_rx_ring {
  int device = 0;
  uint32_t nslots = 0, cap = 0, batch = 0, depth = 0;
  uint8_t* h_slots = nullptr;  // the producer's slots (lnx_rx_ring_slots)
  uint8_t* d_slots = nullptr;  // the same memory as the GPU addresses it (hipHostGetDevicePointer)
  bool zero_copy = true;       // lnx_rx_ring_set_zero_copy
  uint32_t* h_len = nullptr;
  uint8_t* h_ok = nullptr;     // per slot: lnx_rx_ring_ingress results
  uint8_t* h_verdict = nullptr;
  struct Stage {
    hipStream_t s = nullptr;
    uint8_t* d_bytes = nullptr;
    uint64_t* d_start = nullptr;  // slot starts, or the packed batch's offsets (batch + 1)
    uint32_t* d_len = nullptr;
    uint8_t* d_ok = nullptr;
    uint8_t* d_verdict = nullptr;
    // pinned staging of the packed paths: frame bytes back to back, their
    // offsets / starts, lengths and results (batch entries each)
    uint8_t* h_pack = nullptr;
    uint64_t* h_off = nullptr;
    uint32_t* h_len = nullptr;
    uint8_t* h_ok = nullptr;
    uint8_t* h_verdict = nullptr;
  };
  std::vector<Stage> st;
  RxFilter filt{};  // lnx_rx_ring_set_filter; on = 0: accept-all
  // batches of fewer frames run on the host (host_path.cpp), no launch
  // (lnx_rx_ring_set_host_threshold; the default is the measured crossover)
  uint32_t host_below = LNX_HOST_BATCH_DEFAULT;
  lnx_rx_ring_counters stats{};  // lnx_rx_ring_stats (RunnerStatistics-style, x/netdev/runner.go:107-140)
  const void* image = nullptr;
  const void* stage_image = nullptr;  // the staged lane streams' tables (unused since round 5)
  const void* rx_image = nullptr;     // rx_verify_kernel's tables
  int num_cus = 0;
  std::mutex mu;  // one call at a time (the stages are shared)
};

namespace {

using Stage = lnx_rx_ring::Stage;

void ring_free(lnx_rx_ring* r) {
  if (!r) return;
  (void)hipSetDevice(r->device);
  for (auto& s : r->st) {
    if (s.s) (void)hipStreamSynchronize(s.s);
    (void)hipFree(s.d_bytes);
    (void)hipFree(s.d_start);
    (void)hipFree(s.d_len);
    (void)hipFree(s.d_ok);
    (void)hipFree(s.d_verdict);
    (void)hipHostFree(s.h_pack);
    (void)hipHostFree(s.h_off);
    (void)hipHostFree(s.h_len);
    (void)hipHostFree(s.h_ok);
    (void)hipHostFree(s.h_verdict);
    if (s.s) (void)hipStreamDestroy(s.s);
  }
  (void)hipHostFree(r->h_slots);
  (void)hipHostFree(r->h_len);
  (void)hipHostFree(r->h_ok);
  (void)hipHostFree(r->h_verdict);
  delete r;
}

// Host copies of a batch, split over up to 16 threads when it is large.
template <typename F>
void parallel_for(uint32_t nb, F&& fn) {
  const unsigned hw = std::max(1u, std::min(16u, std::thread::hardware_concurrency()));
  const uint32_t nth = nb >= 4096 ? hw : 1;
  if (nth == 1) {
    fn(0u, nb);
    return;
  }
  std::vector<std::thread> th;
  for (uint32_t t = 0; t < nth; ++t)
    th.emplace_back(fn, (uint32_t)((uint64_t)nb * t / nth), (uint32_t)((uint64_t)nb * (t + 1) / nth));
  for (auto& t : th) t.join();
}

// Pack frame j = (ptr(j), len(j)), j < nb, back to back into s.h_pack with
// offsets s.h_off[0..nb]; returns the packed byte count.
template <typename Ptr, typename Len>
uint64_t pack_batch(Stage& s, uint32_t nb, Ptr ptr, Len len) {
  uint64_t o = 0;
  for (uint32_t j = 0; j < nb; ++j) {
    s.h_off[j] = o;
    o += len(j);
  }
  s.h_off[nb] = o;
  parallel_for(nb, [&](uint32_t a, uint32_t b) {
    for (uint32_t j = a; j < b; ++j) {
      const uint64_t l = s.h_off[j + 1] - s.h_off[j];
      if (l) std::memcpy(s.h_pack + s.h_off[j], ptr(j), l);
    }
  });
  return o;
}

// After a failed call: wait for whatever a part-way enqueue left on every
// stage's stream (async copies out of / into the staging), so the next call may
// repack the staging.  Errors here are the failed call's, already reported.
void quiesce(lnx_rx_ring* r) {
  for (auto& s : r->st)
    if (s.s) (void)hipStreamSynchronize(s.s);
}

// Where a batch's frames are for the device.
enum class RxSrc {
  kPacked,       // packed in s.h_pack, offsets s.h_off[0..nb] (copied up)
  kSlotsCopy,    // whole slots [b0, b0 + nb) at `offset`, copied up
  kSlotsDirect,  // slots [b0, b0 + nb) at `offset`, read in place (zero copy)
  kSegDirect,    // frame j at ring byte s.h_off[j], s.h_len[j] bytes, read in place
};

// Whether buffer b (frame b[offset : offset + need]) lies inside the ring's
// slot memory, and its byte position there.
bool in_ring(const lnx_rx_ring* r, const uint8_t* b, uint64_t offset, uint64_t need, uint64_t* pos) {
  const uintptr_t lo = reinterpret_cast<uintptr_t>(r->h_slots), x = reinterpret_cast<uintptr_t>(b);
  const uint64_t size = (uint64_t)r->nslots * r->cap;
  if (x < lo || x - lo > size || offset + need > size - (x - lo)) return false;
  *pos = (uint64_t)(x - lo) + offset;
  return true;
}

// Receive direction on stage s (asynchronous), results into ok_dst /
// verdict_dst (pinned, nb entries), frames as `src` says.  FCS verify unless
// LNX_RX_NO_FCS (then fcs_ok = 1 and the verdict covers the whole frame).
int enqueue_rx(lnx_rx_ring* r, Stage& s, uint32_t nb, RxSrc src, uint32_t b0, uint32_t offset, uint32_t flags,
               uint8_t* ok_dst, uint8_t* verdict_dst) {
  hipError_t e;
  const bool fcs = !(flags & LNX_RX_NO_FCS);
  const uint32_t vflags = flags & (LNX_VERIFY_EVIL_BIT | LNX_VERIFY_ICMP);
  const uint32_t* rx_image = static_cast<const uint32_t*>(r->rx_image);
  if (src == RxSrc::kSegDirect) {
    if ((e = hipMemcpyAsync(s.d_start, s.h_off, (size_t)nb * 8, hipMemcpyHostToDevice, s.s)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_len, s.h_len, (size_t)nb * 4, hipMemcpyHostToDevice, s.s)) != hipSuccess)
      return hip_error(e, "rx ring H2D (frame table)");
    if ((e = launch_rx_verify(r->d_slots, s.d_start, nb, vflags, fcs, s.d_ok, s.d_verdict, s.d_len, &r->filt,
                              rx_image, r->num_cus, s.s, true)) != hipSuccess)
      return hip_error(e, "rx ring rx_verify launch");
  } else if (src == RxSrc::kSlotsDirect) {
    if ((e = hipMemcpyAsync(s.d_len, r->h_len + b0, (size_t)nb * 4, hipMemcpyHostToDevice, s.s)) != hipSuccess)
      return hip_error(e, "rx ring H2D (lengths)");
    const uint32_t grid = std::min<uint32_t>((nb + 255) / 256, 1024);
    hipLaunchKernelGGL(ring_segments_kernel, dim3(grid), dim3(256), 0, s.s, s.d_start, s.d_len, nb, r->cap, offset);
    if ((e = hipGetLastError()) != hipSuccess) return hip_error(e, "ring_segments_kernel launch");
    if ((e = launch_rx_verify(r->d_slots + (size_t)b0 * r->cap, s.d_start, nb, vflags, fcs, s.d_ok, s.d_verdict,
                              s.d_len, &r->filt, rx_image, r->num_cus, s.s, true)) != hipSuccess)
      return hip_error(e, "rx ring rx_verify launch");
  } else if (src == RxSrc::kPacked) {
    const uint64_t total = s.h_off[nb];
    if ((total && (e = hipMemcpyAsync(s.d_bytes, s.h_pack, total, hipMemcpyHostToDevice, s.s)) != hipSuccess) ||
        (e = hipMemcpyAsync(s.d_start, s.h_off, (size_t)(nb + 1) * 8, hipMemcpyHostToDevice, s.s)) != hipSuccess)
      return hip_error(e, "rx ring H2D (packed)");
    // FCS and verdicts in one pass over each frame (rx_verify_kernel.hip)
    if ((e = launch_rx_verify(s.d_bytes, s.d_start, nb, vflags, fcs, s.d_ok, s.d_verdict, nullptr, &r->filt,
                              rx_image, r->num_cus, s.s)) != hipSuccess)
      return hip_error(e, "rx ring rx_verify launch");
  } else {
    const size_t cap = r->cap;
    if ((e = hipMemcpyAsync(s.d_bytes, r->h_slots + (size_t)b0 * cap, (size_t)nb * cap, hipMemcpyHostToDevice,
                            s.s)) != hipSuccess ||
        (e = hipMemcpyAsync(s.d_len, r->h_len + b0, (size_t)nb * 4, hipMemcpyHostToDevice, s.s)) != hipSuccess)
      return hip_error(e, "rx ring H2D");
    const uint32_t grid = std::min<uint32_t>((nb + 255) / 256, 1024);
    hipLaunchKernelGGL(ring_segments_kernel, dim3(grid), dim3(256), 0, s.s, s.d_start, s.d_len, nb, r->cap, offset);
    if ((e = hipGetLastError()) != hipSuccess) return hip_error(e, "ring_segments_kernel launch");
    if ((e = launch_rx_verify(s.d_bytes, s.d_start, nb, vflags, fcs, s.d_ok, s.d_verdict, s.d_len, &r->filt,
                              rx_image, r->num_cus, s.s)) != hipSuccess)
      return hip_error(e, "rx ring rx_verify launch");
  }
  if ((e = hipMemcpyAsync(ok_dst, s.d_ok, nb, hipMemcpyDeviceToHost, s.s)) != hipSuccess ||
      (e = hipMemcpyAsync(verdict_dst, s.d_verdict, nb, hipMemcpyDeviceToHost, s.s)) != hipSuccess)
    return hip_error(e, "rx ring D2H");
  r->stats.device_batches += 1;
  r->stats.device_frames += nb;
  return LNX_OK;
}

// Transmit direction on stage s (asynchronous): the nb frames at starts
// s.h_off[j] with lengths s.h_len[j] (each with room for its padding and FCS)
// get their checksums (LNX_TX_CHECKSUM) and padding + FCS (LNX_TX_FCS) on the
// device and come back with their new lengths; s.h_verdict = the checksum
// status, s.h_ok = the append status.  direct: the starts are ring bytes
// past `base` and the kernels patch the frames in place in the slots (zero
// copy); else they are packed in s.h_pack (total bytes) and copied both ways.
int enqueue_tx(lnx_rx_ring* r, Stage& s, uint32_t nb, uint64_t total, uint32_t capacity, uint32_t flags,
               bool direct = false, uint64_t base = 0) {
  hipError_t e;
  uint8_t* bytes = direct ? r->d_slots + base : s.d_bytes;
  if (direct) total = 0;
  if ((total && (e = hipMemcpyAsync(s.d_bytes, s.h_pack, total, hipMemcpyHostToDevice, s.s)) != hipSuccess) ||
      (e = hipMemcpyAsync(s.d_start, s.h_off, (size_t)nb * 8, hipMemcpyHostToDevice, s.s)) != hipSuccess ||
      (e = hipMemcpyAsync(s.d_len, s.h_len, (size_t)nb * 4, hipMemcpyHostToDevice, s.s)) != hipSuccess)
    return hip_error(e, "tx ring H2D");
  if (direct) {
    // frames in the pinned slots: one kernel reads each frame once over PCIe and
    // stores only the fields, the padding and the FCS (rx_verify_kernel.hip tx_finish)
    if ((e = launch_tx_finish(bytes, s.d_start, s.d_len, nb, capacity, flags, s.d_verdict, s.d_ok,
                              static_cast<const uint32_t*>(r->rx_image), r->num_cus, s.s, true)) != hipSuccess)
      return hip_error(e, "tx ring tx_finish launch");
  } else {
    if ((e = hipMemsetAsync(s.d_verdict, 0, nb, s.s)) != hipSuccess ||
        (e = hipMemsetAsync(s.d_ok, 0, nb, s.s)) != hipSuccess)
      return hip_error(e, "tx ring status reset");
    if ((flags & LNX_TX_CHECKSUM) &&
        (e = launch_tx_checksum(bytes, s.d_start, s.d_len, nb, s.d_verdict, r->num_cus, s.s)) != hipSuccess)
      return hip_error(e, "tx ring checksum launch");
    if ((flags & LNX_TX_FCS) &&
        (e = launch_fcs_append(bytes, s.d_start, s.d_len, nb, capacity, s.d_ok, r->image, r->num_cus, s.s)) !=
            hipSuccess)
      return hip_error(e, "tx ring FCS append launch");
  }
  if ((total && (e = hipMemcpyAsync(s.h_pack, s.d_bytes, total, hipMemcpyDeviceToHost, s.s)) != hipSuccess) ||
      (e = hipMemcpyAsync(s.h_len, s.d_len, (size_t)nb * 4, hipMemcpyDeviceToHost, s.s)) != hipSuccess ||
      (e = hipMemcpyAsync(s.h_ok, s.d_ok, nb, hipMemcpyDeviceToHost, s.s)) != hipSuccess ||
      (e = hipMemcpyAsync(s.h_verdict, s.d_verdict, nb, hipMemcpyDeviceToHost, s.s)) != hipSuccess)
    return hip_error(e, "tx ring D2H");
  r->stats.device_batches += 1;
  r->stats.device_frames += nb;
  return LNX_OK;
}

// The receive step of one frame on the host: frame = p[0 : len], FCS in its
// last 4 bytes unless LNX_RX_NO_FCS (the semantics of enqueue_rx).
void host_rx(const lnx_rx_ring* r, const uint8_t* p, uint32_t len, uint32_t flags, uint8_t* ok, uint8_t* verdict) {
  const bool fcs = !(flags & LNX_RX_NO_FCS);
  const uint32_t trim = fcs ? 4u : 0u;
  *ok = fcs ? host_fcs_ok(p, len) : 1u;
  *verdict = host_verdict(p, len > trim ? len - trim : 0u, flags & (LNX_VERIFY_EVIL_BIT | LNX_VERIFY_ICMP), r->filt);
}

}  // namespace

extern "C" {

int lnx_rx_ring_stats(lnx_rx_ring* r, lnx_rx_ring_counters* out) {
  if (!r || !out) return LNX_EINVAL;
  std::lock_guard<std::mutex> lk(r->mu);
  *out = r->stats;
  return LNX_OK;
}

int lnx_rx_ring_set_host_threshold(lnx_rx_ring* r, uint32_t frames) {
  if (!r) return LNX_EINVAL;
  std::lock_guard<std::mutex> lk(r->mu);
  r->host_below = frames;
  return LNX_OK;
}

int lnx_rx_ring_set_zero_copy(lnx_rx_ring* r, int on) {
  if (!r) return LNX_EINVAL;
  std::lock_guard<std::mutex> lk(r->mu);
  r->zero_copy = on != 0;
  return LNX_OK;
}

int lnx_rx_ring_create(int device, uint32_t nslots, uint32_t slot_cap, uint32_t batch_slots, uint32_t depth,
                       lnx_rx_ring** out) {
  if (!out) return LNX_EINVAL;
  *out = nullptr;
  if (nslots == 0 || slot_cap == 0 || slot_cap % 4 != 0 || depth == 0 || depth > 8) return LNX_EINVAL;
  if (batch_slots == 0 || batch_slots > nslots) batch_slots = nslots;
  if ((uint64_t)batch_slots * slot_cap >= (1ull << 31)) return LNX_EINVAL;  // one segment-mode slice per batch
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || device < 0 || device >= ndev) return LNX_ENODEV;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) return hip_error(e, "hipSetDevice");
  auto* r = new lnx_rx_ring;
  r->device = device, r->nslots = nslots, r->cap = slot_cap, r->batch = batch_slots, r->depth = depth;
  int rc = device_resources(&r->image, &r->num_cus, &r->stage_image, &r->rx_image);
  if (rc != LNX_OK) { ring_free(r); return rc; }
  const size_t slots_bytes = (size_t)nslots * slot_cap;
  if ((e = hipHostMalloc(reinterpret_cast<void**>(&r->h_slots), slots_bytes, hipHostMallocDefault)) != hipSuccess ||
      (e = hipHostMalloc(reinterpret_cast<void**>(&r->h_len), (size_t)nslots * 4, hipHostMallocDefault)) !=
          hipSuccess ||
      (e = hipHostMalloc(reinterpret_cast<void**>(&r->h_ok), nslots, hipHostMallocDefault)) != hipSuccess ||
      (e = hipHostMalloc(reinterpret_cast<void**>(&r->h_verdict), nslots, hipHostMallocDefault)) != hipSuccess) {
    rc = hip_error(e, "hipHostMalloc(rx ring)");
    ring_free(r);
    return rc;
  }
  std::memset(r->h_len, 0, (size_t)nslots * 4);
  if ((e = hipHostGetDevicePointer(reinterpret_cast<void**>(&r->d_slots), r->h_slots, 0)) != hipSuccess) {
    rc = hip_error(e, "hipHostGetDevicePointer(rx ring slots)");
    ring_free(r);
    return rc;
  }
  r->st.resize(depth);
  const size_t bb = (size_t)batch_slots * slot_cap;
  for (auto& s : r->st) {
    if ((e = hipStreamCreateWithFlags(&s.s, hipStreamNonBlocking)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&s.d_bytes), bb)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&s.d_start), ((size_t)batch_slots + 1) * 8)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&s.d_len), (size_t)batch_slots * 4)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&s.d_ok), batch_slots)) != hipSuccess ||
        (e = hipMalloc(reinterpret_cast<void**>(&s.d_verdict), batch_slots)) != hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&s.h_pack), bb, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&s.h_off), ((size_t)batch_slots + 1) * 8, hipHostMallocDefault)) !=
            hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&s.h_len), (size_t)batch_slots * 4, hipHostMallocDefault)) !=
            hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&s.h_ok), batch_slots, hipHostMallocDefault)) != hipSuccess ||
        (e = hipHostMalloc(reinterpret_cast<void**>(&s.h_verdict), batch_slots, hipHostMallocDefault)) != hipSuccess) {
      rc = hip_error(e, "rx ring stage allocation");
      ring_free(r);
      return rc;
    }
  }
  *out = r;
  return LNX_OK;
}

void lnx_rx_ring_destroy(lnx_rx_ring* ring) { ring_free(ring); }

uint8_t* lnx_rx_ring_slots(lnx_rx_ring* ring) { return ring ? ring->h_slots : nullptr; }
uint32_t* lnx_rx_ring_lengths(lnx_rx_ring* ring) { return ring ? ring->h_len : nullptr; }

int lnx_rx_ring_set_filter(lnx_rx_ring* r, const lnx_rx_filter* filter) {
  if (!r) return LNX_EINVAL;
  RxFilter f;
  if (!rx_filter_of(filter, &f)) return LNX_EINVAL;
  std::lock_guard<std::mutex> lk(r->mu);
  r->filt = f;
  return LNX_OK;
}

int lnx_rx_ring_ingress(lnx_rx_ring* r, uint32_t first, uint32_t count, uint32_t offset, uint32_t flags,
                        uint8_t* fcs_ok, uint8_t* verdict) {
  if (!r) return LNX_EINVAL;
  if ((uint64_t)first + count > r->nslots || offset >= r->cap) return LNX_EINVAL;
  if (count == 0) return LNX_OK;
  std::lock_guard<std::mutex> lk(r->mu);
  if (count < r->host_below) {  // below the crossover: no launch
    for (uint32_t i = first; i < first + count; ++i) {
      const uint32_t l = std::min(r->h_len[i], r->cap);
      uint8_t ok, v;
      host_rx(r, r->h_slots + (size_t)i * r->cap + offset, l > offset ? l - offset : 0u, flags, &ok, &v);
      if (fcs_ok) fcs_ok[i - first] = ok;
      if (verdict) verdict[i - first] = v;
    }
    r->stats.host_frames += count;
    return LNX_OK;
  }
  hipError_t e = hipSetDevice(r->device);
  if (e != hipSuccess) return hip_error(e, "hipSetDevice");
  int rc = LNX_OK;
  std::vector<bool> packed_pending(r->depth, false);  // stage k's staging is in use by its last batch
  uint32_t k = 0;
  for (uint32_t b0 = first; b0 < first + count && rc == LNX_OK; b0 += r->batch, ++k) {
    const uint32_t nb = std::min(r->batch, first + count - b0);
    auto& s = r->st[k % r->depth];
    auto flen = [&](uint32_t j) -> uint64_t {
      const uint32_t l = std::min(r->h_len[b0 + j], r->cap);
      return l > offset ? l - offset : 0u;
    };
    uint64_t total = 0;
    for (uint32_t j = 0; j < nb; ++j) total += flen(j);
    // whole slots by DMA when the frames fill them (the copy engine moves full
    // slots faster than the kernel reads them in place: 50.9 against 42.1 GiB/s
    // at 1500 B); else, with zero copy, the frames are read in place (only
    // their bytes cross PCIe), without it packed on the host
    const bool dense = total * 10 >= (uint64_t)nb * r->cap * 9;
    if (r->zero_copy && !dense) {
      rc = enqueue_rx(r, s, nb, RxSrc::kSlotsDirect, b0, offset, flags, r->h_ok + b0, r->h_verdict + b0);
      if (rc == LNX_OK) r->stats.zero_copy_frames += nb;
      continue;
    }
    const bool pack = !dense;
    if (pack) {
      if (packed_pending[k % r->depth] && (e = hipStreamSynchronize(s.s)) != hipSuccess) {
        rc = hip_error(e, "rx ring hipStreamSynchronize");
        break;
      }
      pack_batch(s, nb, [&](uint32_t j) { return r->h_slots + (size_t)(b0 + j) * r->cap + offset; }, flen);
    }
    packed_pending[k % r->depth] = pack;
    rc = enqueue_rx(r, s, nb, pack ? RxSrc::kPacked : RxSrc::kSlotsCopy, b0, offset, flags, r->h_ok + b0,
                    r->h_verdict + b0);
  }
  for (auto& s : r->st) {
    const hipError_t se = hipStreamSynchronize(s.s);
    if (se != hipSuccess && rc == LNX_OK) rc = hip_error(se, "rx ring hipStreamSynchronize");
  }
  if (rc == LNX_OK) {
    if (fcs_ok) std::memcpy(fcs_ok, r->h_ok + first, count);
    if (verdict) std::memcpy(verdict, r->h_verdict + first, count);
  }
  return rc;
}

int lnx_ingress_packets(lnx_rx_ring* r, const uint8_t* const* bufs, const uint32_t* lens, uint64_t n,
                        uint32_t offset, uint32_t flags, uint8_t* fcs_ok, uint8_t* verdict) {
  if (!r || (n > 0 && (!bufs || !lens))) return LNX_EINVAL;
  if (offset >= r->cap) return LNX_EINVAL;
  for (uint64_t i = 0; i < n; ++i)
    if (lens[i] > r->cap || (lens[i] > 0 && !bufs[i])) return LNX_EINVAL;
  if (n == 0) return LNX_OK;
  std::lock_guard<std::mutex> lk(r->mu);
  if (n < r->host_below) {  // below the crossover: no launch (netdev's Runner hands over one buffer per call)
    for (uint64_t i = 0; i < n; ++i) {
      uint8_t ok, v;
      host_rx(r, bufs[i] + offset, lens[i] > offset ? lens[i] - offset : 0u, flags, &ok, &v);
      if (fcs_ok) fcs_ok[i] = ok;
      if (verdict) verdict[i] = v;
    }
    r->stats.host_frames += n;
    return LNX_OK;
  }
  hipError_t e = hipSetDevice(r->device);
  if (e != hipSuccess) return hip_error(e, "hipSetDevice");
  // Batches go round-robin over the stages; batch k is packed into the
  // staging of stage k % depth after that stage's previous batch has drained,
  // so the gather (host memcpy, parallel) of batch k+1 overlaps the copies
  // and kernels of batch k.
  const uint32_t depth = r->depth, per = r->batch;
  int rc = LNX_OK;
  std::vector<std::pair<uint64_t, uint32_t>> pending(depth, {0, 0});  // (first frame, count) per stage
  auto drain = [&](uint32_t k) {
    const uint64_t f0 = pending[k].first;
    const uint32_t cnt = pending[k].second;
    pending[k].second = 0;
    const hipError_t se = hipStreamSynchronize(r->st[k].s);
    if (se != hipSuccess) return hip_error(se, "rx ring hipStreamSynchronize");
    if (fcs_ok) std::memcpy(fcs_ok + f0, r->st[k].h_ok, cnt);
    if (verdict) std::memcpy(verdict + f0, r->st[k].h_verdict, cnt);
    return LNX_OK;
  };
  uint64_t i0 = 0;
  for (uint32_t k = 0; i0 < n && rc == LNX_OK; ++k, i0 += per) {
    const uint32_t sk = k % depth;
    if (pending[sk].second) rc = drain(sk);
    if (rc != LNX_OK) break;
    const uint32_t nb = (uint32_t)std::min<uint64_t>(per, n - i0);
    auto& s = r->st[sk];
    auto flen = [&](uint32_t j) -> uint32_t { return lens[i0 + j] > offset ? lens[i0 + j] - offset : 0u; };
    // the caller's buffers are the ring's own slots (RunnerConfig.Buffers from
    // lnx_rx_ring_slots): a frame table only, the kernel reads them in place
    bool direct = r->zero_copy;
    for (uint32_t j = 0; j < nb && direct; ++j) {
      uint64_t pos = 0;  // (an empty frame reads nothing: any position)
      direct = flen(j) == 0 || in_ring(r, bufs[i0 + j], offset, flen(j), &pos);
      s.h_off[j] = pos;
      s.h_len[j] = flen(j);
    }
    if (!direct) pack_batch(s, nb, [&](uint32_t j) { return bufs[i0 + j] + offset; }, flen);
    rc = enqueue_rx(r, s, nb, direct ? RxSrc::kSegDirect : RxSrc::kPacked, 0, 0, flags, s.h_ok, s.h_verdict);
    if (rc == LNX_OK && direct) r->stats.zero_copy_frames += nb;
    if (rc == LNX_OK) pending[sk] = {i0, nb};
  }
  for (uint32_t k = 0; k < depth; ++k) {
    if (!pending[k].second) continue;
    const int d = drain(k);
    if (rc == LNX_OK) rc = d;
  }
  if (rc != LNX_OK) quiesce(r);
  return rc;
}

int lnx_egress_packets(lnx_rx_ring* r, uint8_t* const* bufs, uint32_t* lens, uint64_t n, uint32_t offset,
                       uint32_t capacity, uint32_t flags, uint8_t* status) {
  if (!r || (n > 0 && (!bufs || !lens))) return LNX_EINVAL;
  if (capacity > r->cap || (flags & ~(uint32_t)(LNX_TX_CHECKSUM | LNX_TX_FCS)) != 0) return LNX_EINVAL;
  for (uint64_t i = 0; i < n; ++i)  // (with LNX_TX_FCS even an empty frame grows: it needs its buffer)
    if (lens[i] > capacity || (!bufs[i] && (lens[i] > 0 || (flags & LNX_TX_FCS)))) return LNX_EINVAL;
  if (n == 0) return LNX_OK;
  std::lock_guard<std::mutex> lk(r->mu);
  if (n < r->host_below) {  // below the crossover: no launch
    for (uint64_t i = 0; i < n; ++i) {
      uint8_t* f = bufs[i] + offset;
      uint32_t l = lens[i];
      const uint8_t ck = (flags & LNX_TX_CHECKSUM) ? host_tx_checksum(f, l) : 0u;
      const uint8_t ap = (flags & LNX_TX_FCS) ? host_fcs_append(f, &l, capacity) : 0u;
      lens[i] = l;
      if (status) status[i] = ck ? ck : ap;
    }
    r->stats.host_frames += n;
    return LNX_OK;
  }
  hipError_t e = hipSetDevice(r->device);
  if (e != hipSuccess) return hip_error(e, "hipSetDevice");
  // as lnx_ingress_packets: batches round-robin over the stages, the gather of
  // batch k + 1 and the scatter of batch k - depth + 1 overlap the device work
  const uint32_t depth = r->depth, per = r->batch;
  int rc = LNX_OK;
  std::vector<std::pair<uint64_t, uint32_t>> pending(depth, {0, 0});
  std::vector<bool> in_place(depth, false);  // the stage's batch was patched in the slots (zero copy)
  std::vector<uint32_t> slot_batch;           // zero copy: the batch (k + 1) that last took each slot
  // A batch's results reach the caller only from a stream that completed: on
  // a failed sync its lens and status stay untouched (and, when it was
  // copied, its frames).
  auto drain = [&](uint32_t k) {
    const uint64_t f0 = pending[k].first;
    const uint32_t cnt = pending[k].second;
    pending[k].second = 0;
    auto& s = r->st[k];
    const hipError_t se = hipStreamSynchronize(s.s);
    if (se != hipSuccess) return hip_error(se, "tx ring hipStreamSynchronize");
    const bool copied = !in_place[k];
    parallel_for(cnt, [&](uint32_t a, uint32_t b) {
      for (uint32_t j = a; j < b; ++j) {
        const uint32_t l = s.h_len[j];
        if (copied && l) std::memcpy(bufs[f0 + j] + offset, s.h_pack + s.h_off[j], l);
        lens[f0 + j] = l;
        if (status) status[f0 + j] = s.h_verdict[j] ? s.h_verdict[j] : s.h_ok[j];
      }
    });
    return LNX_OK;
  };
  uint64_t i0 = 0;
  for (uint32_t k = 0; i0 < n && rc == LNX_OK; ++k, i0 += per) {
    const uint32_t sk = k % depth;
    if (pending[sk].second) rc = drain(sk);
    if (rc != LNX_OK) break;
    const uint32_t nb = (uint32_t)std::min<uint64_t>(per, n - i0);
    auto& s = r->st[sk];
    // zero copy when the buffers are the ring's slots (any order): tx_finish
    // reads each frame in place and patches it there.  Only when every frame's
    // room [offset, offset + capacity) lies inside its own slot and no slot
    // serves two frames of the batch: the kernel's stores into one frame then
    // cannot race with its loads of another (the copying form gathers every
    // frame before writing any back, so it stays exact for any buffers).
    bool direct = r->zero_copy;
    if (direct && slot_batch.size() != r->nslots) slot_batch.assign(r->nslots, 0);
    for (uint32_t j = 0; j < nb && direct; ++j) {
      uint64_t pos = 0;
      direct = in_ring(r, bufs[i0 + j], offset, capacity, &pos);
      const uint64_t rel = pos - offset, slot = rel / r->cap;
      direct = direct && rel % r->cap + offset + capacity <= r->cap && slot_batch[slot] != k + 1;
      if (direct) slot_batch[slot] = k + 1;
      s.h_off[j] = pos;
      s.h_len[j] = lens[i0 + j];
    }
    if (direct) {
      in_place[sk] = true;
      rc = enqueue_tx(r, s, nb, 0, capacity, flags, true, 0);
      if (rc == LNX_OK) pending[sk] = {i0, nb}, r->stats.zero_copy_frames += nb;
      continue;
    }
    in_place[sk] = false;
    // each frame's room: the frame, then its padding to 60 bytes and the FCS
    // when they fit `capacity` (else the append leaves it as it is)
    uint64_t o = 0;
    for (uint32_t j = 0; j < nb; ++j) {
      const uint32_t l = lens[i0 + j];
      const uint32_t grown = std::max(l, 60u) + 4u;
      s.h_off[j] = o;
      s.h_len[j] = l;
      o += (flags & LNX_TX_FCS) && grown <= capacity ? grown : l;
    }
    parallel_for(nb, [&](uint32_t a, uint32_t b) {
      for (uint32_t j = a; j < b; ++j)
        if (s.h_len[j]) std::memcpy(s.h_pack + s.h_off[j], bufs[i0 + j] + offset, s.h_len[j]);
    });
    rc = enqueue_tx(r, s, nb, o, capacity, flags);
    if (rc == LNX_OK) pending[sk] = {i0, nb};
  }
  for (uint32_t k = 0; k < depth; ++k) {
    if (!pending[k].second) continue;
    const int d = drain(k);
    if (rc == LNX_OK) rc = d;
  }
  if (rc != LNX_OK) quiesce(r);
  return rc;
}

}  // extern "C"
