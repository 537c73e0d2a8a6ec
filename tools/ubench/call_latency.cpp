// Per-call latency of the netdev packet entries (lnx_ingress_packets,
// lnx_egress_packets) at n frames per call, on the GPU (host threshold 0) and
// on the host path (threshold above n): the crossover sets
// LNX_HOST_BATCH_DEFAULT.  Frames are 1514-B UDP/IPv4
// frames with valid sums and FCS, so both paths do the whole check.
//
//   g++ -O2 -std=c++17 -I include tools/ubench/call_latency.cpp -o tools/ubench/call_latency
//     -L lneto_amd -llneto_amd -Wl,-rpath,'$ORIGIN/../../lneto_amd'  (one line)
//   ./tools/ubench/call_latency [frame_len]
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "lneto_amd.h"

static double now_us() {
  return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

static uint32_t le32(const uint8_t* p) { return p[0] | p[1] << 8 | p[2] << 16 | (uint32_t)p[3] << 24; }

int main(int argc, char** argv) {
  const uint32_t flen = argc > 1 ? (uint32_t)atoi(argv[1]) : 1514;  // without FCS
  const uint32_t cap = 2048, nmax = 4096;
  lnx_rx_ring* ring = nullptr;
  if (lnx_rx_ring_create(0, nmax, cap, 512, 3, &ring) != LNX_OK) {
    fprintf(stderr, "ring create failed\n");
    return 1;
  }
  // one UDP/IPv4 frame, sums by the library's own TX path, FCS appended
  std::vector<uint8_t> proto(cap, 0);
  const uint8_t hdr[] = {0xc0, 0xff, 0xee, 0x00, 0xde, 0xad, 0x4e, 0x8b, 0x3a, 0xf9, 0xfb, 0x6b, 0x08, 0x00,
                         0x45, 0x00, 0, 0, 0, 0, 0x40, 0, 0x40, 0x11, 0, 0, 0xc0, 0xa8, 10, 1, 0xc0, 0xa8, 10, 2,
                         0x14, 0xe9, 0x00, 0x35, 0, 0, 0, 0};
  std::memcpy(proto.data(), hdr, sizeof hdr);
  for (uint32_t i = sizeof hdr; i < flen; ++i) proto[i] = (uint8_t)(i * 131 + 7);
  if (lnx_tx_checksum(proto.data(), flen) != 0) {
    fprintf(stderr, "tx checksum failed\n");
    return 1;
  }
  uint32_t l = flen;
  if (lnx_fcs_append(proto.data(), &l, cap) != 0 || l != flen + 4) {
    fprintf(stderr, "fcs append failed\n");
    return 1;
  }
  if (lnx_ingress_verdict(proto.data(), flen, 0, nullptr) != 0 || lnx_crc32(proto.data(), l) != 0x2144DF1Cu) {
    fprintf(stderr, "frame does not verify (%08x)\n", lnx_crc32(proto.data(), l));
    return 1;
  }
  std::vector<std::vector<uint8_t>> store(nmax, proto);
  std::vector<const uint8_t*> in(nmax);
  std::vector<uint8_t*> out(nmax);
  std::vector<uint32_t> lens(nmax, l), txl(nmax);
  std::vector<uint8_t> ok(nmax), verdict(nmax), status(nmax);
  for (uint32_t i = 0; i < nmax; ++i) in[i] = out[i] = store[i].data();

  const uint32_t ns[] = {1, 2, 4, 8, 16, 32, 64, 128, 256, 512, 1024, 4096};
  for (uint32_t n : ns) {
    for (int side = 0; side < 2; ++side) {  // 0: GPU, 1: host
      lnx_rx_ring_set_host_threshold(ring, side ? 1u << 30 : 0u);
      const int reps = n <= 64 ? 400 : n <= 1024 ? 100 : 30;
      std::vector<double> ti, te;
      for (int r = 0; r < reps + 10; ++r) {
        double t0 = now_us();
        int rc = lnx_ingress_packets(ring, in.data(), lens.data(), n, 0, 0, ok.data(), verdict.data());
        double t1 = now_us();
        if (rc != LNX_OK) {
          fprintf(stderr, "ingress rc %d\n", rc);
          return 1;
        }
        for (uint32_t i = 0; i < n; ++i)
          if (!ok[i] || verdict[i]) {
            fprintf(stderr, "ingress result wrong at %u (side %d)\n", i, side);
            return 1;
          }
        // egress: strip the FCS, regenerate sums and FCS in place
        for (uint32_t i = 0; i < n; ++i) txl[i] = flen;
        double t2 = now_us();
        rc = lnx_egress_packets(ring, out.data(), txl.data(), n, 0, cap, LNX_TX_CHECKSUM | LNX_TX_FCS, status.data());
        double t3 = now_us();
        if (rc != LNX_OK) {
          fprintf(stderr, "egress rc %d\n", rc);
          return 1;
        }
        for (uint32_t i = 0; i < n; ++i)
          if (status[i] || txl[i] != l || le32(store[i].data() + flen) != le32(proto.data() + flen)) {
            fprintf(stderr, "egress result wrong at %u (side %d)\n", i, side);
            return 1;
          }
        if (r >= 10) {
          ti.push_back(t1 - t0);
          te.push_back(t3 - t2);
        }
      }
      std::sort(ti.begin(), ti.end());
      std::sort(te.begin(), te.end());
      printf("{\"n\": %u, \"frame_len\": %u, \"path\": \"%s\", \"ingress_us\": %.2f, \"egress_us\": %.2f, "
             "\"ingress_p90_us\": %.2f, \"egress_p90_us\": %.2f}\n",
             n, l, side ? "host" : "gpu", ti[ti.size() / 2], te[te.size() / 2], ti[ti.size() * 9 / 10],
             te[te.size() * 9 / 10]);
      fflush(stdout);
    }
  }
  lnx_rx_ring_destroy(ring);
  return 0;
}
