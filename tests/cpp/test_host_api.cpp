// C++ mirror of lneto's own checksum tests, run against include/lneto_amd.hpp:
//   ethernet/crc_test.go:8-100   TestCRC32Search
//   lneto_test.go:119-160        TestIPv4TCPChecksum
// plus the FCS-append tail of StackEthernet.Encapsulate (internet/stack-ethernet.go:203-215).
#include <cstdio>
#include <cstring>
#include <vector>

#include "lneto_amd.hpp"

static int failures = 0;
#define EXPECT(cond, ...)                      \
  do {                                         \
    if (!(cond)) {                             \
      std::printf("FAIL %s:%d ", __FILE__, __LINE__); \
      std::printf(__VA_ARGS__);                \
      std::printf("\n");                       \
      ++failures;                              \
    }                                          \
  } while (0)

static std::vector<uint8_t> makeDataWithCRC(int payloadLen) {  // crc_test.go:10-18
  std::vector<uint8_t> data(payloadLen + 4);
  for (int i = 0; i < payloadLen; ++i) data[i] = uint8_t(i);
  uint32_t crc = ethernet::CRC32(lneto::Bytes(data.data(), payloadLen));
  std::memcpy(&data[payloadLen], &crc, 4);  // little-endian host
  return data;
}

static void TestCRC32Search() {
  {
    auto d = makeDataWithCRC(100);
    EXPECT(ethernet::CRC32Search(d, 0) == 100, "finds CRC at end");
    EXPECT(ethernet::CRC32Search(d, 50) == 100, "minOff before CRC");
    EXPECT(ethernet::CRC32Search(d, 100) == 100, "minOff exactly at CRC");
    EXPECT(ethernet::CRC32Search(d, 101) == -1, "minOff past CRC");
  }
  {
    std::vector<uint8_t> d(100);
    for (int i = 0; i < 100; ++i) d[i] = uint8_t(i);
    EXPECT(ethernet::CRC32Search(d, 0) == -1, "no valid CRC");
  }
  {
    std::vector<uint8_t> d = {1, 2, 3};
    EXPECT(ethernet::CRC32Search(d, 0) == -1, "data too short");
  }
  {
    auto d = makeDataWithCRC(20);
    EXPECT(ethernet::CRC32Search(d, -5) == 20, "negative minOff");
  }
  {
    std::vector<uint8_t> d(4);
    uint32_t crc = ethernet::CRC32(lneto::Bytes());
    std::memcpy(d.data(), &crc, 4);
    EXPECT(ethernet::CRC32Search(d, 0) == 0, "CRC at position 0");
  }
  {
    auto d = makeDataWithCRC(50);
    d.resize(d.size() + 50, 0);
    EXPECT(ethernet::CRC32Search(d, 0) == 50, "first valid CRC wins");
  }
}

static void TestIPv4TCPChecksum() {
  const uint8_t pkts[2][74] = {
      {0xc0, 0xff, 0xee, 0x00, 0xde, 0xad, 0x4e, 0x8b, 0x3a, 0xf9, 0xfb, 0x6b, 0x08, 0x00, 0x45, 0x00,
       0x00, 0x3c, 0x01, 0xbe, 0x40, 0x00, 0x40, 0x06, 0xa3, 0xaa, 0xc0, 0xa8, 0x0a, 0x01, 0xc0, 0xa8,
       0x0a, 0x02, 0xe7, 0x0a, 0x00, 0x50, 0x40, 0x60, 0xd5, 0xcc, 0x00, 0x00, 0x00, 0x00, 0xa0, 0x02,
       0xfa, 0xf0, 0x62, 0xbc, 0x00, 0x00, 0x02, 0x04, 0x05, 0xb4, 0x04, 0x02, 0x08, 0x0a, 0xbb, 0xac,
       0x9b, 0xca, 0x00, 0x00, 0x00, 0x00, 0x01, 0x03, 0x03, 0x07},
      {0xc0, 0xff, 0xee, 0x00, 0xde, 0xad, 0x4e, 0x8b, 0x3a, 0xf9, 0xfb, 0x6b, 0x08, 0x00, 0x45, 0x00,
       0x00, 0x3c, 0xfa, 0xfd, 0x40, 0x00, 0x40, 0x06, 0xaa, 0x6a, 0xc0, 0xa8, 0x0a, 0x01, 0xc0, 0xa8,
       0x0a, 0x02, 0xe7, 0x0e, 0x00, 0x50, 0x9c, 0xdc, 0xfe, 0x05, 0x00, 0x00, 0x00, 0x00, 0xa0, 0x02,
       0xfa, 0xf0, 0xde, 0x02, 0x00, 0x00, 0x02, 0x04, 0x05, 0xb4, 0x04, 0x02, 0x08, 0x0a, 0xbb, 0xac,
       0x9b, 0xca, 0x00, 0x00, 0x00, 0x00, 0x01, 0x03, 0x03, 0x07}};
  for (const auto& p : pkts) {
    std::vector<uint8_t> f(p, p + 74);
    lneto::Bytes ip(f.data() + 14, f.size() - 14);
    uint8_t* ipw = f.data() + 14;
    uint16_t wantIP = uint16_t(ipw[10] << 8 | ipw[11]);
    ipw[10] = ipw[11] = 0;  // zero the CRC field (lneto_test.go:143)
    EXPECT(ipv4::CalculateHeaderCRC(ip) == wantIP, "IPv4 CRC want %x", wantIP);
    uint8_t* tcp = ipw + 20;
    uint16_t wantTCP = uint16_t(tcp[16] << 8 | tcp[17]);
    lneto::CRC791 crc;
    ipv4::CRCWriteTCPPseudo(ip, crc);
    tcp[16] = tcp[17] = 0;  // lneto_test.go:153
    uint16_t got = crc.PayloadSum16(lneto::Bytes(tcp, ipv4::TotalLength(ip) - ipv4::HeaderLength(ip)));
    EXPECT(got == wantTCP, "TCP CRC want %x got %x", wantTCP, got);
  }
}

static void TestAppendFCS() {
  internet::StackEthernetConfig bad;
  bad.AppendCRC32 = true;
  EXPECT(!internet::ValidCRCConfig(bad), "AppendCRC32 without CRC32Update must be rejected");
  internet::StackEthernetConfig cfg;
  cfg.AppendCRC32 = true;
  cfg.CRC32Update = ethernet::CRC32Update;
  EXPECT(internet::ValidCRCConfig(cfg), "valid config");
  std::vector<uint8_t> frame(64 + 4, 0);
  for (int i = 0; i < 42; ++i) frame[i] = uint8_t(i * 7 + 1);  // a 42-byte runt (ARP-sized)
  size_t n = internet::AppendFCS(frame.data(), 42, cfg);
  EXPECT(n == 64, "padded to 60 + 4-byte FCS, got %zu", n);
  EXPECT(ethernet::CRC32Search(lneto::Bytes(frame.data(), n), 0) == 60, "FCS found at 60");
  EXPECT(ethernet::CRC32(lneto::Bytes(frame.data(), n)) == LNX_CRC32_RESIDUE, "residue");
}

// The IPv4/UDP frame of TestRxRing's transmit half, finished (checksums set),
// to `dst` (MAC) and `ip` (IPv4 destination): 52 bytes, no FCS.
static std::vector<uint8_t> udpFrame(const uint8_t* dst, const uint8_t* ip) {
  std::vector<uint8_t> f = {0xc0, 0xff, 0xee, 0, 0xde, 0xad, 0x4e, 0x8b, 0x3a, 0xf9, 0xfb, 0x6b, 0x08, 0x00,
                            0x45, 0, 0, 38, 0, 1, 0x40, 0, 64, 17, 0, 0, 192, 168, 10, 1, 192, 168, 10, 2,
                            0x14, 0xe9, 0, 53, 0, 18, 0, 0};
  for (int i = 0; i < 10; ++i) f.push_back(uint8_t('a' + i));
  std::memcpy(f.data(), dst, 6);
  std::memcpy(f.data() + 30, ip, 4);
  lneto::Bytes iph(f.data() + 14, 20);
  const uint16_t h = ipv4::CalculateHeaderCRC(iph);
  f[24] = uint8_t(h >> 8), f[25] = uint8_t(h);
  lneto::CRC791 c;
  ipv4::CRCWriteUDPPseudo(iph, c, 18);
  const uint16_t u = c.PayloadSum16(lneto::Bytes(f.data() + 34, 18));
  f[40] = uint8_t(u >> 8), f[41] = uint8_t(u);
  return f;
}

// The stack filter and an FCS-stripping device through netdev::RxRing
// (internet/stack-ethernet.go:146-161, internet/stack-ip4.go:108-141): frames
// for another MAC or IPv4 address, with or without a broken sum, get
// ErrPacketDrop (2) before the sum is looked at; the stack's own frame passes,
// and its corrupted copy gets ErrBadCRC (3).
static void TestRxRingFilter(netdev::RxRing& ring) {
  const uint8_t us[6] = {0xc0, 0xff, 0xee, 0, 0xde, 0xad}, other[6] = {2, 0xaa, 0xbb, 0xcc, 0xdd, 0xee};
  const uint8_t ip_us[4] = {192, 168, 10, 2}, ip_other[4] = {192, 168, 10, 77};
  std::vector<std::vector<uint8_t>> frames = {udpFrame(us, ip_us), udpFrame(other, ip_us), udpFrame(us, ip_other),
                                              udpFrame(us, ip_us), udpFrame(other, ip_us), udpFrame(us, ip_other)};
  for (int k = 3; k < 6; ++k) frames[k][50] ^= 0x10;  // a payload byte: the UDP sum fails
  internet::StackFilter sf;
  std::memcpy(sf.MAC, us, 6);
  std::memcpy(sf.Addr4, ip_us, 4);
  EXPECT(ring.SetFilter(&sf) == LNX_OK, "set filter");
  ring.SetDeviceStripsFCS(true);
  std::vector<lneto::Bytes> bufs;
  for (auto& f : frames) bufs.emplace_back(f.data(), f.size());
  std::vector<uint8_t> ok, verdict;
  EXPECT(ring.IngressPackets(bufs, 0, ok, verdict) == LNX_OK, "filtered ingress");
  const uint8_t want[6] = {0, 2, 2, 3, 2, 2};
  for (int k = 0; k < 6; ++k) {
    EXPECT(ok[k] == 1, "no FCS on this device: ok[%d] = %d", k, ok[k]);
    EXPECT(verdict[k] == want[k], "verdict[%d] = %d, want %d", k, verdict[k], want[k]);
  }
  EXPECT(ring.SetFilter(nullptr) == LNX_OK, "accept-all again");
  EXPECT(ring.IngressPackets(bufs, 0, ok, verdict) == LNX_OK, "accept-all ingress");
  for (int k = 0; k < 6; ++k) EXPECT(verdict[k] == (k < 3 ? 0 : 3), "accept-all verdict[%d] = %d", k, verdict[k]);
  ring.SetDeviceStripsFCS(false);
}

// netdev's Runner calls IngressPackets with ONE buffer per call
// (x/netdev/runner.go:432-433,469-470): through the ring that pattern must
// never launch a kernel (the host path below the threshold), and the batching
// loop (netdev::RxBatcher: Put per received frame, one Ingress per drain)
// must reach the GPU in whole batches — with identical results either way,
// equal to the per-frame host functions.
struct Collected {
  std::vector<uint8_t> ok, verdict;
};
static void collect(void* ctx, uint64_t i, uint8_t ok, uint8_t v) {
  auto* c = static_cast<Collected*>(ctx);
  if (c->ok.size() <= i) c->ok.resize(i + 1), c->verdict.resize(i + 1);
  c->ok[i] = ok, c->verdict[i] = v;
}
static void TestRunnerPatterns() {
  netdev::RxRing ring;
  EXPECT(ring.Open(0, 1024, 256, 512, 2) == LNX_OK, "ring open");
  const uint8_t us[6] = {0xc0, 0xff, 0xee, 0, 0xde, 0xad}, ip_us[4] = {192, 168, 10, 2};
  internet::StackEthernetConfig cfg;
  cfg.CRC32Update = ethernet::CRC32Update;
  const int kFrames = 3000;
  std::vector<std::vector<uint8_t>> frames(kFrames);
  for (int k = 0; k < kFrames; ++k) {
    std::vector<uint8_t> f = udpFrame(us, ip_us);
    f.resize(f.size() + 68, 0);
    size_t n = internet::AppendFCS(f.data(), 52, cfg);
    f.resize(n);
    if (k % 7 == 3) f[20 + k % 30] ^= 0x04;   // some bad sums / bad FCS
    if (k % 11 == 5) f[n - 1] ^= 0x80;        // a bad FCS only
    frames[k] = f;
  }
  // the reference's pattern: one buffer per call
  const lnx_rx_ring_counters c0 = ring.Stats();
  std::vector<uint8_t> ok1(kFrames), v1(kFrames);
  for (int k = 0; k < kFrames; ++k) {
    std::vector<lneto::Bytes> one = {lneto::Bytes(frames[k].data(), frames[k].size())};
    std::vector<uint8_t> ok, v;
    EXPECT(ring.IngressPackets(one, 0, ok, v) == LNX_OK, "one-frame ingress %d", k);
    ok1[k] = ok[0], v1[k] = v[0];
  }
  const lnx_rx_ring_counters c1 = ring.Stats();
  EXPECT(c1.device_batches == c0.device_batches, "one frame per call launched %llu batches",
         (unsigned long long)(c1.device_batches - c0.device_batches));
  EXPECT(c1.host_frames - c0.host_frames == uint64_t(kFrames), "host frames %llu",
         (unsigned long long)(c1.host_frames - c0.host_frames));
  // the batching loop: every frame Put into a slot, one Ingress per 1024 frames
  Collected got;
  netdev::RxBatcher batcher(ring, collect, &got);
  for (int k = 0; k < kFrames; ++k) EXPECT(batcher.Put(frames[k].data(), uint32_t(frames[k].size())), "put %d", k);
  EXPECT(batcher.Drain() == LNX_OK, "drain");
  const lnx_rx_ring_counters c2 = ring.Stats();
  EXPECT(c2.device_batches - c1.device_batches == 6, "batched: %llu device batches (1024 + 1024 + 952 frames, 512 "
         "per stage)", (unsigned long long)(c2.device_batches - c1.device_batches));
  EXPECT(c2.device_frames - c1.device_frames == uint64_t(kFrames), "device frames");
  int bad = 0;
  for (int k = 0; k < kFrames; ++k) {
    const auto& f = frames[k];
    const uint8_t wok = ethernet::CRC32(lneto::Bytes(f.data(), f.size())) == LNX_CRC32_RESIDUE;
    const int wv = lnx_ingress_verdict(f.data(), f.size() - 4, 0, nullptr);
    bad += ok1[k] != wok || v1[k] != wv || got.ok[k] != wok || got.verdict[k] != wv;
  }
  EXPECT(bad == 0, "%d frames differ between the host path, the batched GPU path and the per-frame functions", bad);
  // RunnerConfig.Buffers carved from the ring (SlotBuffers): one IngressPackets
  // over the slots the receive handler filled, read in place (zero copy)
  std::vector<lneto::Bytes> slots = ring.SlotBuffers(), view;
  for (uint32_t k = 0; k < ring.Slots(); ++k) {
    std::memcpy(ring.Slot(k), frames[k].data(), frames[k].size());
    view.emplace_back(slots[k].p, frames[k].size());
  }
  std::vector<uint8_t> ok3, v3;
  EXPECT(ring.IngressPackets(view, 0, ok3, v3) == LNX_OK, "slot-buffer ingress");
  const lnx_rx_ring_counters c3 = ring.Stats();
  EXPECT(c3.zero_copy_frames - c2.zero_copy_frames == ring.Slots(), "slot buffers read in place: %llu of %u",
         (unsigned long long)(c3.zero_copy_frames - c2.zero_copy_frames), ring.Slots());
  bad = 0;
  for (uint32_t k = 0; k < ring.Slots(); ++k) bad += ok3[k] != ok1[k] || v3[k] != v1[k];
  EXPECT(bad == 0, "%d slot-buffer frames differ", bad);
}

// The receive ring through the C++ mirror: without a GPU it must refuse to
// open (no silent CPU path); with one, a valid and a corrupted frame.
static void TestRxRing() {
  netdev::RxRing ring;
  const int rc = ring.Open(0, 4, 256);
  if (lnx_device_count() == 0) {
    EXPECT(rc == LNX_ENODEV || rc == LNX_EHIP, "ring without a device: got %d", rc);
    return;
  }
  EXPECT(rc == LNX_OK, "ring open: %d", rc);
  uint8_t* f = ring.Slot(0);
  for (int i = 0; i < 60; ++i) f[i] = uint8_t(i);
  internet::StackEthernetConfig cfg;
  cfg.CRC32Update = ethernet::CRC32Update;
  ring.Len(0) = uint32_t(internet::AppendFCS(f, 60, cfg));
  std::memcpy(ring.Slot(1), f, ring.Len(0));
  ring.Slot(1)[5] ^= 1;
  ring.Len(1) = ring.Len(0);
  uint8_t ok[2] = {9, 9}, verdict[2];
  EXPECT(ring.Ingress(0, 2, 0, ok, verdict) == LNX_OK, "ingress");
  EXPECT(ok[0] == 1 && ok[1] == 0, "fcs ok %d %d", ok[0], ok[1]);
  // transmit: an IPv4/UDP frame with stale length and checksum fields, 52 bytes
  std::vector<uint8_t> buf(2 + 128, 0xEE);
  uint8_t* e = buf.data() + 2;
  const uint8_t hdr[] = {0xc0, 0xff, 0xee, 0, 0xde, 0xad, 0x4e, 0x8b, 0x3a, 0xf9, 0xfb, 0x6b, 0x08, 0x00,
                         0x45, 0, 0x12, 0x34, 0, 1, 0x40, 0, 64, 17, 0xAB, 0xCD, 192, 168, 10, 1, 192, 168, 10, 2,
                         0x14, 0xe9, 0, 53, 0x77, 0x77, 0x55, 0x55};
  std::memcpy(e, hdr, sizeof(hdr));
  for (int i = 0; i < 10; ++i) e[42 + i] = uint8_t('a' + i);
  uint8_t* bufs[1] = {buf.data()};
  uint32_t lens[1] = {52};
  uint8_t st[1] = {9};
  EXPECT(ring.EgressPackets(bufs, lens, 1, 2, 256, st) == LNX_OK, "egress");
  EXPECT(st[0] == 0 && lens[0] == 64, "egress status %d len %u", st[0], lens[0]);
  EXPECT(ethernet::CRC32(lneto::Bytes(e, lens[0])) == LNX_CRC32_RESIDUE, "egress FCS residue");
  EXPECT(ipv4::CalculateHeaderCRC(lneto::Bytes(e + 14, 20)) == 0, "egress IPv4 header CRC verifies");
  lneto::CRC791 c;
  ipv4::CRCWriteUDPPseudo(lneto::Bytes(e + 14, 20), c, 18);
  EXPECT(c.PayloadSum16(lneto::Bytes(e + 34, 18)) == 0, "egress UDP CRC verifies");
  EXPECT(buf[0] == 0xEE && buf[1] == 0xEE && buf[2 + 64] == 0xEE, "bytes outside the frame untouched");
  TestRxRingFilter(ring);
  TestRunnerPatterns();
}

int main() {
  TestRxRing();
  TestCRC32Search();
  TestIPv4TCPChecksum();
  TestAppendFCS();
  if (failures) {
    std::printf("%d failures\n", failures);
    return 1;
  }
  std::printf("ok\n");
  return 0;
}
