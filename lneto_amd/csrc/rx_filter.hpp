// rx_filter.hpp — the stack configuration behind the receive verdicts'
// ErrPacketDrop checks, as the kernel sees it (ingress_kernel.hip), and its
// conversion from the C-ABI's lnx_rx_filter (include/lneto_amd.h).
#pragma once
#include <cstdint>
#include <cstring>
#include "../../include/lneto_amd.h"

namespace lnx {

// Kernel-argument form.  on = 0: accept-all (every destination, a handler for
// every EtherType and IP protocol), the verdicts of lnx_ingress_verify_batch.
struct RxFilter {
  uint32_t on;
  uint32_t mac_lo, mac_hi;  // StackEthernet MAC bytes 0..3, 4..5 (little-endian packed)
  uint32_t eth_mc, ip4_mc, ip4_bc, ip6_mc;
  uint32_t ip4;             // stackip4 address bytes (LE packed); 0 = accept every destination
  uint32_t ip6[4];          // stackip6 address; all 0 = accept every destination
  uint32_t n_et;
  uint32_t et[8];           // EtherTypes with a handler (RegisterEthernet)
  uint32_t p4[8], p6[8];    // IP protocols with a handler (256-bit masks)
};

inline uint32_t le32_of(const uint8_t* b) { return b[0] | (b[1] << 8) | (b[2] << 16) | ((uint32_t)b[3] << 24); }

// NULL: accept-all.  Returns false for a filter with more than 8 EtherTypes,
// or with an EtherType the stack cannot register: RegisterEthernet rejects
// proto <= 1500 (802.3 length values) with ErrInvalidConfig
// (internet/stack-ethernet.go:131-135), so such a frame always ends in DROP.
inline bool rx_filter_of(const lnx_rx_filter* f, RxFilter* out) {
  RxFilter r{};
  if (f) {
    if (f->n_ethertypes > 8) return false;
    for (uint32_t i = 0; i < f->n_ethertypes; ++i)
      if (f->ethertypes[i] <= 1500) return false;
    r.on = 1;
    r.mac_lo = le32_of(f->mac);
    r.mac_hi = f->mac[4] | (f->mac[5] << 8);
    r.eth_mc = f->eth_accept_multicast != 0;
    r.ip4_mc = f->ip4_accept_multicast != 0;
    r.ip4_bc = f->ip4_accept_broadcast != 0;
    r.ip6_mc = f->ip6_accept_multicast != 0;
    r.ip4 = le32_of(f->ip4);
    for (int i = 0; i < 4; ++i) r.ip6[i] = le32_of(f->ip6 + 4 * i);
    r.n_et = f->n_ethertypes;
    for (uint32_t i = 0; i < f->n_ethertypes; ++i) r.et[i] = f->ethertypes[i];
    for (int i = 0; i < 8; ++i) {
      r.p4[i] = le32_of(f->ip4_protocols + 4 * i);
      r.p6[i] = le32_of(f->ip6_protocols + 4 * i);
    }
  }
  *out = r;
  return true;
}

}  // namespace lnx
