/*
 * lneto_amd.h — C-ABI of the MI355X-native checksum path of lneto.
 *
 * Scope: the IEEE 802.3 CRC-32 frame-check-sequence
 * (lneto ethernet/crc.go) and the RFC 791 16-bit one's-complement internet
 * checksum (lneto crc.go, type CRC791).  Everything here is integer / byte
 * arithmetic and bit-identical to the reference.
 *
 * Two families of entry points:
 *
 *  1. Per-frame, host-CPU, exact Go semantics.  These back the drop-in
 *     replacements of the reference's single-frame functions and NEVER launch
 *     a GPU kernel (a launch costs microseconds, a 64-byte CRC costs tens of
 *     nanoseconds; SURVEY.md §7 "cgo/HIP boundary").
 *
 *  2. Batched, device-resident, HIP kernels for gfx950.  Frames are packed back
 *     to back in one device buffer and described by N+1 uint64 byte offsets:
 *     frame i is bytes[off[i] : off[i+1]].  These are the hot path.
 *
 * Conventions (mirroring the reference):
 *  - the caller owns every buffer; nothing is retained after a call returns;
 *  - batch entry points return LNX_OK (0) or a negative LNX_E* code and never
 *    abort; per-frame checksum functions return values, never errors;
 *  - `stream` is a hipStream_t passed as an opaque pointer (NULL = the null
 *    stream of the current device); batch calls are asynchronous on it.
 */
#ifndef LNETO_AMD_H
#define LNETO_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- status codes ------------------------------------------------------ */
#define LNX_OK 0
#define LNX_EINVAL (-1)    /* bad argument (NULL pointer with n > 0, ...) */
#define LNX_ENODEV (-2)    /* no HIP device / bad device ordinal */
#define LNX_EHIP (-3)      /* a HIP runtime call failed; see lnx_last_error() */
#define LNX_ENOMEM (-5)

/* CRC-32/ISO-HDLC residue: CRC32(frame || LE32(CRC32(frame))) == this value. */
#define LNX_CRC32_RESIDUE 0x2144DF1Cu

/* ======================================================================== *
 * 1. Per-frame host functions (exact Go semantics, never touch the GPU)
 * ======================================================================== */

/* Go: crc32.Update(crc, crc32.IEEETable, p) — the CRC32Update plugin hook
 * type of internet.StackEthernetConfig (internet/stack-ethernet.go:31-32),
 * surfaced as xnet.StackConfig.EthernetTxCRC32Update (x/xnet/stack-async.go:89)
 * and called at internet/stack-ethernet.go:211-214. */
uint32_t lnx_crc32_update(uint32_t crc, const uint8_t* p, size_t n);

/* Go: ethernet.CRC32(data) (ethernet/crc.go:19-21). CRC32(nil) == 0. */
uint32_t lnx_crc32(const uint8_t* p, size_t n);

/* Go: ethernet.CRC32Search(data, minOffCRC) (ethernet/crc.go:28-47).
 * First off >= max(minOff,0) with CRC32(data[:off]) == LE32(data[off:]),
 * or -1. */
int64_t lnx_crc32_search(const uint8_t* p, size_t n, int64_t min_off);

/* Go: sumWriteEven (crc.go:23-28) — uint32 wrap-around sum of big-endian
 * 16-bit words.  n must be even (the Go method panics on odd length, crc.go:30);
 * here an odd trailing byte is ignored and the caller is expected not to pass one. */
uint32_t lnx_sum_write_even(uint32_t sum, const uint8_t* p, size_t n);

/* Go: sum16 (crc.go:17-21) — CRC791.Sum16() of a running sum. */
uint16_t lnx_sum16(uint32_t sum);

/* Go: CRC791{sum}.PayloadSum16(p) (crc.go:52-59). */
uint16_t lnx_sum16_payload(uint32_t sum, const uint8_t* p, size_t n);

/* Go: lneto.NeverZeroSum (crc.go:65-71). */
uint16_t lnx_never_zero_sum(uint16_t sum16);

/* The receive path's checksum-stage verdict of ONE Ethernet frame (FCS
 * stripped) on the host: the value lnx_ingress_verify_batch_filtered computes
 * per frame (StackEthernet.Demux, internet/stack-ethernet.go:139-165, then
 * demux4 / demux6, internet/stack-ip4.go:100-164, internet/stack-ip6.go:86-138;
 * codes and flags as documented there; filter NULL = accept-all).  Returns the
 * verdict (>= 0) or LNX_EINVAL.  The packet entries (lnx_ingress_packets,
 * lnx_rx_ring_ingress) use it for batches below their host threshold, so
 * netdev's one-buffer-per-call Runner (x/netdev/runner.go:432-433) never
 * launches a kernel. */
#define LNX_VERIFY_EVIL_BIT 1u /* lneto.ValidateEvilBit on the stack's Validator */
#define LNX_VERIFY_ICMP 2u     /* the ICMPv4 / ICMPv6 clients are attached (StackAsync.EnableICMP) */
struct lnx_rx_filter;
int lnx_ingress_verdict(const uint8_t* frame, size_t len, uint32_t flags, const struct lnx_rx_filter* filter);

/* pcap's checksum re-verification of ONE Ethernet frame on the host: what
 * PacketBreakdown.CaptureEthernet records about the frame's checksums
 * (internet/pcap/capture.go:67-277), which differs from the receive path's
 * verdict: a bad IPv4 header sum is recorded and the transport check still
 * runs (:229-231); on IPv4 the TCP / UDP checks run only when tcp / udp.NewFrame
 * accept the payload (:241-266), a UDP checksum of 0 is not checked (:259),
 * ICMPv4 is always summed with no pseudo-header (:267-273); IPv6 sums UDP and
 * UDPLite over the UDP length (:184-198).  Returns the status byte (>= 0):
 * LNX_PCAP_IP_HDR_BAD | LNX_PCAP_PROTO_BAD | code << 2, code = the errGeneric
 * value (15 ErrInvalidLengthField, 18 ErrTruncatedFrame) of a size check that
 * ends the capture on the way to the transport check (IPv6 UDP / UDPLite: the
 * error pcap records in its place), else 0; or LNX_EINVAL.  802.3 length
 * frames, VLAN-tagged frames and other EtherTypes have no checksum stage in
 * pcap (status 0 unless their Ethernet size check fails). */
#define LNX_PCAP_IP_HDR_BAD 1u /* ErrBadCRC in the IPv4 frame's Errors */
#define LNX_PCAP_PROTO_BAD 2u  /* ipProtoErr == ErrBadCRC (the transport frame's Errors) */
int lnx_pcap_checksums(const uint8_t* frame, size_t len);

/* The transmit checksum step of ONE frame on the host, in place: the per-frame
 * semantics of lnx_tx_checksum_batch (encapsulate4 / encapsulate6 / the ICMP
 * clients, internet/stack-ip4.go:202-228, internet/stack-ip6.go:167-181).
 * Returns the status (0, 18 ErrTruncatedFrame, 15 ErrInvalidLengthField) or
 * LNX_EINVAL. */
int lnx_tx_checksum(uint8_t* frame, size_t len);

/* StackEthernet.Encapsulate's tail with the CRC32Update hook set, ONE frame on
 * the host (internet/stack-ethernet.go:200-214): zero-pad to 60 bytes, append
 * the LE FCS, *len = the new length; 6 (ErrShortBuffer) with the frame
 * untouched when it would outgrow `capacity`; LNX_EINVAL for NULL pointers. */
int lnx_fcs_append(uint8_t* frame, uint32_t* len, uint32_t capacity);

/* ======================================================================== *
 * 2. Batched device-resident HIP path (gfx950)
 * ======================================================================== */

/* d_crc[i] = CRC32(d_bytes[d_off[i] : d_off[i+1]]) for i in [0, n).
 * d_off holds n+1 offsets, non-decreasing for the fast paths; offsets out of
 * order are accepted too (a frame whose end offset is below its start is
 * treated as empty, CRC 0; every other frame, overlapping ones included, gets
 * the CRC of its own bytes).  Frames may have any length and any byte
 * alignment.  Each workgroup slice's kernel is picked on the device from its
 * offsets, so the call never reads device memory on the host
 * and never syncs.  Replaces n calls of
 * ethernet.CRC32 (ethernet/crc.go:19-21) / of the CRC32Update hook with crc=0
 * (internet/stack-ethernet.go:211-214). */
int lnx_crc32_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n,
                    uint32_t* d_crc, void* stream);

/* lnx_crc32_batch / lnx_fcs_verify_batch with flags.  LNX_BATCH_SHORT_FRAMES
 * forces the staged lane-stream kernel (each 128-byte line
 * requested once) for every slice that is not giant, where the plain entries
 * let the device pick per slice (uniform lengths the rows kernel is faster at
 * go to it).  Results are identical either way.  Other bits must be 0. */
#define LNX_BATCH_SHORT_FRAMES 1u
int lnx_crc32_batch_ex(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t* d_crc, uint32_t flags,
                       void* stream);
int lnx_fcs_verify_batch_ex(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint8_t* d_ok,
                            uint32_t flags, void* stream);

/* Segment form of lnx_crc32_batch for frames that are not packed back to back
 * (ring slots): d_crc[i] = CRC32(d_bytes[d_start[i] : d_start[i] + d_len[i]]).
 * Any order, overlap allowed.  Frames in increasing address order that do not
 * overlap take the pipelined rows; a workgroup slice that is not
 * (start[i] + len[i] > start[i + 1] somewhere) is folded frame by frame, each
 * from its own start. */
int lnx_crc32_segments(const uint8_t* d_bytes, const uint64_t* d_start, const uint32_t* d_len, uint64_t n,
                       uint32_t* d_crc, void* stream);

/* Batched TX FCS append: the tail of
 * StackEthernet.Encapsulate with the CRC32Update hook set
 * (internet/stack-ethernet.go:200-214) for every frame
 * d_bytes[d_start[i] : d_start[i] + d_len[i]]: zero-pad to 60 bytes, write
 * LE32(CRC32(padded frame)) after it, d_len[i] = padded length + 4.  Each frame
 * may grow to `capacity` bytes; a frame that would not fit is left untouched
 * with d_status[i] = 6 (lneto.ErrShortBuffer), else d_status[i] = 0.  Frames
 * in any order; their rooms [start, start + capacity) must not overlap.  A
 * workgroup slice in increasing address order takes the pipelined rows
 * (addressed relative to its first frame), any other slice is folded frame by
 * frame from each frame's own start (as lnx_crc32_segments).  The reference's
 * onSend hook (between padding and FCS) has no batch equivalent. */
int lnx_fcs_append_batch(uint8_t* d_bytes, const uint64_t* d_start, uint32_t* d_len, uint64_t n, uint32_t capacity,
                         uint8_t* d_status, void* stream);

/* Batched transmit checksum generate: for every
 * frame d_bytes[d_start[i] : d_start[i] + d_len[i]] — an Ethernet header and
 * the IP packet a stack child just wrote, before padding and FCS — the step
 * encapsulate4 / encapsulate6 and the ICMP clients run after the child
 * (internet/stack-ip4.go:202-228, internet/stack-ip6.go:167-181,
 * ipv4/icmpv4/client.go:210-214, ipv6/icmpv6/client.go:135-148), in place:
 *   IPv4: total length = len - 14; header CRC over the first 20 bytes
 *         (ipv4/frame.go:138-146); TCP CRC with CRCWriteTCPPseudo; UDP length
 *         = n and UDP CRC with CRCWriteUDPPseudo(n) through NeverZeroSum
 *         (crc.go:65-71); ICMP CRC over the message with a zero seed;
 *   IPv6: payload length = len - 54; TCP / UDP / ICMPv6 CRC with
 *         CRCWritePseudo (ipv6/frame.go:104-108), UDP length = n, NeverZeroSum
 *         for UDP.
 * The header length is the frame's own IHL.  d_status[i] = 0 when done (other
 * EtherTypes and IP protocols: nothing, or the IPv4 header CRC / the IPv6
 * payload length only), else the frame is untouched and d_status[i] = 18
 * (lneto.ErrTruncatedFrame: too short for the IP header or for the TCP 20 /
 * UDP 8 / ICMP 8-byte header the step writes) or 15 (ErrInvalidLengthField:
 * IHL < 5, or a length over 16 bits).  Frames must not overlap.  Two
 * launches, one of which works: the generate rows, or for a batch whose mean
 * of 64 sampled lengths is under 896 B lnx_tx_finish_batch's checksum step
 * (the same bytes and status; d_len is not written either way). */
int lnx_tx_checksum_batch(uint8_t* d_bytes, const uint64_t* d_start, const uint32_t* d_len, uint64_t n,
                          uint8_t* d_status, void* stream);

/* The transmit tail in ONE read of each frame: lnx_tx_checksum_batch's
 * checksum step (flags & LNX_TX_CHECKSUM) followed by lnx_fcs_append_batch's
 * padding and FCS (flags & LNX_TX_FCS), over the frames as the stack wrote them
 * (StackEthernet.Encapsulate after encapsulate4 / encapsulate6,
 * internet/stack-ethernet.go:200-214, internet/stack-ip4.go:202-228,
 * internet/stack-ip6.go:167-181).  The CRC is taken over the frame as loaded
 * and corrected for the fields the checksum step writes, so
 * the result equals the two calls in sequence.  d_len[i] is updated; each frame
 * may grow to `capacity` bytes; d_status[i] = the checksum step's status if
 * non-zero (18, 15), else the append's (0, or 6 lneto.ErrShortBuffer with the
 * frame left unpadded).  Frames must not overlap (any order).  The flag values
 * are LNX_TX_CHECKSUM and LNX_TX_FCS (declared with lnx_egress_packets). */
int lnx_tx_finish_batch(uint8_t* d_bytes, const uint64_t* d_start, uint32_t* d_len, uint64_t n, uint32_t capacity,
                        uint32_t flags, uint8_t* d_status, void* stream);

/* FCS verify of received frames that still carry their 4-byte LE FCS:
 * d_ok[i] = 1 iff len_i >= 4 and CRC32(f[:len_i-4]) == LE32(f[len_i-4:]),
 * evaluated as the residue test CRC32(f) == LNX_CRC32_RESIDUE.  This is the
 * check lneto leaves to the PHY (x/netdev/interface.go:34-40) and would do at
 * netdev.Stack.IngressPackets (x/netdev/interface.go:89) — SURVEY.md §8(f).1. */
int lnx_fcs_verify_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n,
                         uint8_t* d_ok, void* stream);

/* Internet checksum of n segments: d_out[i] = CRC791{d_seed[i]}.PayloadSum16(
 * d_bytes[d_off[i] : d_off[i] + d_len[i]])  (crc.go:52-59).  d_seed may be
 * NULL (all-zero seeds).  The seed is the pseudo-header partial sum written by
 * ipv4.Frame.CRCWriteTCPPseudo / CRCWriteUDPPseudo (ipv4/frame.go:154-170) or
 * ipv6.Frame.CRCWritePseudo (ipv6/frame.go:104-108). */
int lnx_sum16_batch(const uint8_t* d_bytes, const uint64_t* d_off, const uint32_t* d_len,
                    const uint32_t* d_seed, uint64_t n, uint16_t* d_out, void* stream);

/* Batched ethernet.CRC32Search (ethernet/crc.go:28-47), SURVEY.md §8(f).4:
 * d_result[i] = CRC32Search(d_bytes[d_off[i] : d_off[i+1]], d_min_off[i]) —
 * the first off >= max(minOff, 0) with CRC32(capture[:off]) ==
 * LE32(capture[off:off+4]), or -1 (also when the capture is shorter than
 * minOff + 4).  d_min_off may be NULL (all 0).  For PIO captures of unknown
 * frame length (phy/rmii.md:265-271); every prefix CRC of a capture is
 * computed in one parallel scan. */
int lnx_crc32_search_batch(const uint8_t* d_bytes, const uint64_t* d_off, const int64_t* d_min_off, uint64_t n,
                           int64_t* d_result, void* stream);

/* Receive-path checksum verdicts, fused kernels: for
 * every Ethernet frame d_bytes[d_off[i] : d_off[i+1]] (FCS already stripped)
 * d_verdict[i] = the result lneto's receive path reaches at its checksum
 * stage — StackEthernet.Demux size checks (internet/stack-ethernet.go:139-165),
 * then by EtherType demux4 (internet/stack-ip4.go:100-164: ValidateExceptCRC,
 * IPv4 header sum over the first 20 bytes, TCP / UDP sums with pseudo-header)
 * or demux6 (internet/stack-ip6.go:86-138).  0 = all checks passed or none
 * applies (other EtherTypes); otherwise the lneto errGeneric value
 * (errors.go:6-28): 2 ErrPacketDrop (evil bit, only with LNX_VERIFY_EVIL_BIT;
 * an ICMPv4 type other than echo / echo reply, only with LNX_VERIFY_ICMP),
 * 3 ErrBadCRC, 14 ErrInvalidField, 15 ErrInvalidLengthField,
 * 18 ErrTruncatedFrame.  Destination filtering and handler lookup are stack
 * configuration and are taken as accept-all.  With LNX_VERIFY_ICMP, ICMP
 * messages also take their client's Demux checks up to the checksum
 * (ipv4/icmpv4/client.go:89-102, ipv6/icmpv6/client.go:100-115).  Two
 * launches, one of which works: the ingress rows, or for a batch whose mean
 * frame is under 1280 B the receive check's rows without the CRC (the same
 * verdicts; the choice is made on the device from d_off[0] and d_off[n], with
 * a word of the stream's scratch, as lnx_crc32_batch). */
int lnx_ingress_verify_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t flags,
                             uint8_t* d_verdict, void* stream);

/* The stack configuration behind the receive path's ErrPacketDrop checks, so
 * that a frame the stack would not accept gets ErrPacketDrop (2) with the
 * reference's precedence over the checksum verdicts:
 *   StackEthernet.Demux (internet/stack-ethernet.go:146-161): before
 *     ValidateSize, a frame that is neither broadcast nor for `mac` is dropped
 *     unless eth_accept_multicast and the destination's group bit is set
 *     (SetAcceptMulticast, :56-58); after it, an EtherType with no handler
 *     (RegisterEthernet) is dropped;
 *   demux4 (internet/stack-ip4.go:108-119,135-141): with ip4 != 0.0.0.0, a
 *     destination other than ip4 is dropped before ValidateExceptCRC unless
 *     ip4_accept_multicast and it is 224/4 or ip4_accept_broadcast and it is
 *     255.255.255.255 (ipv4/definitions.go:17-36); a protocol with no handler
 *     (bit p of ip4_protocols: byte p / 8, bit p % 8) is dropped after the
 *     header sum and before the TCP / UDP sums;
 *   demux6 (internet/stack-ip6.go:93-111): with ip6 != ::, a destination other
 *     than ip6 is dropped before ValidateSize unless ip6_accept_multicast and
 *     it is ff00::/8 (internal/ip.go:30-38); a next header with no handler is
 *     dropped before the sums.
 * A NULL filter is accept-all (lnx_ingress_verify_batch). */
typedef struct lnx_rx_filter {  /* (EtherTypes must be > 1500: RegisterEthernet, stack-ethernet.go:131-135) */
  uint8_t mac[6];                 /* StackEthernetConfig.MAC */
  uint8_t eth_accept_multicast;   /* StackEthernet.SetAcceptMulticast */
  uint8_t ip4_accept_multicast;   /* stackip4 SetAcceptMulticast / SetAcceptBroadcast */
  uint8_t ip4_accept_broadcast;
  uint8_t ip6_accept_multicast;   /* stackip6 SetAcceptMulticast6 */
  uint8_t ip4[4];                 /* stackip4 address, all zero = accept every destination */
  uint8_t ip6[16];                /* stackip6 address, all zero = accept every destination */
  uint16_t ethertypes[8];         /* EtherTypes with a registered handler */
  uint32_t n_ethertypes;          /* entries of ethertypes in use (<= 8) */
  uint8_t ip4_protocols[32];      /* 256-bit set of IP protocols with a handler on the IPv4 stack */
  uint8_t ip6_protocols[32];      /* the same for the IPv6 stack */
} lnx_rx_filter;
int lnx_ingress_verify_batch_filtered(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t flags,
                                      const lnx_rx_filter* filter, uint8_t* d_verdict, void* stream);

/* lneto's whole receive check in ONE pass over each frame:
 * for every frame d_bytes[d_off[i] : d_off[i+1]] carrying its 4-byte LE FCS,
 * d_fcs_ok[i] = the FCS test of lnx_fcs_verify_batch and d_verdict[i] = the
 * verdict lnx_ingress_verify_batch_filtered gives the frame without its FCS
 * (flags LNX_VERIFY_EVIL_BIT / LNX_VERIFY_ICMP, filter NULL = accept-all).
 * With LNX_RX_NO_FCS (a device that strips the FCS) no CRC is taken,
 * d_fcs_ok[i] = 1 and the verdict covers the whole frame.  The receive ring
 * runs it for its batches. */
int lnx_rx_verify_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint32_t flags,
                        const lnx_rx_filter* filter, uint8_t* d_fcs_ok, uint8_t* d_verdict, void* stream);

/* pcap's checksum re-verification over a batch: d_status[i] =
 * lnx_pcap_checksums(d_bytes[d_off[i] : d_off[i+1]]) for every Ethernet frame
 * (FCS stripped; an end offset below its start is an empty frame).  Four
 * frames per wave (16-lane rows); every offset order is allowed. */
int lnx_pcap_verify_batch(const uint8_t* d_bytes, const uint64_t* d_off, uint64_t n, uint8_t* d_status,
                          void* stream);

/* Host-memory convenience: copies h_bytes/h_off to the device, runs
 * lnx_crc32_batch, copies the CRCs back, synchronously.  Used to measure the
 * PCIe-inclusive rate.  nbytes is the length of h_bytes; every
 * offset must be <= nbytes. `device` is the HIP device ordinal. */
int lnx_crc32_batch_host(const uint8_t* h_bytes, uint64_t nbytes, const uint64_t* h_off,
                         uint64_t n, uint32_t* h_crc, int device);

/* Multi-GPU: the frame index range [0, n) is split into ngpu contiguous
 * slices, one host thread per device; device g computes its slice from its own
 * copy of the data: d_bytes_per_gpu[g] / d_off_per_gpu[g] describe that
 * device's frames (offsets local to its buffer), d_crc_per_gpu[g] receives
 * its results.  No collective, no peer traffic. */
int lnx_crc32_batch_multi(int ngpu, const int* devices, const uint8_t* const* d_bytes_per_gpu,
                          const uint64_t* const* d_off_per_gpu, const uint64_t* n_per_gpu,
                          uint32_t* const* d_crc_per_gpu);

/* ======================================================================== *
 * 3. Receive ring: pinned slots + batched FCS verify / ingress verdicts
 *    
 * ======================================================================== */

/* A pool of `nslots` receive slots of `slot_cap` bytes in pinned host memory,
 * modelled on netdev's bufferSelect (x/netdev/buffer.go:25-37: fixed slots, a
 * length per slot), with `depth` device pipeline stages of `batch_slots`
 * slots each (batch_slots * slot_cap < 2 GiB; 0 = nslots).  A producer writes
 * frames straight into the slots (lnx_rx_ring_slots) and their buffer lengths
 * into lnx_rx_ring_lengths.  slot_cap must be a multiple of 4. */
typedef struct lnx_rx_ring lnx_rx_ring;
int lnx_rx_ring_create(int device, uint32_t nslots, uint32_t slot_cap, uint32_t batch_slots, uint32_t depth,
                       lnx_rx_ring** out);
void lnx_rx_ring_destroy(lnx_rx_ring* ring);
/* Pinned slot memory: slot i is bytes [i*slot_cap, (i+1)*slot_cap). */
uint8_t* lnx_rx_ring_slots(lnx_rx_ring* ring);
/* Pinned buffer length per slot (bytes of slot i in use, <= slot_cap). */
uint32_t* lnx_rx_ring_lengths(lnx_rx_ring* ring);

/* The ring's stack configuration for its verdicts (a copy of *filter is
 * kept; NULL = accept-all, the default).  LNX_EINVAL for more than 8 EtherTypes. */
int lnx_rx_ring_set_filter(lnx_rx_ring* ring, const lnx_rx_filter* filter);

/* Batches of fewer than `frames` frames (lnx_rx_ring_ingress counts,
 * lnx_ingress_packets / lnx_egress_packets n) run on the host with the
 * per-frame functions above (lnx_ingress_verdict, lnx_tx_checksum,
 * lnx_fcs_append, the residue test): no kernel launch, no copy.  The default,
 * LNX_HOST_BATCH_DEFAULT, is the measured crossover of the GPU round trip
 * (DESIGN.md §4 "per-call latency"); 0 sends every batch to the GPU. */
#define LNX_HOST_BATCH_DEFAULT 64u
int lnx_rx_ring_set_host_threshold(lnx_rx_ring* ring, uint32_t frames);

/* Where the ring's frames went since it was created (in the spirit of netdev's
 * RunnerStatistics, x/netdev/runner.go:107-140): frames folded on the host
 * below the threshold, frames and batches (one H2D / kernels / D2H round
 * trip each) sent to the GPU. */
typedef struct lnx_rx_ring_counters {
  uint64_t host_frames;
  uint64_t device_frames;
  uint64_t device_batches;
  uint64_t zero_copy_frames;  /* of device_frames: read (and, egress, patched) in place in the slots */
} lnx_rx_ring_counters;
int lnx_rx_ring_stats(lnx_rx_ring* ring, lnx_rx_ring_counters* out);

/* Zero copy (on by default): the ring's slots are mapped into the GPU's
 * address space and the kernels read the frames in place over PCIe, so no host
 * thread copies a frame and only frame bytes cross the link.  This covers
 * lnx_rx_ring_ingress (a batch whose frames fill >= 90 % of their slots still
 * goes up by DMA of whole slots, the faster mover there) and, when every
 * buffer of a batch lies in the ring's slot memory (netdev
 * RunnerConfig.Buffers carved from lnx_rx_ring_slots,
 * x/netdev/runner.go:92-94), lnx_ingress_packets and lnx_egress_packets (whose
 * kernel then patches the frames in place: one read of each frame, stores of
 * the fields, padding and FCS only).  Other buffers are gathered into pinned
 * staging as before.
 * on = 0 selects the copying forms for every batch. */
int lnx_rx_ring_set_zero_copy(lnx_rx_ring* ring, int on);

/* Device delivers frames without their FCS (x/netdev/interface.go:34-40 leaves
 * the FCS to "device or stack"): no FCS check (fcs_ok = 1), verdicts on the
 * whole frame. */
#define LNX_RX_NO_FCS 4u

/* netdev.Stack.IngressPackets (x/netdev/interface.go:82-89;
 * xnet.Netstack.IngressPackets, x/xnet/netstack.go:103-111) for slots
 * [first, first + count): the frame of slot i is slot[offset : len_i] and
 * carries its 4-byte LE FCS (unless LNX_RX_NO_FCS).  fcs_ok[k] = 1 iff that
 * FCS is right (the check lneto leaves to the PHY, x/netdev/interface.go:34-40);
 * verdict[k] = the receive path's checksum-stage verdict of the frame with the
 * FCS stripped, as lnx_ingress_verify_batch_filtered with the ring's filter.
 * Host output arrays of `count` entries (either may be NULL).  Synchronous;
 * internally the slot range is pipelined over the ring's stages (H2D, kernels,
 * D2H on one HIP stream per stage).  A batch whose frames fill less than 90 %
 * of its slots is packed back to back on the host first, so the copy moves the
 * frame bytes and their offsets, not whole slots. */
int lnx_rx_ring_ingress(lnx_rx_ring* ring, uint32_t first, uint32_t count, uint32_t offset, uint32_t flags,
                        uint8_t* fcs_ok, uint8_t* verdict);

/* The same for caller-owned buffers, exactly IngressPackets(bufs, offset):
 * frame k = bufs[k][offset : lens[k]] (lens[k] <= slot_cap).  The frames are
 * gathered back to back into pinned staging (parallel host copies, overlapped
 * with the device work of the previous batch), so PCIe carries the frame bytes
 * plus 8 bytes of offset per frame; nothing is retained after the call. */
int lnx_ingress_packets(lnx_rx_ring* ring, const uint8_t* const* bufs, const uint32_t* lens, uint64_t n,
                        uint32_t offset, uint32_t flags, uint8_t* fcs_ok, uint8_t* verdict);

/* netdev.Stack.EgressPackets(bufs, sizes, offset) (x/netdev/interface.go:85;
 * xnet.Netstack.EgressPackets, x/xnet/netstack.go:87-98) for the device's part
 * of the transmit path: frame k = bufs[k][offset : offset + lens[k]] is what
 * the stack wrote (Ethernet header + IP packet, before padding and FCS).  With
 * LNX_TX_CHECKSUM its length fields and checksums are generated as
 * lnx_tx_checksum_batch does; with LNX_TX_FCS it is padded to 60 bytes and
 * its LE FCS appended as lnx_fcs_append_batch does, within `capacity` bytes
 * (<= the ring's slot_cap).  The frames come back in place, lens[k] = the new
 * length; status[k] (may be NULL) = the checksum step's status if non-zero,
 * else the append's (0, or 6 ErrShortBuffer with the frame unpadded).
 * Synchronous; the batches are pipelined over the ring's stages (gather, H2D,
 * kernels, D2H, scatter), nothing is retained after the call.  Frames travel
 * packed back to back, each with room for its padding and FCS only.  On an
 * error return the frames of batches that completed before the error may
 * already be written back (with their lens and status); the failing batch's
 * and later lens and status are left as they were, and every stage has
 * drained before the call returns.  The failing batch's frames are left as
 * they were too, except under zero copy (lnx_rx_ring_set_zero_copy), where the
 * kernel patches them in place in the slots: they may then already be padded
 * and carry their FCS while their lens are stale.  Zero copy is taken for a
 * batch only when every frame's room [offset, offset + capacity) lies inside
 * one slot and no slot holds two of the batch's frames.  lnx_ingress_packets
 * writes results the same way. */
#define LNX_TX_CHECKSUM 1u
#define LNX_TX_FCS 2u
int lnx_egress_packets(lnx_rx_ring* ring, uint8_t* const* bufs, uint32_t* lens, uint64_t n, uint32_t offset,
                       uint32_t capacity, uint32_t flags, uint8_t* status);

/* Number of visible HIP devices (0 when none). */
int lnx_device_count(void);

/* Human-readable description of the last LNX_EHIP failure on this thread. */
const char* lnx_last_error(void);

/* Library build identification (kernel variant, gfx target). */
const char* lnx_version(void);

#ifdef __cplusplus
}
#endif

#endif /* LNETO_AMD_H */
