/*
 * crc_oracle.c — CPU restatement of lneto's checksum path.  TEST
 * INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py as the checker.  Nothing in lneto_amd/ links or
 * calls this file.
 *
 * Reference being restated (lneto @ /root/reference):
 *   - ethernet/crc.go:13      crcTable = crc32.MakeTable(crc32.IEEE)
 *   - ethernet/crc.go:19-21   CRC32(data) = crc32.Checksum(data, crcTable)
 *   - ethernet/crc.go:28-47   CRC32Search(data, minOffCRC)
 *   - crc.go:17-21            sum16
 *   - crc.go:23-28            sumWriteEven
 *   - crc.go:52-59            (*CRC791).PayloadSum16
 *   - crc.go:65-71            NeverZeroSum
 *
 * The CRC-32 arithmetic itself lives in a dependency that is not in the
 * reference tree: the Go standard library package hash/crc32 (go.mod:3 floor
 * go1.24; CI pins go1.26, .github/workflows/ci.yaml:109).  Its published
 * algorithm for IEEETable is CRC-32/ISO-HDLC: reflected polynomial 0xEDB88320,
 * register initialised to ~crc, one table step per byte
 *     crc = tab[(byte)crc ^ b] ^ (crc >> 8),
 * result complemented (hash/crc32 simpleUpdate / Update).  For inputs >= 16
 * bytes the generic Go path uses slicing-by-8 (slicing8Update) over eight
 * tables derived from the same table; both forms are restated below and are
 * cross-checked against each other by the tests.  Parity of absolute CRC
 * values is pinned by the CRC-32/ISO-HDLC check value 0xCBF43926 and by
 * Python's zlib.crc32 (same algorithm), and by the reference's own
 * self-consistency tests (ethernet/crc_test.go:8-100); see tests/golden/.
 *
 * Build: `make -C oracle` -> oracle/liboracle.so (gcc, no GPU).
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

static uint32_t ieee_tab[8][256];
static int tab_ready = 0;

/* hash/crc32 simpleMakeTable(IEEE) + slicing8 tables */
static void make_tables(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t crc = i;
    for (int j = 0; j < 8; j++) crc = (crc & 1) ? (crc >> 1) ^ 0xEDB88320u : crc >> 1;
    ieee_tab[0][i] = crc;
  }
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t crc = ieee_tab[0][i];
    for (int j = 1; j < 8; j++) {
      crc = ieee_tab[0][crc & 0xff] ^ (crc >> 8);
      ieee_tab[j][i] = crc;
    }
  }
  tab_ready = 1;
}

static inline void ensure_tables(void) {
  if (!tab_ready) make_tables();
}

/* hash/crc32 simpleUpdate: one table step per byte. */
uint32_t oracle_crc32_update_simple(uint32_t crc, const uint8_t* p, size_t n) {
  ensure_tables();
  crc = ~crc;
  for (size_t i = 0; i < n; i++) crc = ieee_tab[0][(uint8_t)crc ^ p[i]] ^ (crc >> 8);
  return ~crc;
}

/* hash/crc32 slicing8Update (used by the generic path for len >= 16). */
uint32_t oracle_crc32_update(uint32_t crc, const uint8_t* p, size_t n) {
  ensure_tables();
  if (n >= 16) {
    crc = ~crc;
    while (n > 8) {
      crc ^= (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24;
      crc = ieee_tab[0][p[7]] ^ ieee_tab[1][p[6]] ^ ieee_tab[2][p[5]] ^ ieee_tab[3][p[4]] ^
            ieee_tab[4][crc >> 24] ^ ieee_tab[5][(crc >> 16) & 0xff] ^ ieee_tab[6][(crc >> 8) & 0xff] ^
            ieee_tab[7][crc & 0xff];
      p += 8;
      n -= 8;
    }
    crc = ~crc;
  }
  if (n == 0) return crc;
  return oracle_crc32_update_simple(crc, p, n);
}

/* ethernet/crc.go:19-21 */
uint32_t oracle_crc32(const uint8_t* p, size_t n) { return oracle_crc32_update(0, p, n); }

/* ethernet/crc.go:28-47 */
int64_t oracle_crc32_search(const uint8_t* p, size_t n, int64_t min_off) {
  if (min_off < 0) min_off = 0;                         /* :29-31 */
  if ((int64_t)n < min_off + 4) return -1;              /* :32-34 */
  uint32_t crc = oracle_crc32(p, (size_t)min_off);      /* :36 */
  for (int64_t off = min_off; off <= (int64_t)n - 4; off++) {  /* :38 */
    uint32_t got = (uint32_t)p[off] | (uint32_t)p[off + 1] << 8 | (uint32_t)p[off + 2] << 16 |
                   (uint32_t)p[off + 3] << 24;           /* :39 LittleEndian.Uint32 */
    if (crc == got) return off;                          /* :40-42 */
    crc = oracle_crc32_update(crc, p + off, 1);          /* :44 */
  }
  return -1;
}

/* crc.go:23-28 (uint32 wrap-around) */
uint32_t oracle_sum_write_even(uint32_t sum, const uint8_t* p, size_t n) {
  for (size_t i = 0; i + 1 < n; i += 2) sum += (uint32_t)p[i] << 8 | p[i + 1];
  return sum;
}

/* crc.go:17-21 */
uint16_t oracle_sum16(uint32_t sum) {
  sum = (sum & 0xffff) + (sum >> 16);
  return (uint16_t)~(uint16_t)(sum + (sum >> 16));
}

/* crc.go:52-59 */
uint16_t oracle_payload_sum16(uint32_t sum, const uint8_t* p, size_t n) {
  size_t odd = n & 1;
  sum = oracle_sum_write_even(sum, p, n - odd);
  if (odd) sum += (uint32_t)p[n - 1] << 8;
  return oracle_sum16(sum);
}

/* crc.go:65-71 */
uint16_t oracle_never_zero_sum(uint16_t s) { return s == 0 ? 0xffff : s; }

/* ---- batch helpers for the tests and the CPU baseline ----------------- */

typedef struct {
  const uint8_t* bytes;
  const uint64_t* off;
  uint64_t lo, hi;
  uint32_t* out;
} crc_job;

static void* crc_worker(void* arg) {
  crc_job* j = (crc_job*)arg;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    uint64_t s = j->off[i], e = j->off[i + 1];
    j->out[i] = e > s ? oracle_crc32(j->bytes + s, (size_t)(e - s)) : 0;
  }
  return NULL;
}

/* out[i] = CRC32(bytes[off[i]:off[i+1]]) with `threads` POSIX threads over
 * disjoint contiguous frame ranges (the "GOMAXPROCS goroutines each owning a
 * frame range" shape of BASELINE.md). */
int oracle_crc32_frames(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t* out,
                        int threads) {
  ensure_tables();
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t th[256];
  crc_job jobs[256];
  uint64_t per = (n + threads - 1) / threads;
  int started = 0;
  for (int t = 0; t < threads; t++) {
    jobs[t].bytes = bytes;
    jobs[t].off = off;
    jobs[t].lo = (uint64_t)t * per < n ? (uint64_t)t * per : n;
    jobs[t].hi = jobs[t].lo + per < n ? jobs[t].lo + per : n;
    jobs[t].out = out;
    if (threads == 1) {
      crc_worker(&jobs[t]);
    } else if (pthread_create(&th[t], NULL, crc_worker, &jobs[t]) == 0) {
      started++;
    } else {
      crc_worker(&jobs[t]);
      th[t] = 0;
    }
  }
  if (threads > 1)
    for (int t = 0; t < threads; t++)
      if (th[t]) pthread_join(th[t], NULL);
  (void)started;
  return 0;
}

/* out[i] = CRC791{seed[i]}.PayloadSum16(bytes[off[i] : off[i]+len[i]]) */
void oracle_sum16_segments(const uint8_t* bytes, const uint64_t* off, const uint32_t* len,
                           const uint32_t* seed, uint64_t n, uint16_t* out) {
  for (uint64_t i = 0; i < n; i++)
    out[i] = oracle_payload_sum16(seed ? seed[i] : 0, bytes + off[i], len[i]);
}
