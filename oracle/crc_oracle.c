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

/* ---- Go's amd64 fast path (CPU baseline only) -------------------------
 * hash/crc32 on amd64 (crc32_amd64.go archUpdateIEEE) folds inputs of >= 64
 * bytes with PCLMULQDQ (ieeeCLMUL in crc32_amd64.s: four 128-bit lanes folded
 * by 512 bits, then by 128, then a Barrett reduction) over the largest
 * multiple of 16 bytes, and finishes the 0..15 remaining bytes with
 * slicing-by-8.  Restated here with the published folding constants of the
 * reflected IEEE polynomial (x^(512+32), x^(512-32), x^(128+32), x^(128-32),
 * x^64 mod P, P', mu), so the CPU baseline runs the algorithm lneto's Go
 * build would; it is checked against the table form by tests/test_oracle.py. */
#if defined(__x86_64__)
#include <immintrin.h>
__attribute__((target("pclmul,sse4.1"))) static uint32_t ieee_clmul(uint32_t crc, const uint8_t* buf, size_t len) {
  /* len >= 64, len % 16 == 0; crc is the internal (inverted) register */
  const __m128i k1k2 = _mm_set_epi64x(0x01c6e41596LL, 0x0154442bd4LL);
  const __m128i k3k4 = _mm_set_epi64x(0x00ccaa009eLL, 0x01751997d0LL);
  const __m128i k5k0 = _mm_set_epi64x(0, 0x0163cd6124LL);
  const __m128i poly = _mm_set_epi64x(0x01f7011641LL, 0x01db710641LL);
  __m128i x1 = _mm_loadu_si128((const __m128i*)(buf + 0x00));
  __m128i x2 = _mm_loadu_si128((const __m128i*)(buf + 0x10));
  __m128i x3 = _mm_loadu_si128((const __m128i*)(buf + 0x20));
  __m128i x4 = _mm_loadu_si128((const __m128i*)(buf + 0x30));
  x1 = _mm_xor_si128(x1, _mm_cvtsi32_si128((int)crc));
  buf += 64, len -= 64;
  while (len >= 64) {
    __m128i x5 = _mm_clmulepi64_si128(x1, k1k2, 0x00), x6 = _mm_clmulepi64_si128(x2, k1k2, 0x00);
    __m128i x7 = _mm_clmulepi64_si128(x3, k1k2, 0x00), x8 = _mm_clmulepi64_si128(x4, k1k2, 0x00);
    x1 = _mm_clmulepi64_si128(x1, k1k2, 0x11), x2 = _mm_clmulepi64_si128(x2, k1k2, 0x11);
    x3 = _mm_clmulepi64_si128(x3, k1k2, 0x11), x4 = _mm_clmulepi64_si128(x4, k1k2, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x5), _mm_loadu_si128((const __m128i*)(buf + 0x00)));
    x2 = _mm_xor_si128(_mm_xor_si128(x2, x6), _mm_loadu_si128((const __m128i*)(buf + 0x10)));
    x3 = _mm_xor_si128(_mm_xor_si128(x3, x7), _mm_loadu_si128((const __m128i*)(buf + 0x20)));
    x4 = _mm_xor_si128(_mm_xor_si128(x4, x8), _mm_loadu_si128((const __m128i*)(buf + 0x30)));
    buf += 64, len -= 64;
  }
  __m128i x5;
  x5 = _mm_clmulepi64_si128(x1, k3k4, 0x00), x1 = _mm_clmulepi64_si128(x1, k3k4, 0x11);
  x1 = _mm_xor_si128(_mm_xor_si128(x1, x2), x5);
  x5 = _mm_clmulepi64_si128(x1, k3k4, 0x00), x1 = _mm_clmulepi64_si128(x1, k3k4, 0x11);
  x1 = _mm_xor_si128(_mm_xor_si128(x1, x3), x5);
  x5 = _mm_clmulepi64_si128(x1, k3k4, 0x00), x1 = _mm_clmulepi64_si128(x1, k3k4, 0x11);
  x1 = _mm_xor_si128(_mm_xor_si128(x1, x4), x5);
  while (len >= 16) {
    x2 = _mm_loadu_si128((const __m128i*)buf);
    x5 = _mm_clmulepi64_si128(x1, k3k4, 0x00), x1 = _mm_clmulepi64_si128(x1, k3k4, 0x11);
    x1 = _mm_xor_si128(_mm_xor_si128(x1, x2), x5);
    buf += 16, len -= 16;
  }
  /* 128 -> 64 bits */
  const __m128i m32 = _mm_setr_epi32(~0, 0, ~0, 0);
  x2 = _mm_clmulepi64_si128(x1, k3k4, 0x10);
  x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), x2);
  x2 = _mm_srli_si128(x1, 4);
  x1 = _mm_clmulepi64_si128(_mm_and_si128(x1, m32), k5k0, 0x00);
  x1 = _mm_xor_si128(x1, x2);
  /* Barrett reduction to 32 bits */
  x2 = _mm_clmulepi64_si128(_mm_and_si128(x1, m32), poly, 0x10);
  x2 = _mm_clmulepi64_si128(_mm_and_si128(x2, m32), poly, 0x00);
  x1 = _mm_xor_si128(x1, x2);
  return (uint32_t)_mm_extract_epi32(x1, 1);
}
static int clmul_ok(void) { return __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1"); }
#else
static uint32_t ieee_clmul(uint32_t crc, const uint8_t* buf, size_t len) { (void)buf; (void)len; return crc; }
static int clmul_ok(void) { return 0; }
#endif

int oracle_has_clmul(void) { return clmul_ok(); }

/* crc32.Update(crc, IEEETable, p) as Go's amd64 build runs it (archUpdateIEEE) */
uint32_t oracle_crc32_update_amd64(uint32_t crc, const uint8_t* p, size_t n) {
  if (n >= 64 && clmul_ok()) {
    const size_t done = n - (n & 15);
    crc = ~ieee_clmul(~crc, p, done);
    p += done, n -= done;
  }
  return n ? oracle_crc32_update(crc, p, n) : crc;
}

/* ---- batch helpers for the tests and the CPU baseline ----------------- */

typedef struct {
  const uint8_t* bytes;
  const uint64_t* off;
  uint64_t lo, hi;
  uint32_t* out;
  int amd64;
} crc_job;

static void* crc_worker(void* arg) {
  crc_job* j = (crc_job*)arg;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    uint64_t s = j->off[i], e = j->off[i + 1];
    j->out[i] = e <= s ? 0
                : j->amd64 ? oracle_crc32_update_amd64(0, j->bytes + s, (size_t)(e - s))
                           : oracle_crc32(j->bytes + s, (size_t)(e - s));
  }
  return NULL;
}

/* out[i] = CRC32(bytes[off[i]:off[i+1]]) with `threads` POSIX threads over
 * disjoint contiguous frame ranges (the "GOMAXPROCS goroutines each owning a
 * frame range" shape of BASELINE.md). */
static int crc32_frames(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t* out, int threads,
                        int amd64);
int oracle_crc32_frames(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t* out,
                        int threads) {
  return crc32_frames(bytes, off, n, out, threads, 0);
}
/* the same with Go's amd64 fast path (CPU baseline) */
int oracle_crc32_frames_amd64(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t* out,
                              int threads) {
  return crc32_frames(bytes, off, n, out, threads, 1);
}
static int crc32_frames(const uint8_t* bytes, const uint64_t* off, uint64_t n, uint32_t* out, int threads,
                        int amd64) {
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
    jobs[t].amd64 = amd64;
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
