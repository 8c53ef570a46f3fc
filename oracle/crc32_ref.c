/*
 * oracle/crc32_ref.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the reference checksum path, used as the parity checker
 * (tests/, __graft_entry__.smoke(), bench.py's cpu_baseline leg). Nothing in
 * the product (ambry_amd/, include/) links or calls this file.
 *
 * What it restates (paths relative to linkedin/ambry):
 *   - ambry-utils/src/main/java/com/github/ambry/utils/Crc32.java
 *       :37-52   state held bit-inverted; reset() -> 0xffffffff; getValue() -> ~crc
 *       :55-98   update(byte[],off,len): slice-by-8 main loop (:58-74) + byte tail (:77-94)
 *       :146-148 update(int b)
 *       :154-179 tables T8_0..T8_7, T8_0 = reflected 0xEDB88320 table,
 *                T8_k[i] = (T8_{k-1}[i] >>> 8) ^ T8_0[T8_{k-1}[i] & 0xff]
 *   - java.util.zip.CRC32 (JDK, zlib-backed; third-party, not in the reference
 *     tree) is the same CRC-32/ISO-HDLC function; crc32_combine below restates
 *     zlib 1.2.11's published GF(2)-matrix combine (crc32.c, crc32_combine_),
 *     which has no Java counterpart in Ambry.
 *
 * Pinning: tests/test_oracle.py checks this file against the table fingerprint
 * parsed from Crc32.java's text (tests/golden/crc32_table_fingerprint.json),
 * the standard check value, zlib, and the golden vectors in tests/golden/.
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>
#include <zlib.h>

#define ORACLE_POLY 0xEDB88320u

static uint32_t T[8][256];
static int tables_ready = 0;
static pthread_once_t tables_once = PTHREAD_ONCE_INIT;

static void build_tables(void) {
  for (uint32_t i = 0; i < 256; ++i) {
    uint32_t c = i;
    for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ ORACLE_POLY : (c >> 1);
    T[0][i] = c;
  }
  for (int k = 1; k < 8; ++k)
    for (int i = 0; i < 256; ++i)
      T[k][i] = (T[k - 1][i] >> 8) ^ T[0][T[k - 1][i] & 0xff];
  tables_ready = 1;
}

static void ensure_tables(void) { pthread_once(&tables_once, build_tables); }

/* Export the 2048-word table in Crc32.java's layout (T8_0 first). */
void oracle_crc32_tables(uint32_t out[2048]) {
  ensure_tables();
  memcpy(out, T, sizeof(T));
}

/* ---- Crc32 object model (Crc32.java:37-52) ---- */
typedef struct { uint32_t crc; } oracle_crc32_t; /* holds the bit-flipped CRC */

void oracle_crc32_reset(oracle_crc32_t* s) { s->crc = 0xffffffffu; }
uint64_t oracle_crc32_get_value(const oracle_crc32_t* s) { return (uint64_t)(~s->crc) & 0xffffffffull; }

/* Crc32.update(byte[] b, int off, int len), Crc32.java:55-98. */
void oracle_crc32_update_bytes(oracle_crc32_t* s, const uint8_t* b, int64_t off, int64_t len) {
  ensure_tables();
  uint32_t c = s->crc;
  while (len > 7) {
    const uint32_t c0 = (b[off + 0] ^ c) & 0xff;
    const uint32_t c1 = (b[off + 1] ^ (c >>= 8)) & 0xff;
    const uint32_t c2 = (b[off + 2] ^ (c >>= 8)) & 0xff;
    const uint32_t c3 = (b[off + 3] ^ (c >>= 8)) & 0xff;
    c = (T[7][c0] ^ T[6][c1]) ^ (T[5][c2] ^ T[4][c3]);
    const uint32_t c4 = b[off + 4], c5 = b[off + 5], c6 = b[off + 6], c7 = b[off + 7];
    c ^= (T[3][c4] ^ T[2][c5]) ^ (T[1][c6] ^ T[0][c7]);
    off += 8;
    len -= 8;
  }
  while (len-- > 0) c = (c >> 8) ^ T[0][(c ^ b[off++]) & 0xff]; /* :77-94 tail */
  s->crc = c;
}

/* Crc32.update(int b), Crc32.java:146-148. */
void oracle_crc32_update_byte(oracle_crc32_t* s, int b) {
  ensure_tables();
  s->crc = (s->crc >> 8) ^ T[0][(s->crc ^ (uint32_t)b) & 0xff];
}

/* zlib-style value semantics: crc32(crc, p, n) == getValue() after seeding. */
uint32_t oracle_crc32(uint32_t crc, const uint8_t* p, uint64_t n) {
  oracle_crc32_t s = {~crc};
  while (n > 0) { /* Java's len is an int: feed in <=1 GiB pieces */
    int64_t piece = n > (1u << 30) ? (1 << 30) : (int64_t)n;
    oracle_crc32_update_bytes(&s, p, 0, piece);
    p += piece;
    n -= (uint64_t)piece;
  }
  return (uint32_t)oracle_crc32_get_value(&s);
}

/* Byte-at-a-time form (Crc32.java:146-148 applied per byte). */
uint32_t oracle_crc32_bytewise(uint32_t crc, const uint8_t* p, uint64_t n) {
  oracle_crc32_t s = {~crc};
  for (uint64_t i = 0; i < n; ++i) oracle_crc32_update_byte(&s, p[i]);
  return (uint32_t)oracle_crc32_get_value(&s);
}

/* ---- zlib 1.2.11 crc32_combine, restated (GF(2) 32x32 matrix squaring) ---- */
static uint32_t gf2_matrix_times(const uint32_t* mat, uint32_t vec) {
  uint32_t sum = 0;
  while (vec) {
    if (vec & 1) sum ^= *mat;
    vec >>= 1;
    mat++;
  }
  return sum;
}

static void gf2_matrix_square(uint32_t* square, const uint32_t* mat) {
  for (int n = 0; n < 32; n++) square[n] = gf2_matrix_times(mat, mat[n]);
}

uint32_t oracle_crc32_combine(uint32_t crc1, uint32_t crc2, uint64_t len2) {
  uint32_t even[32], odd[32];
  if (len2 == 0) return crc1;
  odd[0] = ORACLE_POLY; /* operator for one zero bit */
  uint32_t row = 1;
  for (int n = 1; n < 32; n++) {
    odd[n] = row;
    row <<= 1;
  }
  gf2_matrix_square(even, odd); /* two zero bits */
  gf2_matrix_square(odd, even); /* four zero bits */
  do {
    gf2_matrix_square(even, odd);
    if (len2 & 1) crc1 = gf2_matrix_times(even, crc1);
    len2 >>= 1;
    if (len2 == 0) break;
    gf2_matrix_square(odd, even);
    if (len2 & 1) crc1 = gf2_matrix_times(odd, crc1);
    len2 >>= 1;
  } while (len2 != 0);
  return crc1 ^ crc2;
}

/* ---- deterministic synthetic data (same generator as the GPU fill kernel) ----
 * Byte i of the stream is byte (i & 7) (little-endian) of
 * splitmix64_mix(seed + ((i >> 3) + 1) * 0x9E3779B97F4A7C15). */
static inline uint64_t splitmix_mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oracle_fill_splitmix(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t stream_offset) {
  for (uint64_t i = 0; i < nbytes; ++i) {
    uint64_t pos = stream_offset + i;
    uint64_t w = splitmix_mix(seed + ((pos >> 3) + 1) * 0x9E3779B97F4A7C15ull);
    dst[i] = (uint8_t)(w >> (8 * (pos & 7)));
  }
}

/* ---- batch over independent chunks, optionally threaded (cpu_baseline) ---- */
typedef struct {
  const uint8_t* base;
  const uint64_t* off;
  const uint64_t* len;
  const uint32_t* crc_in;
  uint32_t* out;
  size_t lo, hi;
} batch_job_t;

static void* batch_worker(void* arg) {
  batch_job_t* j = (batch_job_t*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->out[i] = oracle_crc32(j->crc_in ? j->crc_in[i] : 0u, j->base + j->off[i], j->len[i]);
  return NULL;
}

/* The same batch through the system zlib's crc32_z (1.2.11 here): the function
 * java.util.zip.CRC32 wraps, timed as the second CPU baseline SURVEY.md §8d asks for. */
static void* zlib_worker(void* arg) {
  batch_job_t* j = (batch_job_t*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->out[i] = (uint32_t)crc32_z(j->crc_in ? j->crc_in[i] : 0u, j->base + j->off[i], (z_size_t)j->len[i]);
  return NULL;
}

static int run_batch(void* (*worker)(void*), const uint8_t* base, const uint64_t* off, const uint64_t* len,
                     const uint32_t* crc_in, uint32_t* out, size_t n, int threads);

int oracle_zlib_batch(const uint8_t* base, const uint64_t* off, const uint64_t* len, const uint32_t* crc_in,
                      uint32_t* out, size_t n, int threads) {
  return run_batch(zlib_worker, base, off, len, crc_in, out, n, threads);
}

int oracle_crc32_batch(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                       const uint32_t* crc_in, uint32_t* out, size_t n, int threads) {
  ensure_tables();
  return run_batch(batch_worker, base, off, len, crc_in, out, n, threads);
}

static int run_batch(void* (*worker)(void*), const uint8_t* base, const uint64_t* off, const uint64_t* len,
                     const uint32_t* crc_in, uint32_t* out, size_t n, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 256) threads = 256;
  pthread_t tid[256];
  batch_job_t jobs[256];
  size_t per = (n + (size_t)threads - 1) / (size_t)threads;
  int started = 0;
  for (int t = 0; t < threads; ++t) {
    size_t lo = (size_t)t * per, hi = lo + per > n ? n : lo + per;
    if (lo >= hi) break;
    jobs[t] = (batch_job_t){base, off, len, crc_in, out, lo, hi};
    if (threads == 1) {
      worker(&jobs[t]);
    } else {
      if (pthread_create(&tid[t], NULL, worker, &jobs[t]) != 0) return -1;
      started++;
    }
  }
  for (int t = 0; t < started; ++t) pthread_join(tid[t], NULL);
  return 0;
}
