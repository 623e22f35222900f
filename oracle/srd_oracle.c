/*
 * srd_oracle.c -- CPU restatement of SIMD R Drive's open-time hot path.
 * TEST INFRASTRUCTURE ONLY (see srd_oracle.h for who may use it).
 *
 * Third-party arithmetic that the reference pulls from crates which are not
 * vendored in /root/reference:
 *   - xxhash-rust 0.8.15 (Cargo.lock:2578-2581), xxh3_64 with the default
 *     secret and seed 0.  Restated here from the published XXH3 spec
 *     (xxHash v0.8): len 0 / 1-3 / 4-8 / 9-16 / 17-128 / 129-240 / long.
 *   - crc32fast 1.5.0 (Cargo.lock:587-590): IEEE CRC-32 (reflected poly
 *     0xEDB88320, init/xorout 0xFFFFFFFF).  crc32fast's x86_64 path folds
 *     with PCLMULQDQ (fold-by-4 over 128-bit lanes, Barrett reduction); the
 *     same algorithm class is restated in crc32_pclmul() below, with a
 *     slice-by-8 table fallback.
 */
#define _GNU_SOURCE
#include "srd_oracle.h"

#include <pthread.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

/* ------------------------------------------------------------------ */
/* little-endian helpers                                               */
/* ------------------------------------------------------------------ */
static inline uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static inline uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static inline void wr64(uint8_t *p, uint64_t v) { memcpy(p, &v, 8); }
static inline void wr32(uint8_t *p, uint32_t v) { memcpy(p, &v, 4); }

static double now_s(void) {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (double)ts.tv_sec + 1e-9 * (double)ts.tv_nsec;
}

/* ------------------------------------------------------------------ */
/* XXH3-64 (xxhash-rust 0.8.15 xxh3_64; call sites compute_hash.rs:26, */
/* xxh3_build_hasher.rs:12)                                            */
/* ------------------------------------------------------------------ */
static const uint8_t kSecret[192] = {
    0xb8, 0xfe, 0x6c, 0x39, 0x23, 0xa4, 0x4b, 0xbe, 0x7c, 0x01, 0x81, 0x2c, 0xf7, 0x21, 0xad, 0x1c,
    0xde, 0xd4, 0x6d, 0xe9, 0x83, 0x90, 0x97, 0xdb, 0x72, 0x40, 0xa4, 0xa4, 0xb7, 0xb3, 0x67, 0x1f,
    0xcb, 0x79, 0xe6, 0x4e, 0xcc, 0xc0, 0xe5, 0x78, 0x82, 0x5a, 0xd0, 0x7d, 0xcc, 0xff, 0x72, 0x21,
    0xb8, 0x08, 0x46, 0x74, 0xf7, 0x43, 0x24, 0x8e, 0xe0, 0x35, 0x90, 0xe6, 0x81, 0x3a, 0x26, 0x4c,
    0x3c, 0x28, 0x52, 0xbb, 0x91, 0xc3, 0x00, 0xcb, 0x88, 0xd0, 0x65, 0x8b, 0x1b, 0x53, 0x2e, 0xa3,
    0x71, 0x64, 0x48, 0x97, 0xa2, 0x0d, 0xf9, 0x4e, 0x38, 0x19, 0xef, 0x46, 0xa9, 0xde, 0xac, 0xd8,
    0xa8, 0xfa, 0x76, 0x3f, 0xe3, 0x9c, 0x34, 0x3f, 0xf9, 0xdc, 0xbb, 0xc7, 0xc7, 0x0b, 0x4f, 0x1d,
    0x8a, 0x51, 0xe0, 0x4b, 0xcd, 0xb4, 0x59, 0x31, 0xc8, 0x9f, 0x7e, 0xc9, 0xd9, 0x78, 0x73, 0x64,
    0xea, 0xc5, 0xac, 0x83, 0x34, 0xd3, 0xeb, 0xc3, 0xc5, 0x81, 0xa0, 0xff, 0xfa, 0x13, 0x63, 0xeb,
    0x17, 0x0d, 0xdd, 0x51, 0xb7, 0xf0, 0xda, 0x49, 0xd3, 0x16, 0x55, 0x26, 0x29, 0xd4, 0x68, 0x9e,
    0x2b, 0x16, 0xbe, 0x58, 0x7d, 0x47, 0xa1, 0xfc, 0x8f, 0xf8, 0xb8, 0xd1, 0x7a, 0xd0, 0x31, 0xce,
    0x45, 0xcb, 0x3a, 0x8f, 0x95, 0x16, 0x04, 0x28, 0xaf, 0xd7, 0xfb, 0xca, 0xbb, 0x4b, 0x40, 0x7e,
};
#define P32_1 0x9E3779B1u
#define P32_2 0x85EBCA77u
#define P32_3 0xC2B2AE3Du
#define P64_1 0x9E3779B185EBCA87ull
#define P64_2 0xC2B2AE3D27D4EB4Full
#define P64_3 0x165667B19E3779F9ull
#define P64_4 0x85EBCA77C2B2AE63ull
#define P64_5 0x27D4EB2F165667C5ull
#define PMX_1 0x165667919E3779F9ull
#define PMX_2 0x9FB21C651E98DF25ull

static inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static inline uint64_t mul128_fold64(uint64_t a, uint64_t b) {
  __uint128_t p = (__uint128_t)a * b;
  return (uint64_t)p ^ (uint64_t)(p >> 64);
}
static inline uint64_t xxh64_avalanche(uint64_t h) {
  h ^= h >> 33; h *= P64_2; h ^= h >> 29; h *= P64_3; h ^= h >> 32; return h;
}
static inline uint64_t xxh3_avalanche(uint64_t h) {
  h ^= h >> 37; h *= PMX_1; h ^= h >> 32; return h;
}
static inline uint64_t xxh3_rrmxmx(uint64_t h, uint64_t len) {
  h ^= rotl64(h, 49) ^ rotl64(h, 24);
  h *= PMX_2;
  h ^= (h >> 35) + len;
  h *= PMX_2;
  return h ^ (h >> 28);
}
static inline uint64_t mix16B(const uint8_t *in, const uint8_t *sec) {
  return mul128_fold64(rd64(in) ^ rd64(sec), rd64(in + 8) ^ rd64(sec + 8));
}

uint64_t orc_xxh3_64(const void *data, size_t len) {
  const uint8_t *in = (const uint8_t *)data;
  const uint8_t *s = kSecret;
  if (len <= 16) {
    if (len > 8) {
      uint64_t bf1 = rd64(s + 24) ^ rd64(s + 32);
      uint64_t bf2 = rd64(s + 40) ^ rd64(s + 48);
      uint64_t lo = rd64(in) ^ bf1;
      uint64_t hi = rd64(in + len - 8) ^ bf2;
      uint64_t acc = len + __builtin_bswap64(lo) + hi + mul128_fold64(lo, hi);
      return xxh3_avalanche(acc);
    }
    if (len >= 4) {
      uint32_t i1 = rd32(in), i2 = rd32(in + len - 4);
      uint64_t bf = rd64(s + 8) ^ rd64(s + 16);
      uint64_t i64 = (uint64_t)i2 + ((uint64_t)i1 << 32);
      return xxh3_rrmxmx(i64 ^ bf, len);
    }
    if (len > 0) {
      uint8_t c1 = in[0], c2 = in[len >> 1], c3 = in[len - 1];
      uint32_t comb = ((uint32_t)c1 << 16) | ((uint32_t)c2 << 24) | (uint32_t)c3 | ((uint32_t)len << 8);
      uint64_t bf = (uint64_t)(rd32(s) ^ rd32(s + 4));
      return xxh64_avalanche((uint64_t)comb ^ bf);
    }
    return xxh64_avalanche(rd64(s + 56) ^ rd64(s + 64));
  }
  if (len <= 128) {
    uint64_t acc = len * P64_1;
    if (len > 32) {
      if (len > 64) {
        if (len > 96) {
          acc += mix16B(in + 48, s + 96);
          acc += mix16B(in + len - 64, s + 112);
        }
        acc += mix16B(in + 32, s + 64);
        acc += mix16B(in + len - 48, s + 80);
      }
      acc += mix16B(in + 16, s + 32);
      acc += mix16B(in + len - 32, s + 48);
    }
    acc += mix16B(in, s);
    acc += mix16B(in + len - 16, s + 16);
    return xxh3_avalanche(acc);
  }
  if (len <= 240) {
    uint64_t acc = len * P64_1, acc_end;
    unsigned nb = (unsigned)len / 16, i;
    for (i = 0; i < 8; i++) acc += mix16B(in + 16 * i, s + 16 * i);
    acc_end = mix16B(in + len - 16, s + 136 - 17);
    acc = xxh3_avalanche(acc);
    for (i = 8; i < nb; i++) acc_end += mix16B(in + 16 * i, s + 16 * (i - 8) + 3);
    return xxh3_avalanche(acc + acc_end);
  }
  /* long input: 64-byte stripes, 1024-byte blocks, scramble per block */
  uint64_t acc[8] = {P32_3, P64_1, P64_2, P64_3, P64_4, P32_2, P64_5, P32_1};
  const size_t nb_stripes_per_block = (192 - 64) / 8; /* 16 */
  const size_t block_len = 64 * nb_stripes_per_block; /* 1024 */
  size_t nb_blocks = (len - 1) / block_len, b, n, i;
#define ACC512(IN, SEC)                                         \
  for (i = 0; i < 8; i++) {                                     \
    uint64_t dv = rd64((IN) + 8 * i);                           \
    uint64_t dk = dv ^ rd64((SEC) + 8 * i);                     \
    acc[i ^ 1] += dv;                                           \
    acc[i] += (uint64_t)(uint32_t)dk * (dk >> 32);              \
  }
  for (b = 0; b < nb_blocks; b++) {
    for (n = 0; n < nb_stripes_per_block; n++) {
      ACC512(in + b * block_len + n * 64, s + n * 8);
    }
    for (i = 0; i < 8; i++) {
      uint64_t a = acc[i];
      a ^= a >> 47;
      a ^= rd64(s + 192 - 64 + 8 * i);
      a *= P32_1;
      acc[i] = a;
    }
  }
  {
    size_t nb_stripes = ((len - 1) - block_len * nb_blocks) / 64;
    for (n = 0; n < nb_stripes; n++) {
      ACC512(in + nb_blocks * block_len + n * 64, s + n * 8);
    }
    ACC512(in + len - 64, s + 192 - 64 - 7);
  }
#undef ACC512
  uint64_t r = len * P64_1;
  for (i = 0; i < 4; i++)
    r += mul128_fold64(acc[2 * i] ^ rd64(s + 11 + 16 * i), acc[2 * i + 1] ^ rd64(s + 11 + 16 * i + 8));
  return xxh3_avalanche(r);
}

/* compute_hash_batch (compute_hash.rs:64-77): a plain loop of xxh3_64. */
void orc_xxh3_64_batch(const uint8_t *buf, const uint64_t *offs,
                       const uint64_t *lens, uint64_t n, uint64_t *out) {
  for (uint64_t i = 0; i < n; i++) out[i] = orc_xxh3_64(buf + offs[i], lens[i]);
}

/* ------------------------------------------------------------------ */
/* CRC-32 / IEEE (crc32fast 1.5.0; call site compute_checksum.rs:15-20, */
/* entry_handle.rs:260-275)                                             */
/* ------------------------------------------------------------------ */
static uint32_t crc_tab[8][256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
    crc_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; i++)
    for (int t = 1; t < 8; t++)
      crc_tab[t][i] = (crc_tab[t - 1][i] >> 8) ^ crc_tab[0][crc_tab[t - 1][i] & 0xff];
}

/* raw register update (no init / xorout) */
static uint32_t crc_slice8(uint32_t s, const uint8_t *p, size_t n) {
  while (n >= 8) {
    uint32_t a = rd32(p) ^ s, b = rd32(p + 4);
    s = crc_tab[7][a & 0xff] ^ crc_tab[6][(a >> 8) & 0xff] ^ crc_tab[5][(a >> 16) & 0xff] ^
        crc_tab[4][a >> 24] ^ crc_tab[3][b & 0xff] ^ crc_tab[2][(b >> 8) & 0xff] ^
        crc_tab[1][(b >> 16) & 0xff] ^ crc_tab[0][b >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) s = crc_tab[0][(s ^ *p++) & 0xff] ^ (s >> 8);
  return s;
}

#if defined(__x86_64__)
#include <immintrin.h>
/* Fold constants for the reflected CRC-32 polynomial (the values used by the
 * Intel "Fast CRC Computation Using PCLMULQDQ" method, as in crc32fast). */
#define K1 0x154442bd4ll
#define K2 0x1c6e41596ll
#define K3 0x1751997d0ll
#define K4 0x0ccaa009ell
#define K5 0x163cd6124ll
#define PX 0x1DB710641ll
#define UP 0x1F7011641ll

__attribute__((target("pclmul,sse4.1"))) static inline __m128i
fold128(__m128i a, __m128i b, __m128i k) {
  return _mm_xor_si128(_mm_xor_si128(b, _mm_clmulepi64_si128(a, k, 0x00)),
                       _mm_clmulepi64_si128(a, k, 0x11));
}

/* s = raw register (i.e. ~crc); returns raw register. */
__attribute__((target("pclmul,sse4.1"))) static uint32_t
crc_pclmul(uint32_t s, const uint8_t *p, size_t n) {
  if (n < 128) return crc_slice8(s, p, n);
  __m128i x3 = _mm_loadu_si128((const __m128i *)(p + 0));
  __m128i x2 = _mm_loadu_si128((const __m128i *)(p + 16));
  __m128i x1 = _mm_loadu_si128((const __m128i *)(p + 32));
  __m128i x0 = _mm_loadu_si128((const __m128i *)(p + 48));
  p += 64;
  n -= 64;
  x3 = _mm_xor_si128(x3, _mm_cvtsi32_si128((int)s));
  const __m128i k12 = _mm_set_epi64x(K2, K1);
  while (n >= 64) {
    x3 = fold128(x3, _mm_loadu_si128((const __m128i *)(p + 0)), k12);
    x2 = fold128(x2, _mm_loadu_si128((const __m128i *)(p + 16)), k12);
    x1 = fold128(x1, _mm_loadu_si128((const __m128i *)(p + 32)), k12);
    x0 = fold128(x0, _mm_loadu_si128((const __m128i *)(p + 48)), k12);
    p += 64;
    n -= 64;
  }
  const __m128i k34 = _mm_set_epi64x(K4, K3);
  __m128i x = fold128(x3, x2, k34);
  x = fold128(x, x1, k34);
  x = fold128(x, x0, k34);
  while (n >= 16) {
    x = fold128(x, _mm_loadu_si128((const __m128i *)p), k34);
    p += 16;
    n -= 16;
  }
  /* 128 -> 64 bits */
  x = _mm_xor_si128(_mm_clmulepi64_si128(x, k34, 0x10), _mm_srli_si128(x, 8));
  x = _mm_xor_si128(
      _mm_clmulepi64_si128(_mm_and_si128(x, _mm_set_epi32(0, 0, 0, ~0)), _mm_set_epi64x(0, K5), 0x00),
      _mm_srli_si128(x, 4));
  /* Barrett reduction, bit-reflected variant */
  const __m128i pu = _mm_set_epi64x(UP, PX);
  __m128i t1 = _mm_clmulepi64_si128(_mm_and_si128(x, _mm_set_epi32(0, 0, 0, ~0)), pu, 0x10);
  __m128i t2 = _mm_clmulepi64_si128(_mm_and_si128(t1, _mm_set_epi32(0, 0, 0, ~0)), pu, 0x00);
  uint32_t c = (uint32_t)_mm_extract_epi32(_mm_xor_si128(x, t2), 1);
  return n ? crc_slice8(c, p, n) : c;
}
#endif

static int g_pclmul = -1;
int orc_has_pclmul(void) {
#if defined(__x86_64__)
  if (g_pclmul < 0) {
    __builtin_cpu_init();
    g_pclmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
  }
  return g_pclmul;
#else
  return 0;
#endif
}

uint32_t orc_crc32_update(uint32_t crc, const void *data, size_t len) {
  pthread_once(&crc_once, crc_init);
  uint32_t s = ~crc;
#if defined(__x86_64__)
  if (orc_has_pclmul()) return ~crc_pclmul(s, (const uint8_t *)data, len);
#endif
  return ~crc_slice8(s, (const uint8_t *)data, len);
}
uint32_t orc_crc32(const void *data, size_t len) { return orc_crc32_update(0, data, len); }

/* compute_checksum (compute_checksum.rs:15-20) of n byte ranges of buf,
 * buf[starts[i], starts[i] + lens[i]), on `threads` threads (contiguous
 * blocks of ranges): the independent checker of the GPU's crc_computed at
 * full C3 size (tests/test_gpu_scale.py) */
typedef struct {
  const uint8_t *buf;
  const uint64_t *starts, *lens;
  uint32_t *out;
  uint64_t lo, hi;
} crc_range_job;
static void *crc_range_worker(void *p) {
  crc_range_job *j = (crc_range_job *)p;
  for (uint64_t i = j->lo; i < j->hi; i++) j->out[i] = orc_crc32(j->buf + j->starts[i], (size_t)j->lens[i]);
  return NULL;
}
void orc_crc32_ranges(const uint8_t *buf, const uint64_t *starts, const uint64_t *lens, uint64_t n,
                      uint32_t *out, int threads) {
  if (threads < 1) threads = 1;
  if (threads > 64) threads = 64;
  pthread_t th[64];
  crc_range_job jobs[64];
  for (int t = 0; t < threads; t++) {
    jobs[t] = (crc_range_job){buf, starts, lens, out, n * (uint64_t)t / threads, n * (uint64_t)(t + 1) / threads};
    pthread_create(&th[t], NULL, crc_range_worker, &jobs[t]);
  }
  for (int t = 0; t < threads; t++) pthread_join(th[t], NULL);
}
uint32_t orc_crc32_table(const void *data, size_t len) {
  pthread_once(&crc_once, crc_init);
  return ~crc_slice8(~0u, (const uint8_t *)data, len);
}

/* EntryHandle::is_valid_checksum (entry_handle.rs:260-275): 4 KiB chunks */
static uint32_t crc_chunked(const uint8_t *p, uint64_t n) {
  uint32_t c = 0;
  uint64_t off = 0;
  while (off < n) {
    uint64_t e = off + 4096 < n ? off + 4096 : n;
    c = orc_crc32_update(c, p + off, e - off);
    off = e;
  }
  return c;
}

/* ------------------------------------------------------------------ */
/* format + writer                                                     */
/* ------------------------------------------------------------------ */
/* prepad_len: data_store.rs:670-673 (a = PAYLOAD_ALIGNMENT = 64) */
uint64_t orc_prepad_len(uint64_t offset) { return (64 - (offset % 64)) & 63; }

/* batch_write_with_key_hashes: data_store.rs:847-939 */
int64_t orc_write_entries(uint8_t *out, uint64_t cap, uint64_t tail,
                          const uint64_t *key_hashes, const uint8_t *payload_buf,
                          const uint64_t *payload_offs,
                          const uint64_t *payload_lens, uint64_t n,
                          int allow_null_bytes) {
  for (uint64_t i = 0; i < n; i++) {
    const uint8_t *pl = payload_buf + payload_offs[i];
    uint64_t len = payload_lens[i];
    if (len == 1 && pl[0] == 0) { /* tombstone: :864-895 */
      if (!allow_null_bytes) return -1;
      if (tail + 21 > cap) return -2;
      uint32_t c = orc_crc32(pl, 1);
      out[tail] = 0;
      wr64(out + tail + 1, key_hashes[i]);
      wr64(out + tail + 9, tail);
      wr32(out + tail + 17, c);
      tail += 21;
      continue;
    }
    if (len == 0) return -1; /* :900-905 */
    uint64_t link = tail, pad = orc_prepad_len(tail);
    if (tail + pad + len + 20 > cap) return -2;
    memset(out + tail, 0, pad);
    tail += pad;
    uint32_t c = orc_crc32(pl, len);
    memcpy(out + tail, pl, len);
    wr64(out + tail + len, key_hashes[i]);
    wr64(out + tail + len + 8, link);
    wr32(out + tail + len + 16, c);
    tail += len + 20;
  }
  return (int64_t)tail;
}

/* Counter-mode splitmix64: word j of entry i's payload (little endian). */
uint64_t orc_synth_word(uint64_t seed, uint64_t entry, uint64_t word) {
  uint64_t z = seed + ((entry << 32) + word + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t orc_synth_store(uint8_t *out, uint64_t n_entries, uint64_t fixed_len,
                         const uint64_t *lens, uint64_t seed) {
  uint64_t tail = 0;
  char key[64];
  for (uint64_t i = 0; i < n_entries; i++) {
    uint64_t len = lens ? lens[i] : fixed_len;
    uint64_t pad = orc_prepad_len(tail);
    if (out) {
      memset(out + tail, 0, pad);
      uint8_t *pl = out + tail + pad;
      for (uint64_t w = 0; w * 8 < len; w++) {
        uint64_t v = orc_synth_word(seed, i, w);
        uint64_t k = len - w * 8 < 8 ? len - w * 8 : 8;
        memcpy(pl + w * 8, &v, k);
      }
      int kl = snprintf(key, sizeof key, "bench-key-%llu", (unsigned long long)i);
      uint64_t kh = orc_xxh3_64(key, (size_t)kl);
      uint32_t c = orc_crc32(pl, len);
      wr64(pl + len, kh);
      wr64(pl + len + 8, tail);
      wr32(pl + len + 16, c);
    }
    tail += pad + len + 20;
  }
  return tail;
}

/* ------------------------------------------------------------------ */
/* recover_valid_chain: data_store.rs:383-482 (literal restatement,     */
/* release-mode wrapping u64 arithmetic)                               */
/* ------------------------------------------------------------------ */
uint64_t orc_recover_valid_chain(const uint8_t *mmap, uint64_t file_len) {
  const uint64_t MS = 20;
  if (file_len < MS) return 0; /* :384-386 */
  uint64_t cursor = file_len;
  while (cursor >= MS) { /* :390 */
    uint64_t metadata_offset = cursor - MS;
    const uint8_t *mb = mmap + metadata_offset;
    uint64_t prev_tail = rd64(mb + 8);
    uint64_t derived_start = prev_tail + orc_prepad_len(prev_tail); /* wrapping */
    uint64_t entry_end = metadata_offset;
    uint64_t entry_start;
    if (entry_end > prev_tail && entry_end - prev_tail == 1 && mmap[prev_tail] == 0)
      entry_start = prev_tail; /* :404-408 tombstone */
    else
      entry_start = derived_start;
    if (entry_start >= metadata_offset) { /* :418-421 */
      cursor -= 1;
      continue;
    }
    int chain_valid = 1;
    uint64_t back_cursor = prev_tail;
    uint64_t total_size = (metadata_offset - entry_start) + MS;
    while (back_cursor != 0) { /* :428-471 */
      if (back_cursor < MS) { chain_valid = 0; break; }
      uint64_t pmo = back_cursor - MS;
      if (pmo + MS > file_len) { chain_valid = 0; break; }
      uint64_t ppt = rd64(mmap + pmo + 8);
      uint64_t pes;
      if (pmo > ppt && pmo - ppt == 1 && mmap[ppt] == 0)
        pes = ppt;
      else
        pes = ppt + orc_prepad_len(ppt);
      if (pes >= pmo) { chain_valid = 0; break; }
      uint64_t entry_size = pmo > pes ? pmo - pes : 0;
      total_size += entry_size + MS;
      if (ppt >= pmo) { chain_valid = 0; break; }
      back_cursor = ppt;
    }
    if (chain_valid && back_cursor == 0 && total_size <= file_len) /* :473 */
      return metadata_offset + MS;
    cursor -= 1;
  }
  return 0;
}

/* ------------------------------------------------------------------ */
/* chain enumeration (the walk recover/build perform)                  */
/* ------------------------------------------------------------------ */
static void fill_entry(const uint8_t *mmap, uint64_t mo, orc_entry *e, int crc) {
  uint64_t p = rd64(mmap + mo + 8);
  e->meta_off = mo;
  e->key_hash = rd64(mmap + mo);
  e->prev_offset = p;
  e->crc_stored = rd32(mmap + mo + 16);
  /* start derivation: entry_iterator.rs:83-95 */
  if (mo > p && mo - p == 1 && mmap[p] == 0) {
    e->payload_start = p;
    e->is_tombstone = 1;
  } else {
    e->payload_start = p + orc_prepad_len(p);
    e->is_tombstone = 0;
  }
  e->payload_len = mo - e->payload_start;
  if (crc) {
    e->crc_computed = crc_chunked(mmap + e->payload_start, e->payload_len);
    e->crc_ok = e->crc_computed == e->crc_stored;
  } else {
    e->crc_computed = 0;
    e->crc_ok = 0;
  }
}

uint64_t orc_chain(const uint8_t *mmap, uint64_t tail, orc_entry *out,
                   uint64_t cap, int compute_crc) {
  uint64_t n = 0, cur = tail;
  while (cur >= 20) {
    uint64_t mo = cur - 20;
    n++;
    uint64_t p = rd64(mmap + mo + 8);
    if (p == 0) break;
    cur = p;
  }
  /* second pass, fill in file order */
  uint64_t i = n;
  cur = tail;
  while (cur >= 20 && i > 0) {
    uint64_t mo = cur - 20;
    i--;
    if (i < cap) fill_entry(mmap, mo, &out[i], compute_crc);
    uint64_t p = rd64(mmap + mo + 8);
    if (p == 0) break;
    cur = p;
  }
  return n;
}

/* ------------------------------------------------------------------ */
/* XXH3-hashed open-addressing set/map (the Xxh3BuildHasher HashMap /   */
/* HashSet of key_indexer.rs:99-100): hash = xxh3_64(le8(key)).          */
/* ------------------------------------------------------------------ */
typedef struct {
  uint64_t *keys;
  uint64_t *vals;
  uint8_t *used;
  uint64_t cap, n;
} xmap;

static uint64_t hkey(uint64_t k) { return orc_xxh3_64(&k, 8); }
static void xmap_init(xmap *m, uint64_t cap) {
  m->cap = cap;
  m->n = 0;
  m->keys = (uint64_t *)malloc(cap * 8);
  m->vals = (uint64_t *)malloc(cap * 8);
  m->used = (uint8_t *)calloc(cap, 1);
}
static void xmap_free(xmap *m) { free(m->keys); free(m->vals); free(m->used); }
static int64_t xmap_find(const xmap *m, uint64_t k) {
  uint64_t i = hkey(k) & (m->cap - 1);
  while (m->used[i]) {
    if (m->keys[i] == k) return (int64_t)i;
    i = (i + 1) & (m->cap - 1);
  }
  return -1;
}
static void xmap_put(xmap *m, uint64_t k, uint64_t v);
static void xmap_grow(xmap *m) {
  xmap nm;
  xmap_init(&nm, m->cap * 2);
  for (uint64_t i = 0; i < m->cap; i++)
    if (m->used[i]) xmap_put(&nm, m->keys[i], m->vals[i]);
  xmap_free(m);
  *m = nm;
}
static void xmap_put(xmap *m, uint64_t k, uint64_t v) {
  if ((m->n + 1) * 8 > m->cap * 7) xmap_grow(m);
  uint64_t i = hkey(k) & (m->cap - 1);
  while (m->used[i]) {
    if (m->keys[i] == k) { m->vals[i] = v; return; }
    i = (i + 1) & (m->cap - 1);
  }
  m->used[i] = 1;
  m->keys[i] = k;
  m->vals[i] = v;
  m->n++;
}

/* KeyIndexer::build: key_indexer.rs:98-124; tag/pack :64-93 */
static void key_indexer_build(const uint8_t *mmap, uint64_t tail, xmap *index) {
  xmap seen;
  xmap_init(&seen, 16);
  xmap_init(index, 16);
  uint64_t cursor = tail;
  while (cursor >= 20) {
    uint64_t mo = cursor - 20;
    uint64_t kh = rd64(mmap + mo), p = rd64(mmap + mo + 8);
    if (xmap_find(&seen, kh) >= 0) { cursor = p; continue; }
    xmap_put(&seen, kh, 1);
    uint64_t tag = kh >> 48;
    xmap_put(index, kh, (tag << 48) | mo);
    if (p == 0) break;
    cursor = p;
  }
  xmap_free(&seen);
}

static int cmp_u64pair(const void *a, const void *b) {
  const uint64_t *x = (const uint64_t *)a, *y = (const uint64_t *)b;
  return x[0] < y[0] ? -1 : x[0] > y[0];
}

uint64_t orc_key_indexer_build(const uint8_t *mmap, uint64_t tail,
                               uint64_t *keys_out, uint64_t *packed_out,
                               uint64_t cap) {
  xmap idx;
  key_indexer_build(mmap, tail, &idx);
  uint64_t n = idx.n, j = 0;
  uint64_t *pairs = (uint64_t *)malloc((n ? n : 1) * 16);
  for (uint64_t i = 0; i < idx.cap; i++)
    if (idx.used[i]) { pairs[2 * j] = idx.keys[i]; pairs[2 * j + 1] = idx.vals[i]; j++; }
  qsort(pairs, n, 16, cmp_u64pair);
  for (uint64_t i = 0; i < n && i < cap; i++) {
    keys_out[i] = pairs[2 * i];
    packed_out[i] = pairs[2 * i + 1];
  }
  free(pairs);
  xmap_free(&idx);
  return n;
}

/* ------------------------------------------------------------------ */
/* timed CPU baseline                                                  */
/* ------------------------------------------------------------------ */
typedef struct {
  const uint8_t *mmap;
  const uint64_t *mo;
  uint64_t lo, hi;
  uint64_t bad, x;
} crc_job;

static void *crc_worker(void *arg) {
  crc_job *j = (crc_job *)arg;
  for (uint64_t i = j->lo; i < j->hi; i++) {
    orc_entry e;
    fill_entry(j->mmap, j->mo[i], &e, 1);
    j->bad += !e.crc_ok;
    j->x ^= e.crc_computed;
  }
  return NULL;
}

int orc_validate_index(const uint8_t *mmap, uint64_t file_len, int threads,
                       orc_stats *st) {
  memset(st, 0, sizeof *st);
  double t0 = now_s();
  uint64_t tail = orc_recover_valid_chain(mmap, file_len);
  double t1 = now_s();
  xmap idx;
  key_indexer_build(mmap, tail, &idx);
  double t2 = now_s();
  st->final_len = tail;
  st->n_index = idx.n;
  for (uint64_t i = 0; i < idx.cap; i++)
    if (idx.used[i]) st->index_xor ^= idx.keys[i] ^ (idx.vals[i] * 31);
  xmap_free(&idx);
  /* is_valid_checksum over every chain entry */
  if (threads <= 1) {
    uint64_t cur = tail;
    while (cur >= 20) {
      orc_entry e;
      fill_entry(mmap, cur - 20, &e, 1);
      st->n_chain++;
      st->n_crc_bad += !e.crc_ok;
      st->crc_xor ^= e.crc_computed;
      if (e.prev_offset == 0) break;
      cur = e.prev_offset;
    }
  } else {
    uint64_t n = 0, cur = tail, capn = 1024;
    uint64_t *mo = (uint64_t *)malloc(capn * 8);
    while (cur >= 20) {
      if (n == capn) { capn *= 2; mo = (uint64_t *)realloc(mo, capn * 8); }
      mo[n++] = cur - 20;
      uint64_t p = rd64(mmap + cur - 20 + 8);
      if (p == 0) break;
      cur = p;
    }
    pthread_t th[256];
    crc_job jobs[256];
    if (threads > 256) threads = 256;
    for (int t = 0; t < threads; t++) {
      jobs[t].mmap = mmap; jobs[t].mo = mo;
      jobs[t].lo = n * (uint64_t)t / threads;
      jobs[t].hi = n * (uint64_t)(t + 1) / threads;
      jobs[t].bad = 0; jobs[t].x = 0;
      pthread_create(&th[t], NULL, crc_worker, &jobs[t]);
    }
    for (int t = 0; t < threads; t++) {
      pthread_join(th[t], NULL);
      st->n_crc_bad += jobs[t].bad;
      st->crc_xor ^= jobs[t].x;
    }
    st->n_chain = n;
    free(mo);
  }
  double t3 = now_s();
  st->t_recover_s = t1 - t0;
  st->t_index_s = t2 - t1;
  st->t_crc_s = t3 - t2;
  return 0;
}
