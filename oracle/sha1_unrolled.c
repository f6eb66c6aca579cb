/*
 * oracle/sha1_unrolled.c -- TEST INFRASTRUCTURE ONLY (CPU comparator).
 *
 * A second CPU SHA-1, written in the shape the reference compiles: the fully
 * unrolled 80-round Transform of Crypto++ 5.2.1 (cpp/extern/crypto++/5.2.1/
 * sha.cpp:34-69: the R0..R4 round macros with the five working variables
 * renamed round to round, and the 16-word rolling schedule W[i & 15] of the
 * blk0/blk1 macros, sha.cpp:14-15), fed block by block as
 * IteratedHashBase::HashMultipleBlocks does on a little-endian host
 * (iterhash.cpp:73-84 -> iterhash.h:123-132: byte-reverse the 64 input bytes
 * into a 16-word buffer, then Transform), with the padding of PadLastBlock /
 * TruncatedFinal (iterhash.cpp:86-99, iterhash.h:106-121).
 *
 * Why a second one: oracle/sha1_oracle.c is the parity checker and is written
 * as a loop with a per-round branch on the round function, which gcc -O2 does
 * not unroll; it runs ~1.5x slower than the reference's macro form
 * ("What's missing" #3).  bench.py's cpu_baseline therefore times
 * THIS file as the reference-speed comparator, and keeps the loop form as a
 * secondary figure.  It is checked bit-exact against the checker oracle and
 * the KAT / tail goldens (tests/test_oracle.py).
 *
 * Portable C, -O2, no SHA-NI and no SIMD intrinsics: Crypto++ 5.2.1 has no SHA
 * extension code path.  Nothing in the product links or loads this file.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <stdlib.h>

#define ROL32(x, n) (((x) << (n)) | ((x) >> (32 - (n))))

/* round functions (sha.cpp:28-31): choose, parity, majority, parity */
#define F_CH(b, c, d) ((d) ^ ((b) & ((c) ^ (d))))
#define F_PAR(b, c, d) ((b) ^ (c) ^ (d))
#define F_MAJ(b, c, d) (((b) & (c)) | ((d) & ((b) | (c))))

/* schedule word t: the raw word for t < 16, else the rolling xor/rotate */
#define W_RAW(t) (w[t] = blk[t])
#define W_EXP(t) (w[(t) & 15] = ROL32(w[((t) + 13) & 15] ^ w[((t) + 8) & 15] ^ w[((t) + 2) & 15] ^ w[(t) & 15], 1))

/* one round: e += f(b,c,d) + W + K + rotl(a,5); b = rotl(b,30).  The caller
 * passes the five variables in rotated order, so no moves are generated. */
#define RND(F, K, WT, a, b, c, d, e)              \
  do {                                            \
    (e) += F((b), (c), (d)) + (WT) + (K) + ROL32((a), 5); \
    (b) = ROL32((b), 30);                         \
  } while (0)

#define K1 0x5A827999u
#define K2 0x6ED9EBA1u
#define K3 0x8F1BBCDCu
#define K4 0xCA62C1D6u

/* five rounds with the variables rotated one place each time */
#define FIVE(F, K, WM, t, a, b, c, d, e) \
  RND(F, K, WM(t), a, b, c, d, e);       \
  RND(F, K, WM((t) + 1), e, a, b, c, d); \
  RND(F, K, WM((t) + 2), d, e, a, b, c); \
  RND(F, K, WM((t) + 3), c, d, e, a, b); \
  RND(F, K, WM((t) + 4), b, c, d, e, a)

static void sha1_compress_unrolled(uint32_t st[5], const uint32_t blk[16]) {
  uint32_t w[16];
  uint32_t a = st[0], b = st[1], c = st[2], d = st[3], e = st[4];
  /* rounds 0..15 take the block's own words, 16..19 the first expanded ones */
  FIVE(F_CH, K1, W_RAW, 0, a, b, c, d, e);
  FIVE(F_CH, K1, W_RAW, 5, a, b, c, d, e);
  FIVE(F_CH, K1, W_RAW, 10, a, b, c, d, e);
  RND(F_CH, K1, W_RAW(15), a, b, c, d, e);
  RND(F_CH, K1, W_EXP(16), e, a, b, c, d);
  RND(F_CH, K1, W_EXP(17), d, e, a, b, c);
  RND(F_CH, K1, W_EXP(18), c, d, e, a, b);
  RND(F_CH, K1, W_EXP(19), b, c, d, e, a);
  FIVE(F_PAR, K2, W_EXP, 20, a, b, c, d, e);
  FIVE(F_PAR, K2, W_EXP, 25, a, b, c, d, e);
  FIVE(F_PAR, K2, W_EXP, 30, a, b, c, d, e);
  FIVE(F_PAR, K2, W_EXP, 35, a, b, c, d, e);
  FIVE(F_MAJ, K3, W_EXP, 40, a, b, c, d, e);
  FIVE(F_MAJ, K3, W_EXP, 45, a, b, c, d, e);
  FIVE(F_MAJ, K3, W_EXP, 50, a, b, c, d, e);
  FIVE(F_MAJ, K3, W_EXP, 55, a, b, c, d, e);
  FIVE(F_PAR, K4, W_EXP, 60, a, b, c, d, e);
  FIVE(F_PAR, K4, W_EXP, 65, a, b, c, d, e);
  FIVE(F_PAR, K4, W_EXP, 70, a, b, c, d, e);
  FIVE(F_PAR, K4, W_EXP, 75, a, b, c, d, e);
  st[0] += a;
  st[1] += b;
  st[2] += c;
  st[3] += d;
  st[4] += e;
}

static inline uint32_t be32(const uint8_t* p) {
  uint32_t v;
  memcpy(&v, p, 4);
  return __builtin_bswap32(v); /* little-endian host, iterhash.h:127-130 */
}

/* One-shot SHA-1 of len bytes (len < 2^32, as Base64Encode's U32 size). */
void unrolled_sha1(const uint8_t* data, uint32_t len, uint8_t out[20]) {
  uint32_t st[5] = {0x67452301u, 0xEFCDAB89u, 0x98BADCFEu, 0x10325476u, 0xC3D2E1F0u};
  uint32_t blk[16];
  uint32_t left = len;
  const uint8_t* p = data;
  while (left >= 64u) { /* HashMultipleBlocks: reverse into m_data, Transform */
    for (int i = 0; i < 16; ++i) blk[i] = be32(p + 4 * i);
    sha1_compress_unrolled(st, blk);
    p += 64;
    left -= 64;
  }
  uint8_t tail[128];
  memset(tail, 0, sizeof(tail));
  memcpy(tail, p, left);
  tail[left] = 0x80;
  unsigned nblk = left + 1u + 8u <= 64u ? 1u : 2u;
  uint64_t bits = (uint64_t)len << 3;
  uint8_t* lenp = tail + 64u * nblk - 8u;
  for (int i = 0; i < 8; ++i) lenp[i] = (uint8_t)(bits >> (56 - 8 * i));
  for (unsigned k = 0; k < nblk; ++k) {
    for (int i = 0; i < 16; ++i) blk[i] = be32(tail + 64u * k + 4 * i);
    sha1_compress_unrolled(st, blk);
  }
  for (int i = 0; i < 5; ++i) {
    out[4 * i + 0] = (uint8_t)(st[i] >> 24);
    out[4 * i + 1] = (uint8_t)(st[i] >> 16);
    out[4 * i + 2] = (uint8_t)(st[i] >> 8);
    out[4 * i + 3] = (uint8_t)st[i];
  }
}

typedef struct {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* sizes;
  uint64_t begin, end;
  uint8_t* digests;
} ubatch_job;

static void* ubatch_worker(void* arg) {
  ubatch_job* j = (ubatch_job*)arg;
  for (uint64_t i = j->begin; i < j->end; ++i)
    unrolled_sha1(j->base + j->offsets[i], j->sizes[i], j->digests + 20 * i);
  return NULL;
}

/* Chunk-parallel batch over (offset, size) descriptors on nthreads threads. */
void unrolled_sha1_batch(const uint8_t* base, const uint64_t* offsets, const uint32_t* sizes, uint64_t n,
                         uint8_t* digests, int nthreads) {
  if (nthreads <= 1 || n < 2) {
    ubatch_job j = {base, offsets, sizes, 0, n, digests};
    ubatch_worker(&j);
    return;
  }
  if ((uint64_t)nthreads > n) nthreads = (int)n;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  ubatch_job* jobs = (ubatch_job*)malloc(sizeof(ubatch_job) * (size_t)nthreads);
  int started = 0;
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].base = base;
    jobs[t].offsets = offsets;
    jobs[t].sizes = sizes;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)nthreads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
    jobs[t].digests = digests;
    if (pthread_create(&th[t], NULL, ubatch_worker, &jobs[t]) != 0) {
      ubatch_worker(&jobs[t]); /* run it here rather than drop the range */
      continue;
    }
    th[started++] = th[t];
  }
  for (int t = 0; t < started; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

/* Approximate core clock of the calling thread: a chain of dependent 64-bit
 * adds retires one per cycle on x86-64 cores, so iterations / seconds ~ Hz.
 * Returns the iteration count run; the caller times it. */
uint64_t unrolled_clock_probe(uint64_t iters) {
  uint64_t x = 1;
  for (uint64_t i = 0; i < iters; ++i) {
    x += i;
    __asm__ volatile("" : "+r"(x));
  }
  return x;
}

/* fread-inclusive single-thread encode of one file in Encoder::EncodeFile's
 * shape (Encoder.cpp:40-79: one chunk_size buffer, fread, hash, repeat), with
 * this file's hash.  Returns the chunk count, or -1 when the file cannot be
 * opened. */
int64_t unrolled_encode_file(const char* path, uint32_t chunk_size, uint8_t* digests, uint64_t max_chunks) {
  FILE* f = fopen(path, "rb");
  if (!f || chunk_size == 0) {
    if (f) fclose(f);
    return -1;
  }
  uint8_t* buf = (uint8_t*)malloc(chunk_size);
  if (!buf) {
    fclose(f);
    return -1;
  }
  int64_t idx = 0;
  for (;;) {
    size_t got = fread(buf, 1, chunk_size, f);
    if (got == 0) break;
    if ((uint64_t)idx < max_chunks) unrolled_sha1(buf, (uint32_t)got, digests + 20 * idx);
    ++idx;
  }
  free(buf);
  fclose(f);
  return idx;
}
