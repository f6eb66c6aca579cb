/*
 * oracle/sha1_oracle.c -- TEST INFRASTRUCTURE ONLY.
 *
 * CPU restatement of the bitflood chunk-hash path, used as the parity checker
 * for the MI355X kernels and as the `cpu_baseline` leg of bench.py.  Nothing in
 * the product (liblbfhash.so, libbitflood.so, the bitflood_amd package) links,
 * loads or calls this file; only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg do.
 *
 * Parity anchors (all paths relative to /root/reference):
 *   - SHA-1 compression: cpp/extern/crypto++/5.2.1/sha.cpp:14-79
 *       (InitState :19-26, f1..f4 :28-31, R0..R4 :34-38, Transform :40-79)
 *   - Merkle-Damgard framing: cpp/extern/crypto++/5.2.1/iterhash.cpp:9-63
 *       (Update), :73-84 (HashMultipleBlocks), :86-99 (PadLastBlock);
 *       iterhash.h:30-31 (bit count), :106-121 (TruncatedFinal),
 *       :123-132 (HashBlock: byte reverse on little-endian hosts)
 *   - digest -> 27-char base64: cpp/extern/crypto++/5.2.1/basecode.cpp:39-104
 *       driven by cpp/src/Encoder.cpp:104-120 (alphabet, no padding byte)
 *   - chunking loop: cpp/src/Encoder.cpp:37-79 (fixed-size chunks, short tail)
 *
 * Pinned by: the Crypto++ SHA-1 known-answer tests
 * (cpp/extern/crypto++/5.2.1/TestVectors/sha.txt:1-11, validat3.cpp:171-176)
 * and by golden fixtures generated independently with Python hashlib/base64
 * (tests/golden/make_golden.py).  Building or running the reference itself
 * was denied in the survey session; this restatement is the
 * CPU comparator ("kind": "port").
 *
 * Build: see oracle/Makefile (gcc -O2, portable C, no SHA-NI: the reference is
 * portable C++ and Crypto++ 5.2.1 has no SHA extension path).
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

/* ------------------------------------------------------------------------ */
/* SHA-1 state, mirroring IteratedHashBase<word32>: m_digest, m_data and the  */
/* split 32-bit byte counter m_countLo/m_countHi (iterhash.h:38-42).          */
/* ------------------------------------------------------------------------ */
typedef struct {
  uint32_t digest[5];
  uint32_t data[16];
  uint32_t count_lo;
  uint32_t count_hi;
} oracle_sha1_ctx;

static uint32_t rotl32(uint32_t x, unsigned n) { return (x << n) | (x >> (32u - n)); }

static uint32_t byte_reverse(uint32_t v) {
  return (v >> 24) | ((v >> 8) & 0x0000ff00u) | ((v << 8) & 0x00ff0000u) | (v << 24);
}

/* sha.cpp:19-26 */
static void sha1_init_state(uint32_t* s) {
  s[0] = 0x67452301u;
  s[1] = 0xEFCDAB89u;
  s[2] = 0x98BADCFEu;
  s[3] = 0x10325476u;
  s[4] = 0xC3D2E1F0u;
}

/* sha.cpp:40-79.  The schedule is the 16-word rolling window of the blk0/blk1
 * macros (sha.cpp:14-15); the round functions are f1 (choose), f2/f4 (parity)
 * and f3 (majority) with the four round constants of R0..R4 (sha.cpp:28-38).
 * Written as a loop over the 80 rounds with the (a,b,c,d,e) rotation made
 * explicit, which is exactly the register renaming of the unrolled macros. */
static void sha1_transform(uint32_t* state, const uint32_t* block) {
  uint32_t w[16];
  uint32_t a = state[0], b = state[1], c = state[2], d = state[3], e = state[4];
  for (int i = 0; i < 80; ++i) {
    uint32_t wi;
    if (i < 16) {
      wi = w[i] = block[i];                                   /* blk0 */
    } else {
      wi = w[i & 15] = rotl32(w[(i + 13) & 15] ^ w[(i + 8) & 15] ^
                              w[(i + 2) & 15] ^ w[i & 15], 1); /* blk1 */
    }
    uint32_t f, k;
    if (i < 20)      { f = d ^ (b & (c ^ d));        k = 0x5A827999u; } /* f1 */
    else if (i < 40) { f = b ^ c ^ d;                k = 0x6ED9EBA1u; } /* f2 */
    else if (i < 60) { f = (b & c) | (d & (b | c));  k = 0x8F1BBCDCu; } /* f3 */
    else             { f = b ^ c ^ d;                k = 0xCA62C1D6u; } /* f4 */
    uint32_t t = e + f + wi + k + rotl32(a, 5);
    e = d;
    d = c;
    c = rotl32(b, 30);
    b = a;
    a = t;
  }
  state[0] += a;
  state[1] += b;
  state[2] += c;
  state[3] += d;
  state[4] += e;
}

/* iterhash.h:123-132: on a little-endian host each 64-byte block is byte
 * reversed into big-endian words before Transform. */
static void sha1_hash_block(oracle_sha1_ctx* c, const uint8_t* bytes) {
  uint32_t blk[16];
  memcpy(blk, bytes, 64);
  for (int i = 0; i < 16; ++i) blk[i] = byte_reverse(blk[i]);
  sha1_transform(c->digest, blk);
}

void oracle_sha1_init(oracle_sha1_ctx* c) {
  sha1_init_state(c->digest);
  memset(c->data, 0, sizeof(c->data));
  c->count_lo = 0;
  c->count_hi = 0;
}

/* iterhash.cpp:9-63.  Same counter arithmetic (carry into count_hi, length
 * is a 32-bit unsigned as in the reference signature), same left-over
 * handling: partial data is parked in `data` until a block fills. */
void oracle_sha1_update(oracle_sha1_ctx* c, const uint8_t* input, uint32_t len) {
  uint32_t tmp = c->count_lo;
  if ((c->count_lo = tmp + len) < tmp) c->count_hi++;
  /* SafeRightShift<32>(len) == 0 for a 32-bit len (iterhash.cpp:14) */
  uint32_t num = tmp & 63u;
  uint8_t* buf = (uint8_t*)c->data;
  if (num != 0) {
    if (num + len >= 64u) {
      memcpy(buf + num, input, 64u - num);
      sha1_hash_block(c, buf);
      input += 64u - num;
      len -= 64u - num;
    } else {
      memcpy(buf + num, input, len);
      return;
    }
  }
  while (len >= 64u) { /* HashMultipleBlocks, iterhash.cpp:73-84 */
    sha1_hash_block(c, input);
    input += 64;
    len -= 64;
  }
  memcpy(buf, input, len);
}

/* iterhash.h:106-121 + iterhash.cpp:86-99 (PadLastBlock(56, 0x80)) */
void oracle_sha1_final(oracle_sha1_ctx* c, uint8_t out[20]) {
  uint8_t* buf = (uint8_t*)c->data;
  uint32_t num = c->count_lo & 63u;
  buf[num++] = 0x80;
  if (num <= 56u) {
    memset(buf + num, 0, 56u - num);
  } else {
    memset(buf + num, 0, 64u - num);
    sha1_hash_block(c, buf);
    memset(buf, 0, 56u);
  }
  uint32_t blk[16];
  memcpy(blk, buf, 56);
  for (int i = 0; i < 14; ++i) blk[i] = byte_reverse(blk[i]); /* CorrectEndianess */
  /* GetBitCountHi/Lo, iterhash.h:30-31; big-endian order puts Hi first */
  blk[14] = (c->count_lo >> 29) + (c->count_hi << 3);
  blk[15] = c->count_lo << 3;
  sha1_transform(c->digest, blk);
  for (int i = 0; i < 5; ++i) {
    uint32_t v = c->digest[i];
    out[4 * i + 0] = (uint8_t)(v >> 24);
    out[4 * i + 1] = (uint8_t)(v >> 16);
    out[4 * i + 2] = (uint8_t)(v >> 8);
    out[4 * i + 3] = (uint8_t)v;
  }
  oracle_sha1_init(c); /* Restart(), iterhash.h:120 */
}

/* One-shot SHA-1 of a buffer, as Encoder::Base64Encode feeds it
 * (StringSource(..., pumpAll=true) -> HashFilter -> Update + Final). */
void oracle_sha1(const uint8_t* data, uint32_t len, uint8_t out[20]) {
  oracle_sha1_ctx c;
  oracle_sha1_init(&c);
  oracle_sha1_update(&c, data, len);
  oracle_sha1_final(&c, out);
}

/* ------------------------------------------------------------------------ */
/* base64-27: BaseN_Encoder(alphabet, log2base=6) with no padding parameter, */
/* basecode.cpp:13-37 (m_padding = -1) and :39-104 (MSB-first bit packing).  */
/* ------------------------------------------------------------------------ */
static const char k_b64_alphabet[] =
    "ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789+/"; /* Encoder.cpp:104-105 */

/* Generic base-2^bits encoder restating Put2's bit loop; returns chars written. */
static int basen_encode(const uint8_t* in, int len, int bits, char* out) {
  int nout = 0;
  unsigned acc = 0;      /* m_outBuf[m_bytePos] under construction */
  int bitpos = 0;        /* m_bitPos */
  for (int i = 0; i < len; ++i) {
    unsigned b = in[i];
    int left_src = 8;
    for (;;) {
      int left_tgt = bits - bitpos;
      acc |= b >> (8 - left_tgt);
      if (left_src >= left_tgt) {
        out[nout++] = k_b64_alphabet[acc & ((1u << bits) - 1u)];
        acc = 0;
        bitpos = 0;
        left_src -= left_tgt;
        if (left_src == 0) break;
        b = (b << left_tgt) & 0xffu;
      } else {
        bitpos += left_src;
        break;
      }
    }
  }
  if (bitpos > 0) out[nout++] = k_b64_alphabet[acc & ((1u << bits) - 1u)]; /* messageEnd */
  return nout;
}

/* 20-byte digest -> 27 chars + NUL */
void oracle_b64_27(const uint8_t digest[20], char out[28]) {
  int n = basen_encode(digest, 20, 6, out);
  out[n] = '\0';
}

/* Encoder::Base64Encode(data, size, string) restated */
void oracle_base64_encode(const uint8_t* data, uint32_t size, char out[28]) {
  uint8_t d[20];
  oracle_sha1(data, size, d);
  oracle_b64_27(d, out);
}

/* ------------------------------------------------------------------------ */
/* Chunking (Encoder.cpp:37-79): chunk i covers [i*cs, min((i+1)*cs, len)). */
/* Returns the number of chunks (0 for an empty file: the fread loop breaks   */
/* on the first zero-byte read and no Chunk is pushed).                       */
/* ------------------------------------------------------------------------ */
uint64_t oracle_chunk_count(uint64_t len, uint32_t chunk_size) {
  if (chunk_size == 0) return 0;
  return (len + chunk_size - 1) / chunk_size;
}

uint64_t oracle_encode_buffer(const uint8_t* data, uint64_t len, uint32_t chunk_size,
                              uint8_t* digests /* n*20 */) {
  uint64_t n = oracle_chunk_count(len, chunk_size);
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t off = i * (uint64_t)chunk_size;
    uint64_t sz = len - off < chunk_size ? len - off : chunk_size;
    oracle_sha1(data + off, (uint32_t)sz, digests + 20 * i);
  }
  return n;
}

/* fread-inclusive single-thread encode of one file, as Encoder::EncodeFile
 * does it (one buffer of chunk_size bytes, sequential fread + hash).
 * Returns chunk count, or -1 when the file cannot be opened. */
int64_t oracle_encode_file(const char* path, uint32_t chunk_size, uint8_t* digests,
                           uint64_t max_chunks, uint32_t* sizes_out) {
  FILE* f = fopen(path, "rb");
  if (!f || chunk_size == 0) {
    if (f) fclose(f);
    return -1;
  }
  uint8_t* buf = (uint8_t*)malloc(chunk_size);
  int64_t idx = 0;
  for (;;) {
    size_t got = fread(buf, 1, chunk_size, f);
    if (got == 0) break;
    if ((uint64_t)idx < max_chunks) {
      oracle_sha1(buf, (uint32_t)got, digests + 20 * idx);
      if (sizes_out) sizes_out[idx] = (uint32_t)got;
    }
    ++idx;
  }
  free(buf);
  fclose(f);
  return idx;
}

/* ------------------------------------------------------------------------ */
/* Batch over (offset, size) descriptors, optionally chunk-parallel across   */
/* threads: the "all host cores" comparator of SURVEY §8d (ii).  The         */
/* reference itself is single threaded (Encoder.cpp:40-79).                  */
/* ------------------------------------------------------------------------ */
typedef struct {
  const uint8_t* base;
  const uint64_t* offsets;
  const uint32_t* sizes;
  uint64_t begin, end;
  uint8_t* digests;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  for (uint64_t i = j->begin; i < j->end; ++i)
    oracle_sha1(j->base + j->offsets[i], j->sizes[i], j->digests + 20 * i);
  return NULL;
}

void oracle_sha1_batch(const uint8_t* base, const uint64_t* offsets, const uint32_t* sizes,
                       uint64_t n, uint8_t* digests, int nthreads) {
  if (nthreads <= 1 || n < 2) {
    batch_job j = {base, offsets, sizes, 0, n, digests};
    batch_worker(&j);
    return;
  }
  if ((uint64_t)nthreads > n) nthreads = (int)n;
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  batch_job* jobs = (batch_job*)malloc(sizeof(batch_job) * (size_t)nthreads);
  for (int t = 0; t < nthreads; ++t) {
    jobs[t].base = base;
    jobs[t].offsets = offsets;
    jobs[t].sizes = sizes;
    jobs[t].begin = n * (uint64_t)t / (uint64_t)nthreads;
    jobs[t].end = n * (uint64_t)(t + 1) / (uint64_t)nthreads;
    jobs[t].digests = digests;
    pthread_create(&th[t], NULL, batch_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}

/* ------------------------------------------------------------------------ */
/* Synthetic bytes: counter-mode splitmix64.  Word k of stream  */
/* `seed` is mix64(seed*0xD1B54A32D192ED03 + (k+1)*0x9E3779B97F4A7C15), laid */
/* out little-endian.  Identical definition in tests/golden/make_golden.py   */
/* (numpy) and in the product's device fill kernel (lbf_fill_synthetic).     */
/* ------------------------------------------------------------------------ */
static uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t oracle_synth_word(uint64_t seed, uint64_t k) {
  return mix64(seed * 0xD1B54A32D192ED03ull + (k + 1) * 0x9E3779B97F4A7C15ull);
}

/* Fill out[0..len) with stream bytes starting at byte offset `start`. */
void oracle_synth_fill(uint8_t* out, uint64_t len, uint64_t seed, uint64_t start) {
  uint64_t i = 0;
  while (i < len) {
    uint64_t pos = start + i;
    uint64_t w = oracle_synth_word(seed, pos >> 3);
    unsigned sh = (unsigned)(pos & 7u);
    if (sh == 0 && len - i >= 8) {
      memcpy(out + i, &w, 8); /* little-endian host */
      i += 8;
    } else {
      out[i++] = (uint8_t)(w >> (8 * sh));
    }
  }
}

typedef struct {
  uint8_t* out;
  uint64_t len, seed, start;
} fill_job;

static void* fill_worker(void* arg) {
  fill_job* j = (fill_job*)arg;
  oracle_synth_fill(j->out, j->len, j->seed, j->start);
  return NULL;
}

void oracle_synth_fill_mt(uint8_t* out, uint64_t len, uint64_t seed, uint64_t start, int nthreads) {
  if (nthreads <= 1 || len < (1u << 20)) {
    oracle_synth_fill(out, len, seed, start);
    return;
  }
  pthread_t* th = (pthread_t*)malloc(sizeof(pthread_t) * (size_t)nthreads);
  fill_job* jobs = (fill_job*)malloc(sizeof(fill_job) * (size_t)nthreads);
  uint64_t per = ((len / (uint64_t)nthreads) + 7) & ~7ull;
  int used = 0;
  for (int t = 0; t < nthreads; ++t) {
    uint64_t b = per * (uint64_t)t;
    if (b >= len) break;
    uint64_t e = b + per < len ? b + per : len;
    jobs[t].out = out + b;
    jobs[t].len = e - b;
    jobs[t].seed = seed;
    jobs[t].start = start + b;
    pthread_create(&th[t], NULL, fill_worker, &jobs[t]);
    ++used;
  }
  for (int t = 0; t < used; ++t) pthread_join(th[t], NULL);
  free(th);
  free(jobs);
}
