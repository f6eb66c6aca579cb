// sha1_device.hpp -- SHA-1 building blocks for the CDNA4 (gfx950) chunk-hash kernels.
//
// Semantics follow the reference's hash exactly (Crypto++ 5.2.1 SHA via
// Encoder::Base64Encode, /root/reference/cpp/src/Encoder.cpp:107-120):
//   init state           cpp/extern/crypto++/5.2.1/sha.cpp:19-26
//   80-round compression  sha.cpp:28-79 (f1 choose, f2/f4 parity, f3 majority)
//   big-endian words      iterhash.h:123-132 (ByteReverse on little-endian hosts)
//   0x80 pad + 64-bit big-endian bit length in words 14-15, one or two final
//   blocks                iterhash.cpp:86-99, iterhash.h:30-31,106-121
//
// Everything here is 32-bit integer VALU work: rotates lower to v_alignbit_b32,
// the three round functions and the schedule's 3-way xor to gfx950's
// v_bitop3_b32, byte swaps to v_perm_b32, the 5-term round sums to two
// v_add3_u32.  No MFMA: hashing is not a contraction.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

namespace lbf {

constexpr uint32_t kH0 = 0x67452301u;
constexpr uint32_t kH1 = 0xEFCDAB89u;
constexpr uint32_t kH2 = 0x98BADCFEu;
constexpr uint32_t kH3 = 0x10325476u;
constexpr uint32_t kH4 = 0xC3D2E1F0u;

constexpr uint32_t kK1 = 0x5A827999u;  // rounds  0-19 (R0/R1)
constexpr uint32_t kK2 = 0x6ED9EBA1u;  // rounds 20-39 (R2)
constexpr uint32_t kK3 = 0x8F1BBCDCu;  // rounds 40-59 (R3)
constexpr uint32_t kK4 = 0xCA62C1D6u;  // rounds 60-79 (R4)

__device__ __forceinline__ uint32_t rotl(uint32_t x, int n) { return (x << n) | (x >> (32 - n)); }

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_bswap32(x); }

// gfx950 v_bitop3_b32 evaluates any 3-input bitwise function in one VALU op:
// result bit = LUT[(S0<<2)|(S1<<1)|S2], i.e. LUT = f(0xF0, 0xCC, 0xAA).
constexpr uint32_t kLutChoose = 0xCA;  // (b & c) | (~b & d)          f1, sha.cpp:28
constexpr uint32_t kLutParity = 0x96;  // b ^ c ^ d                    f2/f4, sha.cpp:29,31
constexpr uint32_t kLutMajor = 0xE8;   // (b & c) | (d & (b | c))     f3, sha.cpp:30

template <uint32_t kLut>
__device__ __forceinline__ uint32_t bitop3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, kLut);
}
__device__ __forceinline__ uint32_t f_choose(uint32_t b, uint32_t c, uint32_t d) {
  return bitop3<kLutChoose>(b, c, d);
}
__device__ __forceinline__ uint32_t f_major(uint32_t b, uint32_t c, uint32_t d) {
  return bitop3<kLutMajor>(b, c, d);
}
__device__ __forceinline__ uint32_t f_parity(uint32_t b, uint32_t c, uint32_t d) {
  return bitop3<kLutParity>(b, c, d);
}
// blk1 (sha.cpp:15): rotl(w[i-3] ^ w[i-8] ^ w[i-14] ^ w[i-16], 1)
__device__ __forceinline__ uint32_t sched(uint32_t w3, uint32_t w8, uint32_t w14, uint32_t w16) {
  return rotl(bitop3<kLutParity>(w3, w8, w14) ^ w16, 1);
}

struct Digest {
  uint32_t h[5];
  __device__ __forceinline__ void init() {
    h[0] = kH0; h[1] = kH1; h[2] = kH2; h[3] = kH3; h[4] = kH4;
  }
};

// One SHA-1 round (sha.cpp:34-38) with round index i known at compile time
// after unrolling.  `x` is the schedule word W[i].  The five-term sum is two
// v_add3_u32 (the round constant rides in an SGPR/literal).
__device__ __forceinline__ void round_step(int i, uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                           uint32_t& e, uint32_t x) {
  uint32_t f, k;
  if (i < 20) {
    f = f_choose(b, c, d);
    k = kK1;
  } else if (i < 40) {
    f = f_parity(b, c, d);
    k = kK2;
  } else if (i < 60) {
    f = f_major(b, c, d);
    k = kK3;
  } else {
    f = f_parity(b, c, d);
    k = kK4;
  }
  const uint32_t t = rotl(a, 5) + f + (e + x + k);
  e = d;
  d = c;
  c = rotl(b, 30);
  b = a;
  a = t;
}

// One compression of a 16-word big-endian block.  `w` is consumed as the
// 16-word rolling message schedule (the blk1 window of sha.cpp:15).
__device__ __forceinline__ void compress(Digest& s, uint32_t (&w)[16]) {
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
  for (int i = 0; i < 80; ++i) {
    uint32_t x;
    if (i < 16) {
      x = w[i];
    } else {
      x = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]);
      w[i & 15] = x;
    }
    round_step(i, a, b, c, d, e, x);
  }
  s.h[0] += a;
  s.h[1] += b;
  s.h[2] += c;
  s.h[3] += d;
  s.h[4] += e;
}

// The four round constants in VGPRs.  A v_add3_u32 that reads K from an SGPR
// costs a lone wave ≈5 more cycles per round than one reading three VGPRs
// (25.6 vs 23.2 cycles per round, tools/probe_lds_lanes.hip modes 3/4), so the
// consumers that add K themselves take it from here.  The asm keeps the
// compiler from folding the constants back into SGPR operands.
struct RoundK {
  uint32_t k[4];
  __device__ __forceinline__ RoundK() {
    const uint32_t c[4] = {kK1, kK2, kK3, kK4};
#pragma unroll
    for (int j = 0; j < 4; ++j) asm volatile("v_mov_b32 %0, %1" : "=v"(k[j]) : "s"(c[j]));
  }
};

// One round of the two-add3 form with K from a VGPR:
// t = rotl5(a) + f + (e + x + K).
__device__ __forceinline__ void round_step_kv(int i, uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                              uint32_t& e, uint32_t x, const RoundK& K) {
  uint32_t f;
  if (i < 20) f = f_choose(b, c, d);
  else if (i < 40 || i >= 60) f = f_parity(b, c, d);
  else f = f_major(b, c, d);
  const uint32_t t = rotl(a, 5) + f + (e + x + K.k[i / 20]);
  e = d;
  d = c;
  c = rotl(b, 30);
  b = a;
  a = t;
}

// Compression with the 80-word schedule already expanded (by a producer wave)
// and stored in LDS as 20 uint4 per chain, `stride` uint4 apart.
__device__ __forceinline__ void compress_expanded(Digest& s, const uint4* w, int stride, const RoundK& K) {
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
  for (int q = 0; q < 20; ++q) {
    const uint4 v = w[q * stride];
    round_step_kv(4 * q + 0, a, b, c, d, e, v.x, K);
    round_step_kv(4 * q + 1, a, b, c, d, e, v.y, K);
    round_step_kv(4 * q + 2, a, b, c, d, e, v.z, K);
    round_step_kv(4 * q + 3, a, b, c, d, e, v.w, K);
  }
  s.h[0] += a;
  s.h[1] += b;
  s.h[2] += c;
  s.h[3] += d;
  s.h[4] += e;
}

// Expand a 16-word block into the 80-word schedule and store it as 20 uint4
// (`stride` uint4 apart): the producer half of compress_expanded.
__device__ __forceinline__ void expand_store(uint32_t (&w)[16], uint4* out, int stride) {
#pragma unroll
  for (int q = 0; q < 4; ++q) out[q * stride] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
#pragma unroll
  for (int q = 4; q < 20; ++q) {
    uint32_t x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * q + j;
      x[j] = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]);
      w[i & 15] = x[j];
    }
    out[q * stride] = make_uint4(x[0], x[1], x[2], x[3]);
  }
}

// Round constant of round i (sha.cpp:43-78).
__host__ __device__ constexpr uint32_t round_k(int i) {
  return i < 20 ? kK1 : (i < 40 ? kK2 : (i < 60 ? kK3 : kK4));
}

// A round whose schedule word already carries the round constant (wk = W[i] +
// K[i], added by the producer).  The remaining four-term sum is one VOP2 add and
// one v_add3_u32: a lone wave then issues the round's five VALU ops back to back
// (≈20.4 cycles), while the two-add3 form stalls ≈5 cycles per round on gfx950
// (tools/gen_round_order.py).
__device__ __forceinline__ void round_step_wk(int i, uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                              uint32_t& e, uint32_t wk) {
  uint32_t f;
  if (i < 20) f = f_choose(b, c, d);
  else if (i < 40 || i >= 60) f = f_parity(b, c, d);
  else f = f_major(b, c, d);
  const uint32_t s = e + wk;
  const uint32_t n = rotl(a, 5) + f + s;
  e = d;
  d = c;
  c = rotl(b, 30);
  b = a;
  a = n;
}

__device__ __forceinline__ void compress_expanded_wk(Digest& s, const uint4* w, int stride) {
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
  for (int q = 0; q < 20; ++q) {
    const uint4 v = w[q * stride];
    round_step_wk(4 * q + 0, a, b, c, d, e, v.x);
    round_step_wk(4 * q + 1, a, b, c, d, e, v.y);
    round_step_wk(4 * q + 2, a, b, c, d, e, v.z);
    round_step_wk(4 * q + 3, a, b, c, d, e, v.w);
  }
  s.h[0] += a;
  s.h[1] += b;
  s.h[2] += c;
  s.h[3] += d;
  s.h[4] += e;
}

// Half (kHalf = 0: words 0..39, 1: words 40..79) of the 80-word schedule with
// the round constants added, stored as 10 uint4 `stride` apart.  `w` is the
// 16-word rolling window and carries over from half 0 to half 1.
template <int kHalf>
__device__ __forceinline__ void expand_store_wk(uint32_t (&w)[16], uint4* out, int stride) {
#pragma unroll
  for (int q = 10 * kHalf; q < 10 * kHalf + 10; ++q) {
    uint32_t x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * q + j;
      if (i < 16) {
        x[j] = w[i];
      } else {
        x[j] = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]);
        w[i & 15] = x[j];
      }
      x[j] += round_k(i);
    }
    out[q * stride] = make_uint4(x[0], x[1], x[2], x[3]);
  }
}

// expand_store_wk with the words stored as 20 uint2 pairs (`stride` uint2
// apart) for consumers that read the schedule with ds_read_b64.
template <int kHalf>
__device__ __forceinline__ void expand_store_wk2(uint32_t (&w)[16], uint2* out, int stride) {
#pragma unroll
  for (int q = 20 * kHalf; q < 20 * kHalf + 20; ++q) {
    uint32_t x[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = 2 * q + j;
      if (i < 16) {
        x[j] = w[i];
      } else {
        x[j] = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]);
        w[i & 15] = x[j];
      }
      x[j] += round_k(i);
    }
    out[q * stride] = make_uint2(x[0], x[1]);
  }
}

// The whole 80-word schedule as 40 uint2 pairs (`stride` uint2 apart), with
// the round constant added to words kKFrom..79 only: the consumer adds K
// itself in rounds 0..kKFrom-1 (pcx4, where one producer feeds one consumer).
template <int kKFrom>
__device__ __forceinline__ void expand_store_split(uint32_t (&w)[16], uint2* out, int stride) {
#pragma unroll
  for (int q = 0; q < 40; ++q) {
    uint32_t x[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = 2 * q + j;
      if (i < 16) {
        x[j] = w[i];
      } else {
        x[j] = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]);
        w[i & 15] = x[j];
      }
      if (i >= kKFrom) x[j] += round_k(i);
    }
    out[q * stride] = make_uint2(x[0], x[1]);
  }
}

// Words 16..79 of the schedule as 32 uint2 pairs (`stride` uint2 apart), K
// added to words kKFrom..79: the consumer takes words 0..15 from the raw block.
template <int kKFrom>
__device__ __forceinline__ void expand_store_from16(uint32_t (&w)[16], uint2* out, int stride) {
#pragma unroll
  for (int q = 8; q < 40; ++q) {
    uint32_t x[2];
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int i = 2 * q + j;
      x[j] = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]);
      w[i & 15] = x[j];
      if (i >= kKFrom) x[j] += round_k(i);
    }
    out[(q - 8) * stride] = make_uint2(x[0], x[1]);
  }
}

// Big-endian block from four 16-byte little-endian vectors.
__device__ __forceinline__ void block_from_vec(uint32_t (&w)[16], const uint4& q0, const uint4& q1,
                                               const uint4& q2, const uint4& q3) {
  w[0] = bswap(q0.x);  w[1] = bswap(q0.y);  w[2] = bswap(q0.z);  w[3] = bswap(q0.w);
  w[4] = bswap(q1.x);  w[5] = bswap(q1.y);  w[6] = bswap(q1.z);  w[7] = bswap(q1.w);
  w[8] = bswap(q2.x);  w[9] = bswap(q2.y);  w[10] = bswap(q2.z); w[11] = bswap(q2.w);
  w[12] = bswap(q3.x); w[13] = bswap(q3.y); w[14] = bswap(q3.z); w[15] = bswap(q3.w);
}

// 64 bytes at any alignment as 16 little-endian words, for chunks whose start
// is not 16-byte aligned and for the tail.  Only dwords that hold at least one
// of the `valid` (>= 1) readable bytes are loaded -- an aligned dword never
// straddles a page, so nothing past the chunk's last byte page is touched --
// and v_alignbyte_b32 funnels them into place.  Words past `valid` hold
// don't-care bytes the caller masks.
__device__ __forceinline__ void load_words_any(uint32_t (&le)[16], const uint8_t* p, uint32_t valid) {
  const uint32_t sh = (uint32_t)(reinterpret_cast<uintptr_t>(p) & 3u);
  const uint32_t* b = reinterpret_cast<const uint32_t*>(p - sh);
  const uint32_t last = (sh + valid - 1) >> 2;  // last dword holding a valid byte (<= 16)
  uint32_t d[17];
#pragma unroll
  for (uint32_t m = 0; m < 17; ++m) d[m] = b[m < last ? m : last];
#pragma unroll
  for (int k = 0; k < 16; ++k) le[k] = __builtin_amdgcn_alignbyte(d[k + 1], d[k], sh);
}

// Final-block words: the r = size % 64 trailing bytes, the 0x80 pad byte and
// (when `with_len`) the big-endian bit length (iterhash.cpp:86-99,
// iterhash.h:30-31,106-121).  `which` = 0 builds the block holding the tail
// bytes; 1 builds the all-zero second block used when r >= 56.
__device__ __forceinline__ void final_block(uint32_t (&w)[16], const uint8_t* tail, uint32_t r, uint32_t total,
                                            bool second) {
  if (r && !second) {
    load_words_any(w, tail, r);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = 0;
  }
  const uint32_t rr = second ? 0u : r;
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int rem = (int)rr - 4 * k;  // chunk bytes left in this word
    uint32_t v = bswap(w[k]);
    if (rem <= 0) v = 0;
    if (!second && rem >= 0 && rem < 4) {
      const uint32_t sh = 8u * (uint32_t)rem;
      v = (v & ~(0xFFFFFFFFu >> sh)) | (0x80000000u >> sh);  // keep `rem` bytes, then 0x80
    }
    w[k] = v;
  }
  if (second || r < 56) {
    w[14] = total >> 29;  // GetBitCountHi for a 32-bit byte count
    w[15] = total << 3;   // GetBitCountLo
  }
}

// Final one or two compressions of a chunk whose full blocks are done (the
// lane kernel's tail; the pc kernel's producer builds the same words with
// final_block instead).
__device__ __forceinline__ void finish(Digest& s, const uint8_t* tail, uint32_t r, uint32_t total) {
  uint32_t w[16];
  final_block(w, tail, r, total, false);
  if (r >= 56) {
    compress(s, w);
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = 0;
    w[14] = total >> 29;
    w[15] = total << 3;
  }
  compress(s, w);
}

// splitmix64 counter-mode synthetic stream; identical to
// oracle_synth_word in oracle/sha1_oracle.c and synth_np in
// tests/golden/make_golden.py.
__device__ __forceinline__ uint64_t synth_word(uint64_t seed, uint64_t k) {
  uint64_t z = seed * 0xD1B54A32D192ED03ull + (k + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

}  // namespace lbf
