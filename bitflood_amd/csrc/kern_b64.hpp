// kern_b64.hpp -- the receiver's base64 decode on the device (gfx950).
//
// A SendChunk frame carries the chunk as XML-RPC base64 text
// (/root/reference/cpp/src/ChunkMethods.cpp:141-163, decoded by xmlrpc++ 0.7
// XmlRpcValue::binaryFromXml, XmlRpcValue.cpp:417-436, with the decoder of
// base64.h:215-330).  lbf_b64_verify_batch decodes each chunk's text here, in
// HBM, and the shipped hash kernels verify the decoded bytes where they lie,
// so the receiver's two per-chunk passes (decode, then hash) both run on the
// GPU and only the text crosses PCIe on the way in.
//
// Decode rules (base64.h:215-330, restated in bitflood_amd/host/PeerWire.cpp
// Base64Get and tests/test_gpu_b64.py):
//   - characters outside the alphabet (the frame's spaces, anything else) are
//     skipped;
//   - the remaining characters S[0..m) are taken four at a time; a group that
//     holds '=' ends the data: "xx==" gives one byte, "xxx=" two, '=' in the
//     first or second place none; an incomplete last group gives nothing.
// So with q = the index of the first '=' in S (m if none), the output is the
// 3 * floor(min(q, m) / 4) bytes of the complete groups, plus one byte when
// q % 4 == 2 or two when q % 4 == 3 (q < m).
//
// Text laid out as the encoder writes it (nearly every frame) goes through
// b64_decode_canon_kernel: one pass, each lane decodes four groups from their
// known places, 7/3 bytes moved per decoded byte.  Any other text goes through
// b64_decode_kernel, one workgroup per chunk: pass 1 compacts the text (4 KiB
// tiles, each lane classifies 16 characters, a workgroup scan gives every
// valid character its index in S, and the sextets are written to a scratch
// area laid out like the text); pass 2 turns four groups (16 sextets, one
// 16-byte load) into 12 bytes per lane.  5 bytes moved per decoded byte (4/3
// each for the text read and the sextets written and read back, 1 for the
// bytes written).
//
// Part of the single translation unit sha1_kernels.hip (included from there).
#pragma once

#include <hip/hip_runtime.h>

#include "lbf_internal.hpp"

namespace lbf {
namespace {

constexpr uint8_t kB64Eq = 64, kB64Skip = 255;
constexpr int kB64Threads = 256;  // one lane per entry of the decode table below

struct B64Table {
  uint8_t v[256];
};

constexpr B64Table make_b64_table() {
  B64Table t{};
  for (int c = 0; c < 256; ++c) t.v[c] = kB64Skip;
  for (int c = 'A'; c <= 'Z'; ++c) t.v[c] = (uint8_t)(c - 'A');
  for (int c = 'a'; c <= 'z'; ++c) t.v[c] = (uint8_t)(26 + c - 'a');
  for (int c = '0'; c <= '9'; ++c) t.v[c] = (uint8_t)(52 + c - '0');
  t.v['+'] = 62;
  t.v['/'] = 63;
  t.v['='] = kB64Eq;
  return t;
}

__constant__ B64Table g_b64_table = make_b64_table();

// Exclusive scan of one value per lane over the 256-lane workgroup; returns
// the lane's prefix and writes the total to *total.  `sums` is 4 words of LDS.
__device__ __forceinline__ uint32_t wg_exclusive_scan(uint32_t v, uint32_t* sums, uint32_t* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) sums[wave] = x;
  __syncthreads();
  uint32_t before = 0, all = 0;
#pragma unroll
  for (int w = 0; w < kB64Threads / 64; ++w) {
    const uint32_t s = sums[w];
    before += w < wave ? s : 0u;
    all += s;
  }
  __syncthreads();  // sums is reused by the next call
  *total = all;
  return before + x - v;
}

// ---------------------------------------------------------------------------
// One pass for text laid out as the encoder writes it (round 4).  Almost every
// frame carries exactly what xmlrpc++'s encoder wrote: group g of the chunk at
// 4g + g/18, a separator (any character outside the alphabet) after every 18th
// group, '=' only as "xx==" / "xxx=" in the last group.  For such a text the
// place of every character is known without a scan, so each lane decodes four
// groups straight from the text into the output: 7/3 bytes moved per decoded
// byte instead of 5, one pass instead of two, and no workgroup barrier.  The
// lanes check the layout as they read it; a chunk whose text breaks it
// anywhere (junk, a dropped or extra character, '=' elsewhere) is marked in
// redo[] and decoded again by b64_decode_kernel, whose general rules give the
// same result as this pass on every canonical text.
//
// A canonical text of G groups has length L = 73 q + 4 r for G = 18 q + r,
// r < 18, so G follows from L alone.  grid = (chunks, parts): part y of chunk
// i takes tasks [y * per, (y + 1) * per) of four groups each.
// ---------------------------------------------------------------------------
__device__ __forceinline__ bool b64_canon_groups(uint32_t len, uint32_t* groups) {
  const uint32_t q = len / 73, rem = len % 73;
  if (rem % 4 != 0 || rem / 4 >= 18) return false;
  *groups = 18 * q + rem / 4;
  return true;
}

__global__ void __launch_bounds__(kB64Threads) b64_decode_canon_kernel(const uint8_t* __restrict__ text,
                                                                       const uint64_t* __restrict__ text_off,
                                                                       const uint32_t* __restrict__ text_len,
                                                                       uint8_t* __restrict__ out,
                                                                       const uint64_t* __restrict__ out_off,
                                                                       const uint32_t* __restrict__ cap,
                                                                       uint32_t* __restrict__ sizes,
                                                                       uint8_t* __restrict__ over,
                                                                       uint8_t* __restrict__ redo) {
  __shared__ uint8_t tab[256];
  tab[threadIdx.x] = g_b64_table.v[threadIdx.x];
  __syncthreads();
  const uint32_t i = blockIdx.x, part = blockIdx.y, parts = gridDim.y;
  const uint8_t* t = text + text_off[i];
  const uint32_t len = text_len[i];
  uint32_t groups = 0;
  if (!b64_canon_groups(len, &groups)) {
    if (part == 0 && threadIdx.x == 0) redo[i] = 1;
    return;
  }
  const uint32_t limit = cap[i];
  uint8_t* o = out + out_off[i];
  // the last group: "xxxx", "xxx=" or "xx=="; its byte count sets the length
  uint32_t last = 3;
  bool bad = false;
  if (groups > 0) {
    const uint32_t g = groups - 1, at = 4 * g + g / 18;
    const uint8_t c2 = tab[t[at + 2]], c3 = tab[t[at + 3]];
    last = c3 < 64 ? 3u : c2 < 64 ? 2u : 1u;
    bad = c3 == kB64Skip || c2 == kB64Skip || (c2 == kB64Eq && c3 != kB64Eq);
  }
  const uint64_t want = groups ? 3ull * (groups - 1) + last : 0;
  if (part == 0 && threadIdx.x == 0) {
    sizes[i] = (uint32_t)min<uint64_t>(want, limit);
    over[i] = want > limit ? 1 : 0;
  }
  const uint32_t tasks = (groups + 3) / 4;
  const uint32_t per = (tasks + parts - 1) / parts;
  const uint32_t end = min(tasks, (part + 1) * per);
  for (uint32_t k = part * per + threadIdx.x; k < end; k += kB64Threads) {
    uint8_t b[12];
    uint32_t nb = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t g = 4 * k + j;
      if (g >= groups) break;
      const uint32_t at = 4 * g + g / 18;
      const uint8_t v0 = tab[t[at]], v1 = tab[t[at + 1]], v2 = tab[t[at + 2]], v3 = tab[t[at + 3]];
      if (g + 1 < groups) {
        bad |= (v0 | v1 | v2 | v3) >= 64;  // '=' (64) or skip (255) inside the text
        if (g % 18 == 17) bad |= tab[t[at + 4]] != kB64Skip;  // the separator
      } else {
        bad |= v0 >= 64 || v1 >= 64;  // the last group's padding was checked above
        if (g % 18 == 17) bad |= tab[t[at + 4]] != kB64Skip;
      }
      const uint32_t x = ((uint32_t)(v0 & 63) << 18) | ((uint32_t)(v1 & 63) << 12) | ((uint32_t)(v2 & 63) << 6) |
                         (v3 & 63);
      b[3 * j] = (uint8_t)(x >> 16);
      b[3 * j + 1] = (uint8_t)(x >> 8);
      b[3 * j + 2] = (uint8_t)x;
      nb = g + 1 < groups ? nb + 3 : nb + last;
    }
    const uint64_t at = 12ull * k;
    if (nb == 12 && at + 12 <= limit && (reinterpret_cast<uintptr_t>(o + at) & 3u) == 0) {
      uint32_t* d = reinterpret_cast<uint32_t*>(o + at);
#pragma unroll
      for (int j = 0; j < 3; ++j)
        d[j] = (uint32_t)b[4 * j] | ((uint32_t)b[4 * j + 1] << 8) | ((uint32_t)b[4 * j + 2] << 16) |
               ((uint32_t)b[4 * j + 3] << 24);
    } else {
      for (uint32_t j = 0; j < nb && at + j < limit; ++j) o[at + j] = b[j];
    }
  }
  if (bad) redo[i] = 1;  // every writer stores the same 1
}

// blockIdx.x = chunk (skipped when redo is given and redo[chunk] == 0).
// Chunk i's text is text[text_off[i] .. + text_len[i])
// (any alignment; 4-byte aligned reads faster) and its sextets go to
// scratch[sext_off[i] ..) (16-byte aligned, room for text_len[i]: the
// compacted stream is never longer than the text).  out[out_off[i] .. + cap[i])
// receives the decoded bytes; sizes[i] = min(decoded length, cap[i]) and
// over[i] = 1 when the text decodes to more than cap[i] bytes.
__global__ void __launch_bounds__(kB64Threads) b64_decode_kernel(const uint8_t* __restrict__ text,
                                                                 uint8_t* __restrict__ scratch,
                                                                 const uint64_t* __restrict__ text_off,
                                                                 const uint64_t* __restrict__ sext_off,
                                                                 const uint32_t* __restrict__ text_len,
                                                                 uint8_t* __restrict__ out,
                                                                 const uint64_t* __restrict__ out_off,
                                                                 const uint32_t* __restrict__ cap,
                                                                 uint32_t* __restrict__ sizes,
                                                                 uint8_t* __restrict__ over,
                                                                 const uint8_t* __restrict__ redo) {
  // after b64_decode_canon_kernel: only the chunks it could not take
  if (redo && !redo[blockIdx.x]) return;
  __shared__ uint32_t sums[kB64Threads / 64];
  __shared__ uint32_t first_eq;
  __shared__ uint8_t tab[256];  // per-lane lookups: LDS serves divergent addresses, the constant table does not
  tab[threadIdx.x] = g_b64_table.v[threadIdx.x];
  const uint32_t i = blockIdx.x;
  const uint8_t* t = text + text_off[i];
  uint8_t* s = scratch + sext_off[i];
  const uint32_t len = text_len[i];
  if (threadIdx.x == 0) first_eq = 0xFFFFFFFFu;
  __syncthreads();
  // ---- pass 1: compact the alphabet characters (and '=') into sextets ----
  uint32_t base = 0;  // sextets written by earlier tiles
  for (uint32_t tile = 0; tile < len; tile += kB64Threads * 16) {
    const uint32_t at = tile + threadIdx.x * 16;
    uint8_t c[16];
    if (at + 16 <= len) {
      // the text of a chunk need not be 16-byte aligned: four dword loads
      // when it is 4-byte aligned, bytes otherwise
      if ((reinterpret_cast<uintptr_t>(t + at) & 3u) == 0) {
        const uint32_t* p = reinterpret_cast<const uint32_t*>(t + at);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t w = p[k];
          c[4 * k] = (uint8_t)w;
          c[4 * k + 1] = (uint8_t)(w >> 8);
          c[4 * k + 2] = (uint8_t)(w >> 16);
          c[4 * k + 3] = (uint8_t)(w >> 24);
        }
      } else {
#pragma unroll
        for (int k = 0; k < 16; ++k) c[k] = t[at + k];
      }
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) c[k] = at + k < len ? t[at + k] : (uint8_t)' ';
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      c[k] = tab[c[k]];
      cnt += c[k] != kB64Skip;
    }
    uint32_t total;
    uint32_t pos = base + wg_exclusive_scan(cnt, sums, &total);
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (c[k] == kB64Skip) continue;
      if (c[k] == kB64Eq) atomicMin(&first_eq, pos);
      s[pos++] = c[k];
    }
    base += total;
  }
  __threadfence_block();
  __syncthreads();
  const uint32_t m = base, q = min(first_eq, m);
  const uint32_t groups = q / 4;  // complete groups before any '='
  const uint32_t r = q % 4;
  // q < m: S[q] is '=': "xx=" gives one byte, "xxx=" two.  q == m: an
  // incomplete last group gives nothing.
  const uint32_t extra = q < m ? (r == 2 ? 1u : r == 3 ? 2u : 0u) : 0u;
  const uint64_t want = 3ull * groups + extra;
  const uint32_t limit = cap[i];
  uint8_t* o = out + out_off[i];
  // ---- pass 2: four groups (16 sextets) -> 12 bytes per lane ----
  for (uint32_t g4 = threadIdx.x * 4; g4 < groups; g4 += kB64Threads * 4) {
    uint8_t v[16];
    if (g4 + 4 <= groups) {
      const uint4 w = *reinterpret_cast<const uint4*>(s + 4ull * g4);  // 16-byte aligned: s is
      const uint32_t ws[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = (uint8_t)(ws[k >> 2] >> (8 * (k & 3)));
    } else {
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = 4 * g4 + k < 4ull * groups ? s[4 * g4 + k] : (uint8_t)0;
    }
    uint8_t b[12];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint32_t x = ((uint32_t)v[4 * k] << 18) | ((uint32_t)v[4 * k + 1] << 12) | ((uint32_t)v[4 * k + 2] << 6) |
                         v[4 * k + 3];
      b[3 * k] = (uint8_t)(x >> 16);
      b[3 * k + 1] = (uint8_t)(x >> 8);
      b[3 * k + 2] = (uint8_t)x;
    }
    const uint64_t at = 3ull * g4;
    const uint32_t nb = (uint32_t)min<uint64_t>(12, 3ull * (groups - g4));
    if (nb == 12 && at + 12 <= limit && (reinterpret_cast<uintptr_t>(o + at) & 3u) == 0) {
      uint32_t* d = reinterpret_cast<uint32_t*>(o + at);
#pragma unroll
      for (int k = 0; k < 3; ++k)
        d[k] = (uint32_t)b[4 * k] | ((uint32_t)b[4 * k + 1] << 8) | ((uint32_t)b[4 * k + 2] << 16) |
               ((uint32_t)b[4 * k + 3] << 24);
    } else {
      for (uint32_t k = 0; k < nb && at + k < limit; ++k) o[at + k] = b[k];
    }
  }
  if (threadIdx.x == 0) {
    if (extra) {
      const uint32_t a = 4 * groups;
      const uint32_t x = ((uint32_t)s[a] << 18) | ((uint32_t)s[a + 1] << 12) |
                         ((uint32_t)(extra == 2 ? s[a + 2] : 0) << 6);
      const uint64_t at = 3ull * groups;
      if (at < limit) o[at] = (uint8_t)(x >> 16);
      if (extra == 2 && at + 1 < limit) o[at + 1] = (uint8_t)(x >> 8);
    }
    sizes[i] = (uint32_t)min<uint64_t>(want, limit);
    over[i] = want > limit ? 1 : 0;
  }
}

}  // namespace
}  // namespace lbf

namespace lbf {
namespace {

// ---------------------------------------------------------------------------
// The sender's base64 encode (lbf_verify_encode_b64_batch): the text a
// SendChunk frame carries for chunk i, written as xmlrpc++ 0.7's encoder
// writes it (base64.h:154-210) and as the frame sends it (CR/LF become spaces,
// PeerConnection.cpp:132-156): four characters per three bytes, a space after
// every 18th complete group, the last one or two bytes as "xx==" / "xxx=".
// Group g of chunk i lands at 4g + g/18, so every lane writes its groups
// independently.  blockIdx.x = chunk; data[data_off[i] .. + size[i]) ->
// text[text_off[i] .. + b64_put_length(size[i])).
// ---------------------------------------------------------------------------
__host__ __device__ constexpr uint64_t b64_put_length(uint64_t size) {
  return 4 * (size / 3) + (size % 3 ? 4 : 0) + size / 3 / 18;
}

__global__ void __launch_bounds__(kB64Threads) b64_encode_kernel(const uint8_t* __restrict__ data,
                                                                 const uint64_t* __restrict__ data_off,
                                                                 const uint32_t* __restrict__ size,
                                                                 uint8_t* __restrict__ text,
                                                                 const uint64_t* __restrict__ text_off) {
  __shared__ uint8_t alpha[64];
  if (threadIdx.x < 64) {
    const uint32_t c = threadIdx.x;
    alpha[c] = (uint8_t)(c < 26 ? 'A' + c : c < 52 ? 'a' + (c - 26) : c < 62 ? '0' + (c - 52) : c == 62 ? '+' : '/');
  }
  __syncthreads();
  const uint32_t i = blockIdx.x;
  const uint8_t* d = data + data_off[i];
  uint8_t* t = text + text_off[i];
  const uint32_t n = size[i], full = n / 3;
  for (uint32_t g = threadIdx.x; g < full; g += kB64Threads) {
    const uint32_t x = ((uint32_t)d[3 * g] << 16) | ((uint32_t)d[3 * g + 1] << 8) | d[3 * g + 2];
    uint8_t* o = t + 4ull * g + g / 18;
    o[0] = alpha[x >> 18];
    o[1] = alpha[(x >> 12) & 63];
    o[2] = alpha[(x >> 6) & 63];
    o[3] = alpha[x & 63];
    if (g % 18 == 17) o[4] = ' ';  // base64.h:197-205's newline, framed as a space
  }
  if (threadIdx.x == 0 && n % 3) {
    uint8_t* o = t + 4ull * full + full / 18;
    const uint32_t x = ((uint32_t)d[3 * full] << 16) | (n % 3 == 2 ? (uint32_t)d[3 * full + 1] << 8 : 0u);
    o[0] = alpha[x >> 18];
    o[1] = alpha[(x >> 12) & 63];
    o[2] = n % 3 == 2 ? alpha[(x >> 6) & 63] : (uint8_t)'=';
    o[3] = '=';
  }
}

}  // namespace
}  // namespace lbf
