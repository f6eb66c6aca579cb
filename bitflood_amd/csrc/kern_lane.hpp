// kern_lane.hpp -- one chunk per lane: "lane" (variant 1) and "lds2" (11),
// the kernels for many chains (every SIMD busy).  "lds2" grew out of "lds"
// (variant 3: one 64-byte block per DMA step), kept in tools/experimental/.
//
// Part of the single translation unit sha1_kernels.hip (included from there);
// DESIGN.md §4 has the measurements behind each kernel.
#pragma once

#include <hip/hip_runtime.h>

#include "kern_common.hpp"

namespace lbf {
namespace {

__device__ __forceinline__ void load_block(uint4 (&q)[4], const uint4* src) {
  q[0] = src[0];
  q[1] = src[1];
  q[2] = src[2];
  q[3] = src[3];
}

// Full 64-byte blocks of a 16-byte aligned chunk, two blocks in flight ahead of
// the compression that consumes them.
__device__ __forceinline__ void hash_blocks_aligned(Digest& s, const uint8_t* src, uint32_t nblk) {
  if (nblk == 0) return;
  const uint4* q = reinterpret_cast<const uint4*>(src);
  const uint32_t last = nblk - 1;
  uint4 A[4], B[4];
  load_block(A, q);
  load_block(B, q + 4 * (last < 1u ? last : 1u));
  for (uint32_t b = 0; b < nblk; ++b) {
    uint4 C[4] = {A[0], A[1], A[2], A[3]};
    A[0] = B[0]; A[1] = B[1]; A[2] = B[2]; A[3] = B[3];
    const uint32_t nb = b + 2 < last ? b + 2 : last;  // clamp: re-read the last block
    load_block(B, q + 4 * nb);
    uint32_t w[16];
    block_from_vec(w, C[0], C[1], C[2], C[3]);
    compress(s, w);
  }
}

__device__ __forceinline__ void hash_blocks_unaligned(Digest& s, const uint8_t* src, uint32_t nblk) {
  for (uint32_t b = 0; b < nblk; ++b) {
    uint32_t w[16];
    load_words_any(w, src + 64ull * b, 64);
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = bswap(w[k]);
    compress(s, w);
  }
}

template <bool kUniform>
__global__ void __launch_bounds__(256) sha1_lane_kernel(ChunkParams p) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= p.n) return;
  uint64_t off;
  uint32_t size;
  if (kUniform) {
    off = (p.first_chunk + i) * (uint64_t)p.chunk_size;
    const uint64_t rem = p.len - off;
    size = rem < p.chunk_size ? (uint32_t)rem : p.chunk_size;
  } else {
    off = p.offsets[i];
    size = p.sizes[i];
  }
  const uint8_t* src = p.base + off;
  Digest s;
  s.init();
  const uint32_t nblk = size >> 6;
  if ((reinterpret_cast<uintptr_t>(src) & 15u) == 0) {
    hash_blocks_aligned(s, src, nblk);
  } else {
    hash_blocks_unaligned(s, src, nblk);
  }
  finish(s, src + 64ull * nblk, size & 63u, size);

  uint32_t be[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) be[k] = bswap(s.h[k]);  // digest bytes in big-endian order
  if (p.digests) {
    uint32_t* o = reinterpret_cast<uint32_t*>(p.digests + 20ull * i);
#pragma unroll
    for (int k = 0; k < 5; ++k) o[k] = be[k];
  }
  if (p.verdicts) {
    const uint32_t* e = reinterpret_cast<const uint32_t*>(p.expected + 20ull * i);
    uint32_t diff = 0;
#pragma unroll
    for (int k = 0; k < 5; ++k) diff |= be[k] ^ e[k];
    p.verdicts[i] = diff == 0 ? 1 : 0;
  }
}


// ---------------------------------------------------------------------------
// Kernel "lds2" (variant 11): one chunk per lane for MANY chains, fetching
// each chain's bytes a whole 128-B line at a time.
//
// With >= 4 waves per SIMD the VALU itself is the limit (≈2,040 SIMD cycles per
// 64-byte block) and what is left to win is memory stall: in the
// lane kernel the compiler sinks every 16-byte load next to its use, so each
// block waits a full HBM round trip.  Each wave streams its 64 chains' next
// blocks global -> LDS with DMA (no VGPRs in flight, so the compiler cannot
// move them) and waits by count.  The first form, `lds`, DMAs one 64-byte block per lane per step, so the two halves of a 128-B
// line are requested one step (≈2 M other lines chip-wide at C3) apart and
// HBM traffic reads 1.14 x algorithmic at 262 K chains (profiles/r01/c3_lds).
// Here the DMA for blocks 2j and 2j+1 goes out as 8 back-to-back instructions,
// so the second half merges with the first half's fill.  4 block slots per
// wave (16 KiB): 2 workgroups per CU, 2 waves per SIMD, which still keeps the
// VALU busy.
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lds2_dma_pair(const ChainInfo& c, uint32_t pair, uint32_t wave_lds) {
#pragma unroll
  for (uint32_t h = 0; h < 2; ++h) {
    const uint32_t b = 2 * pair + h;
    const bool ok = c.aligned && b < c.nfull;
    const uint8_t* src = ok ? c.src + 64ull * b : reinterpret_cast<const uint8_t*>(g_pc_dummy);
    const uint32_t slot = wave_lds + (b % 4) * (kPcRawU4 * 16);
#pragma unroll
    for (int j = 0; j < 4; ++j) dma16(src + 16 * j, slot + j * (kPcLanes * 16));
  }
}

template <bool kUniform>
__global__ void __launch_bounds__(256) sha1_lds2_kernel(ChunkParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 stage[];  // [wave][4 blocks][4][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const ChainInfo c = chain_info<kUniform>(p, i);
  uint4* mine = stage + wave * (4 * kPcRawU4);
  const uint32_t wave_lds = (uint32_t)reinterpret_cast<uintptr_t>(mine);
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane(wave_max(c.nfull));
  const bool any_unaligned = __builtin_amdgcn_readfirstlane(
      (uint32_t)(__ballot(c.total != 0 && !c.aligned) != 0));
  Digest s;
  s.init();
  lds2_dma_pair(c, 0, wave_lds);
  lds2_dma_pair(c, 1, wave_lds);
  for (uint32_t k = 0; k < nsteps; ++k) {
    // pair k/2 has landed once only pair k/2 + 1 (8 DMAs) is pending
    if ((k & 1u) == 0) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    const uint4* raw = mine + (k % 4) * kPcRawU4 + lane;
    uint32_t w[16];
    block_from_vec(w, raw[0], raw[kPcLanes], raw[2 * kPcLanes], raw[3 * kPcLanes]);
    if (any_unaligned && !c.aligned && k < c.nfull) {
      load_words_any(w, c.src + 64ull * k, 64);
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = bswap(w[q]);
    }
    if (k & 1u) {
      // both slots of pair k/2 are read: refill them with pair k/2 + 2
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      lds2_dma_pair(c, (k >> 1) + 2, wave_lds);
    }
    if (k < c.nfull) compress(s, w);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the wave
  if (i >= p.n) return;
  finish(s, c.src + 64ull * c.nfull, c.size & 63u, c.size);
  write_result(p, i, s);
}
constexpr int kLds2Bytes = 4 * 4 * kPcRawU4 * 16;  // 4 waves x 16 KiB

}  // namespace
}  // namespace lbf
