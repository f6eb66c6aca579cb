// kern_pcx.hpp -- two producer/consumer pairs per workgroup pinned to its
// CU, one producer each, for 16 K-32 K chains: "pcx5" (10), kept for A/B
// against pc4x2 (12); the "pcx4" (9) it grew out of is in tools/experimental/.
//
// Part of the single translation unit sha1_kernels.hip (included from there);
// DESIGN.md §4 has the measurements behind each kernel.
#pragma once

#include <hip/hip_runtime.h>

#include "kern_pc.hpp"

namespace lbf {
namespace {

// ---------------------------------------------------------------------------
// Kernel "pcx4" (variant 9): two pc4-style pairs per workgroup, one workgroup
// per CU, for 16 K-32 K chains (C4 per GPU: 32,768 x 1 MiB).
//
// Two 64-chain pairs share a CU: waves 0/1 consume, waves 2/3 produce, and
// every wave owns a SIMD (112 KiB of LDS pins one workgroup per CU).  With one
// producer per consumer the producer is the tighter side: a whole step of
// W+K costs it ≈2,000 cycles, ≈690 of them for the 20 KiB of ds_write
// (tools/probe_producer.hip), against ≈1,810 for a pc4 consumer.  So the work
// is split: the consumer adds K itself in rounds 0..kKFrom-1 (two-add3 round,
// ≈2.8 cycles more per round, K in VGPRs) and the producer adds it to words
// kKFrom..79 only.  The consumer double-buffers the schedule in registers like
// pc4 and reads it as 8-byte pairs in three batches (variant 7).
//
// Ring: 2 slots per pair, step s in slot s % 2.  Invariant at barrier k
// (k >= 0): steps <= k+1 are complete and the consumer has step k in
// registers.  In interval k+1 the consumer runs step k and loads step k+1;
// the producer writes step k+2 into slot k % 2, which the consumer finished
// loading before barrier k.  The prologue therefore has one extra barrier P:
// producers build steps 0 and 1 before P, consumers load step 0 between P
// and barrier 0 while the producers wait.  Raw blocks: 4 DMA slots per
// producer, issued 4 steps ahead.
// ---------------------------------------------------------------------------
constexpr int kPx4Ring = 2;

template <int kKFrom>
__device__ __forceinline__ void px4_round(int i, uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                          uint32_t x, const RoundK& K) {
  if (i < kKFrom) round_step_kv(i, a, b, c, d, e, x, K);
  else round_step_wk(i, a, b, c, d, e, x);
}

// ---------------------------------------------------------------------------
// Kernel "pcx5" (variant 10): pcx4 with the producer's first 16 words left in
// the raw block.
//
// pcx4 is producer-bound (≈2,170 cycles per step); ≈690 of a producer's
// cycles are its 20 KiB of stores.  Words 0..15 of a step are the chunk's own
// 64 bytes, already in LDS from the DMA, so the consumer reads them there
// (4 ds_read_b128 of the raw slot); the producer stores words 16..79 (16 KiB)
// and writes words 0..15 back over the raw block byte-swapped (4 KiB), so the
// consumer issues no v_perm: pcx5 is consumer-bound, and moving the 16 swaps
// to the producer took C4 from 14.00 to 13.69 ms (profiles/r02/px5_be).  For
// final and misaligned blocks those words are the ones the producer built, so
// the consumer's read is the same for every step.  The consumer's load count
// stays at 20 instructions per step.
//
// Raw slots: 6 per pair, block s in slot s % 6.  The consumer reads block s in
// interval s (like the words of step s), so the slot is refilled only when
// the producer builds step s + 2 (interval s + 1): block s + 6 is requested
// then, four steps ahead of its use (vmcnt(12) before each build).
// ---------------------------------------------------------------------------
constexpr int kPx5Raw = 6;
constexpr int kPx5SlotU4 = 32 * kPcLanes / 2;                              // 16 KiB: 32 pairs x 64 lanes
constexpr int kPx5PairU4 = kPx4Ring * kPx5SlotU4 + kPx5Raw * kPcRawU4;     // 56 KiB per pair
constexpr int kPx5LdsBytes = 2 * kPx5PairU4 * 16;                          // 112 KiB
constexpr int kPx5B1 = 14, kPx5B1At = 7;   // raw + pairs 0..13 first; 14..23 after round 16
constexpr int kPx5B2 = 24, kPx5B2At = 19;  // pairs 24..31 after round 40

struct Px5Sched {
  uint4 raw[4];  // words 0..15, big-endian (swapped by the producer)
  uint2 v[32];   // words 16..79
};

__device__ __forceinline__ void px5_load_all(Px5Sched& d, const uint4* raw, const uint2* pairs) {
#pragma unroll
  for (int j = 0; j < 4; ++j) d.raw[j] = raw[j * kPcLanes];
#pragma unroll
  for (int q = 0; q < 32; ++q) d.v[q] = pairs[q * kPcLanes];
}

template <int kKFrom>
__device__ __forceinline__ void px5_compress(Digest& s, const Px5Sched& cur, Px5Sched& nxt, const uint4* next_raw,
                                             const uint2* next_pairs, const RoundK& K, bool live, bool all_live) {
#pragma unroll
  for (int j = 0; j < 4; ++j) nxt.raw[j] = next_raw[j * kPcLanes];
#pragma unroll
  for (int q = 0; q < kPx5B1; ++q) nxt.v[q] = next_pairs[q * kPcLanes];
  asm volatile("" : "+v"(s.h[0]), "+v"(s.h[1]), "+v"(s.h[2]), "+v"(s.h[3]), "+v"(s.h[4])::"memory");
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    px4_round<kKFrom>(4 * j + 0, a, b, c, d, e, cur.raw[j].x, K);
    px4_round<kKFrom>(4 * j + 1, a, b, c, d, e, cur.raw[j].y, K);
    px4_round<kKFrom>(4 * j + 2, a, b, c, d, e, cur.raw[j].z, K);
    px4_round<kKFrom>(4 * j + 3, a, b, c, d, e, cur.raw[j].w, K);
  }
#pragma unroll
  for (int q = 0; q < 32; ++q) {
    px4_round<kKFrom>(16 + 2 * q, a, b, c, d, e, cur.v[q].x, K);
    px4_round<kKFrom>(17 + 2 * q, a, b, c, d, e, cur.v[q].y, K);
    if (q == kPx5B1At || q == kPx5B2At) {
      asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
      const int lo = q == kPx5B1At ? kPx5B1 : kPx5B2;
      const int hi = q == kPx5B1At ? kPx5B2 : 32;
#pragma unroll
      for (int r = lo; r < hi; ++r) nxt.v[r] = next_pairs[r * kPcLanes];
      // (all five operands: fencing on e alone, as pc5_compress does, dropped the
      // s_nop after it but cost C4 1.1 %, profiles/r02/pc4_light_fence/c4/)
      asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
    }
  }
  if (all_live) {
    s.h[0] += a;
    s.h[1] += b;
    s.h[2] += c;
    s.h[3] += d;
    s.h[4] += e;
  } else {
    s.h[0] = live ? s.h[0] + a : s.h[0];
    s.h[1] = live ? s.h[1] + b : s.h[1];
    s.h[2] = live ? s.h[2] + c : s.h[2];
    s.h[3] = live ? s.h[3] + d : s.h[3];
    s.h[4] = live ? s.h[4] + e : s.h[4];
  }
}

// Raw bytes of `block` into raw slot block % 6 of this pair: 4 DMA ops always.
__device__ __forceinline__ void px5_dma(const ChainInfo& c, uint32_t block, uint32_t raw_lds) {
  const bool ok = c.aligned && block < c.nfull;
  const uint8_t* src = ok ? c.src + 64ull * block : reinterpret_cast<const uint8_t*>(g_pc_dummy);
  const uint32_t slot = raw_lds + (block % kPx5Raw) * (kPcRawU4 * 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma16(src + 16 * j, slot + j * (kPcLanes * 16));
}

template <int kKFrom>
__device__ __forceinline__ void px5_produce(uint4* ring, uint32_t raw_lds, const ChainInfo& c, uint32_t step,
                                            int lane) {
  uint32_t w[16];
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // block `step` landed; steps +1..+3 pending
  uint4* raw = ring + kPx4Ring * kPx5SlotU4 + (step % kPx5Raw) * kPcRawU4 + lane;
  if (c.aligned && step < c.nfull) {
    block_from_vec(w, raw[0], raw[kPcLanes], raw[2 * kPcLanes], raw[3 * kPcLanes]);
  } else if (step < c.nfull) {
    load_words_any(w, c.src + 64ull * step, 64);
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = bswap(w[k]);
  } else {
    // (zeroing the words of lanes past their last block instead, as p2_block
    // does, cost C4 0.6 %: profiles/r02/idle_lanes/)
    final_block(w, c.src + 64ull * c.nfull, c.size & 63u, c.size, step != c.nfull);
  }
  // The consumer reads words 0..15 of every step from the raw slot: the
  // producer leaves them there byte-swapped (big-endian), so the consumer,
  // the side that bounds pcx5, issues no v_perm (4 KiB more of producer
  // stores, which it has the slack for: DESIGN.md §4.3f).
#pragma unroll
  for (int j = 0; j < 4; ++j) raw[j * kPcLanes] = make_uint4(w[4 * j], w[4 * j + 1], w[4 * j + 2], w[4 * j + 3]);
  px5_dma(c, step + kPx5Raw - 2, raw_lds);  // into the slot of block step - 2, read before barrier step - 2
  expand_store_from16<kKFrom>(w, reinterpret_cast<uint2*>(ring + (step % kPx4Ring) * kPx5SlotU4) + lane, kPcLanes);
}

template <bool kUniform, int kKFrom>
__global__ void __launch_bounds__(256) sha1_pcx5_kernel(ChunkParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds_all[];  // per pair: W[2][32][64] uint2 | raw[6][4][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave & 1;
  uint4* ring = lds_all + pair * kPx5PairU4;
  uint4* raw_base = ring + kPx4Ring * kPx5SlotU4;
  const uint32_t i = blockIdx.x * (2 * kPcLanes) + pair * kPcLanes + lane;
  const ChainInfo c = chain_info<kUniform>(p, i);
  __shared__ uint32_t wg_steps;
  if (threadIdx.x == 0) wg_steps = 0;
  __syncthreads();
  const uint32_t mine = __builtin_amdgcn_readfirstlane(wave_max(c.total));
  if (lane == 0) atomicMax(&wg_steps, mine);
  __syncthreads();
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane(wg_steps);
  if (nsteps == 0) return;  // uniform over the workgroup

#ifdef LBF_PC_STAMPS
  unsigned long long acc[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0, t2 = 0;
#endif
  if (wave >= 2) {
    // ---------------- producer ----------------
    const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(raw_base);
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kPx5Raw - 2; ++r) px5_dma(c, r, raw_lds);
    px5_produce<kKFrom>(ring, raw_lds, c, 0, lane);
    if (nsteps > 1) px5_produce<kKFrom>(ring, raw_lds, c, 1, lane);
    __syncthreads();  // barrier P: steps 0 and 1 complete
    __syncthreads();  // barrier 0: the consumers hold step 0
    for (uint32_t k = 0; k + 1 < nsteps; ++k) {
      PC_STAMP(t0);
      if (k + 2 < nsteps) px5_produce<kKFrom>(ring, raw_lds, c, k + 2, lane);
      PC_STAMP(t1);
      __syncthreads();  // barrier k+1
      PC_STAMP(t2);
      PC_ACC(1, t0, t1);  // producer: work (incl. its vmcnt wait)
      PC_ACC(2, t1, t2);  // producer: barrier
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  } else {
    // ---------------- consumer ----------------
    Digest s;
    s.init();
    const RoundK K;
    Px5Sched A, B;
#ifdef LBF_PC_STAMPS
#define PX5_ACC , acc
#else
#define PX5_ACC
#endif
    const uint2* pairs0 = reinterpret_cast<const uint2*>(ring) + lane;
    const uint2* pairs1 = reinterpret_cast<const uint2*>(ring + kPx5SlotU4) + lane;
    const uint32_t min_steps = __builtin_amdgcn_readfirstlane(wave_min(i < p.n ? c.total : 0xFFFFFFFFu));
    __syncthreads();  // barrier P
    px5_load_all(A, raw_base + lane, pairs0);
    __syncthreads();  // barrier 0 (its fence completes the loads)
    uint32_t k = 0;
    // six steps per iteration (lcm of the 2 register sets, 2 W slots and 6 raw
    // slots) while every chain runs and each step is followed by a barrier
    // (folding this test into one bound, as pc4 does, cost C4 2.4 %: the compiler
    // scheduled the loop differently, profiles/r02/pc4_loop_bound/c4/)
    for (; k + 6 <= min_steps && k + 6 < nsteps; k += 6) {
#pragma unroll
      for (int u = 0; u < 6; u += 2) {
        px5_compress<kKFrom>(s, A, B, raw_base + ((u + 1) % kPx5Raw) * kPcRawU4 + lane, pairs1, K, true, true);
        pc4_barrier(s PX5_ACC);
        px5_compress<kKFrom>(s, B, A, raw_base + ((u + 2) % kPx5Raw) * kPcRawU4 + lane, pairs0, K, true, true);
        pc4_barrier(s PX5_ACC);
      }
    }
    for (; k < nsteps; k += 2) {
      px5_compress<kKFrom>(s, A, B, raw_base + ((k + 1) % kPx5Raw) * kPcRawU4 + lane, pairs1, K, k < c.total,
                           k < min_steps);
      if (k + 1 >= nsteps) break;
      pc4_barrier(s PX5_ACC);  // barrier k+1
      px5_compress<kKFrom>(s, B, A, raw_base + ((k + 2) % kPx5Raw) * kPcRawU4 + lane, pairs0, K, k + 1 < c.total,
                           k + 1 < min_steps);
      if (k + 2 >= nsteps) break;
      pc4_barrier(s PX5_ACC);  // barrier k+2
    }
    if (i < p.n) write_result(p, i, s);
#undef PX5_ACC
  }
#ifdef LBF_PC_STAMPS
  if (lane == 0) {  // [wg][wave][0..3]: consumer {barrier wait, -, -, steps}; producer {-, work, barrier, steps}
    unsigned long long* o = g_pc_stamps + (blockIdx.x * 4 + wave) * 4;
    o[0] = acc[0];
    o[1] = acc[1];
    o[2] = acc[2];
    o[3] = nsteps;
  }
#endif
}

// K split for pcx5: the consumer adds K in rounds 0..63.  With the producer's
// stores down to 16 KiB the two sides balance near there: splitting at 40 ran
// 2 % slower, 48 and 56 within 0.5 % (profiles/r01/sweep_v9_pcx5_k40_k48.log,
// sweep_pcx5_k48_k56_k64.log); 72 ran 1.5 % and 80 (no K in the producer)
// 5 % slower (sweep_pcx5_k64_k72_k80.log).
#ifndef LBF_PX5_KFROM  // A/B builds only (tools/px5_ab.sh)
#define LBF_PX5_KFROM 64
#endif
constexpr int kPx5KFrom = LBF_PX5_KFROM;

template <int kKFrom>
void launch_pcx5(const ChunkParams& p, hipStream_t stream) {
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pcx5_kernel<false, kKFrom>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kPx5LdsBytes);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pcx5_kernel<true, kKFrom>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kPx5LdsBytes);
  });
  const uint32_t blocks = (p.n + 2 * kPcLanes - 1) / (2 * kPcLanes);
  if (p.offsets) hipLaunchKernelGGL((sha1_pcx5_kernel<false, kKFrom>), dim3(blocks), dim3(256), kPx5LdsBytes, stream, p);
  else hipLaunchKernelGGL((sha1_pcx5_kernel<true, kKFrom>), dim3(blocks), dim3(256), kPx5LdsBytes, stream, p);
}

}  // namespace
}  // namespace lbf
