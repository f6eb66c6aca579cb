// kern_pc.hpp -- producer/consumer kernels for few chains: "pc4" (variant 7,
// one 64-chain group per workgroup, C2) and "pc4x2" (variant 12, two groups per
// workgroup, 16 K-32 K chains, C4 per GPU).  The superseded forms they grew out
// of (pc, pcx2, pc2, pc4 with uint4 or single loads, the pc4x2 diagnostics)
// live in tools/experimental/, outside the shipped library.
//
// Part of the single translation unit sha1_kernels.hip (included from there);
// DESIGN.md §4 has the measurements behind each kernel.
#pragma once

#include <hip/hip_runtime.h>

#include "kern_common.hpp"

namespace lbf {
namespace {

// Producer side shared by pc4 and pc4x2: two producer waves per 64 chains
// alternate block steps (producer X builds steps X, X+2, ...), each staging its
// chains' raw blocks in two 4 KiB LDS slots filled by LDS-DMA.
constexpr int kP2Raw = 2;  // raw slots per producer

// Raw bytes of `step` into raw slot `slot` of this producer: 4 DMA ops always.
__device__ __forceinline__ void p2_dma(const ChainInfo& c, uint32_t step, uint32_t raw_lds, uint32_t slot) {
  const bool ok = c.aligned && step < c.nfull;
  const uint8_t* src = ok ? c.src + 64ull * step : reinterpret_cast<const uint8_t*>(g_pc_dummy);
  const uint32_t base = raw_lds + slot * (kPcRawU4 * 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma16(src + 16 * j, base + j * (kPcLanes * 16));
}

// The 16 message words of `step`: full blocks from the raw slot (aligned) or
// global memory (misaligned), final blocks built from the tail.  Past its last
// block a lane's words are never used: it only zeroes them, so a ragged wave
// pays for the final-block branch only in the steps where some lane really
// builds one.
__device__ __forceinline__ void p2_block(uint32_t (&w)[16], const uint4* raw, const ChainInfo& c, uint32_t step) {
  if (step < c.nfull) {
    if (c.aligned) {
      block_from_vec(w, raw[0], raw[kPcLanes], raw[2 * kPcLanes], raw[3 * kPcLanes]);
    } else {
      load_words_any(w, c.src + 64ull * step, 64);
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap(w[k]);
    }
  } else if (step < c.total) {
    final_block(w, c.src + 64ull * c.nfull, c.size & 63u, c.size, step != c.nfull);
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = 0;
  }
}

// ---------------------------------------------------------------------------
// Kernel "pc4" (variant 7): two producers per 64 chains, with the schedule
// double-buffered in the consumer's registers.
//
// The consumer's round is cheapest (five VALU ops issued back to back) when
// its schedule word already carries the round constant; adding K costs more
// than one producer wave has to spare, so two producers alternate steps, each
// spending two barrier intervals on one (words 0..39, then 40..79).  In the
// form this grew out of (pc2, tools/experimental/) the consumer loaded step k's 80 words after barrier k and its first round
// waits for the first of them: an LDS round trip per step, longer while the
// producers' writes and DMA share the LDS.  Here the producers run one step
// further ahead (step k+1 is complete at barrier k), and right after barrier k
// the consumer loads ALL of step k+1 into a second register set while it runs
// step k from the set it loaded one step earlier.  The loads complete during
// the step, so no round ever waits for LDS.  Fifteen loads go out at once (the
// lgkm counter holds 15) and five more after the fourth quad of rounds.  The
// step loop is unrolled by two so the sets swap roles without copies.
//
// Interval b ends at barrier b.  In interval b producer (b+1) % 2 writes words
// 40..79 of step b+1 and the other one words 0..39 of step b+2; interval 0
// also builds steps 0 and 1 whole.  Step s is in slot s % 4: its first half
// is written after barrier s-3, and the consumer finished loading step s-4
// from that slot before barrier s-4 (3 slots would do; the fourth costs
// nothing and makes the slot index a mask).  LDS 96 KiB: one
// workgroup per CU, so each of the three waves has a SIMD of its own.
// ---------------------------------------------------------------------------
constexpr int kPc4Ring = 4;
// Diagnostic builds only (tools/probe_pc.hip): LBF_PC4_NOBARRIER drops the
// barriers (wrong digests; it isolates what the barriers cost).
#ifdef LBF_PC4_NOBARRIER
#define PC4_SYNC() do {} while (0)
#else
#define PC4_SYNC() __syncthreads()
#endif
constexpr int kPc4LdsBytes = (kPc4Ring * kPcSlotU4 + 2 * kP2Raw * kPcRawU4) * 16;

// One consumer step with the schedule read as 40 ds_read_b64 (variant 7).  A lone
// wave pays ≈96 cycles per block for 20 ds_read_b128 over the same rounds fed
// from registers, and ≈4 for 40 ds_read_b64 (tools/probe_lds_lanes.hip,
// profiles/r01/probe_lds_lanes.log).  The lgkm counter holds 15, so the next
// step's 40 pairs go out in three batches: before round 0, after round 16 and
// after round 40, each batch pinned between the rounds by fences.
// Even batch sizes (14, 14, 12) let the compiler pair every load into a
// ds_read2st64_b64: 20 LDS instructions per step instead of 21 with (15, 13,
// 12) -- 0.1 %, inside the noise (profiles/r02/pc4_even_batches/).
constexpr int kPc5Pairs = 40;
constexpr int kPc5B1 = 14, kPc5B1At = 7;   // pairs 0..13 first; 14..27 after pair 7's rounds
constexpr int kPc5B2 = 28, kPc5B2At = 19;  // pairs 28..39 after pair 19's rounds
// kSplit keeps every load a single ds_read_b64: a memory fence between loads
// stops the compiler from pairing them into ds_read2st64_b64 (which returns
// four VGPRs per lane, like ds_read_b128).
template <bool kSplit>
__device__ __forceinline__ void pc5_load(uint2& dst, const uint2* base, int q) {
  if (kSplit) asm volatile("" ::: "memory");  // the pairing pass does not look across it
  dst = base[q * kPcLanes];
}
template <bool kSplit>
__device__ __forceinline__ void pc5_compress(Digest& s, const uint2 (&cur)[kPc5Pairs], uint2 (&nxt)[kPc5Pairs],
                                             const uint2* next_slot, bool live, bool all_live) {
#pragma unroll
  for (int q = 0; q < kPc5B1; ++q) pc5_load<kSplit>(nxt[q], next_slot, q);
  asm volatile("" : "+v"(s.h[0]), "+v"(s.h[1]), "+v"(s.h[2]), "+v"(s.h[3]), "+v"(s.h[4])::"memory");
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
  for (int q = 0; q < kPc5Pairs; ++q) {
    round_step_wk(2 * q + 0, a, b, c, d, e, cur[q].x);
    round_step_wk(2 * q + 1, a, b, c, d, e, cur[q].y);
    if (q == kPc5B1At || q == kPc5B2At) {
      asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
      const int lo = q == kPc5B1At ? kPc5B1 : kPc5B2;
      const int hi = q == kPc5B1At ? kPc5B2 : kPc5Pairs;
#pragma unroll
      for (int r = lo; r < hi; ++r) pc5_load<kSplit>(nxt[r], next_slot, r);
      // Fencing on e alone is enough to keep the loads here (the fence above
      // pins them after the earlier rounds), and unlike a fence on all five
      // it needs no s_nop after it: C2 3.150 -> 3.140 ms
      // (profiles/r02/pc4_light_fence/).
      asm volatile("" : "+v"(e)::"memory");
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

// The consumer's side of one pc4 step: the 20 KiB slot read as uint2 pairs
// (kVec 2, shipped; loads may pair up into ds_read2st64_b64).  kVec 1 keeps
// every load a single ds_read_b64 and kVec 4 reads uint4 quads: both are
// superseded forms, specialised in tools/experimental/.
template <int kVec>
struct Pc4Sched {
  uint2 v[kPc5Pairs];
  static __device__ __forceinline__ const uint2* col(const uint4* ring, int slot, int lane) {
    return reinterpret_cast<const uint2*>(ring + slot * kPcSlotU4) + lane;
  }
  __device__ __forceinline__ void load_all(const uint2* src) {
#pragma unroll
    for (int q = 0; q < kPc5Pairs; ++q) v[q] = src[q * kPcLanes];
  }
};
template <int kVec>
__device__ __forceinline__ void pc4_step(Digest& s, const Pc4Sched<kVec>& cur, Pc4Sched<kVec>& nxt,
                                         const uint2* next_slot, bool live, bool all_live) {
  pc5_compress<kVec == 1>(s, cur.v, nxt.v, next_slot, live, all_live);
}

// Producer side: half kHalf of step `step` into its slot, in the kVec layout.
template <int kVec, int kHalf>
__device__ __forceinline__ void pc4_store_half(uint32_t (&w)[16], uint4* ring, uint32_t step, int lane) {
  uint4* slot = ring + (step % 4) * kPcSlotU4;
  if (kVec == 4) expand_store_wk<kHalf>(w, slot + lane, kPcLanes);
  else expand_store_wk2<kHalf>(w, reinterpret_cast<uint2*>(slot) + lane, kPcLanes);
}

// A barrier the consumer's rounds cannot cross: the compiler may otherwise move
// register-only round code over __syncthreads (it orders memory only), which
// put a barrier right behind a fresh batch of loads and made it wait for them.
#ifdef LBF_PC_STAMPS
#define PC4_ACC_ARGS , unsigned long long (&acc)[4]
#else
#define PC4_ACC_ARGS
#endif
__device__ __forceinline__ void pc4_barrier(Digest& s PC4_ACC_ARGS) {
  asm volatile("" : "+v"(s.h[0]), "+v"(s.h[1]), "+v"(s.h[2]), "+v"(s.h[3]), "+v"(s.h[4])::"memory");
#ifdef LBF_PC_STAMPS
  unsigned long long t0 = 0, t1 = 0;
  PC_STAMP(t0);
#endif
  PC4_SYNC();
#ifdef LBF_PC_STAMPS
  PC_STAMP(t1);
  PC_ACC(0, t0, t1);
#endif
  asm volatile("" : "+v"(s.h[0]), "+v"(s.h[1]), "+v"(s.h[2]), "+v"(s.h[3]), "+v"(s.h[4])::"memory");
}

// kUnroll: steps per fast-loop iteration.  Eight since round 3: 0.3-1.1 %
// faster than four at C2 in alternating runs (profiles/r03/pc4x2/diag/sweep_7_16_*.jsonl).
// The producers run at the default wave priority: raising either one's
// (s_setprio 1-3) measured 0.1-0.5 %, below the box-to-box noise
// (profiles/r03/pc4x2/prio/).
template <bool kUniform, int kVec, int kUnroll = 8>
__global__ void __launch_bounds__(192) sha1_pc4_kernel(ChunkParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 ring[];  // W[3][20][64] | raw[2][2][4][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t i = blockIdx.x * kPcLanes + lane;
  const ChainInfo c = chain_info<kUniform>(p, i);
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane(wave_max(c.total));
#ifdef LBF_PC_STAMPS
  unsigned long long acc[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0, t2 = 0;
#define PC4_ACC , acc
#else
#define PC4_ACC
#endif

  if (wave != 0) {
    // ---------------- producer X = wave - 1: steps X, X+2, ... ----------------
    const uint32_t X = wave - 1;
    uint4* raw = ring + kPc4Ring * kPcSlotU4 + X * (kP2Raw * kPcRawU4);
    const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(raw);
    p2_dma(c, X, raw_lds, 0);
    p2_dma(c, X + 2, raw_lds, 1);
    uint32_t w[16];
    // words 0..39 of this producer's step `step` (its j-th); the raw slot is
    // refilled with step + 4
    auto first_half = [&](uint32_t step) {
      const uint32_t j = (step - X) >> 1;
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // block j landed; only j+1's DMAs pending
      p2_block(w, raw + (j & 1u) * kPcRawU4 + lane, c, step);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // raw slot read before it is refilled
      p2_dma(c, step + 4, raw_lds, j & 1u);
      pc4_store_half<kVec, 0>(w, ring, step, lane);
    };
    for (uint32_t b = 0; b < nsteps; ++b) {
      PC_STAMP(t0);
      if (b == 0 && X == 0) {  // prologue: step 0 whole
        first_half(0);
        pc4_store_half<kVec, 1>(w, ring, 0, lane);
      }
      const uint32_t fin = b + 1;  // finished in interval b by producer fin % 2
      if ((fin & 1u) == X && fin < nsteps) {
        if (b == 0) first_half(fin);
        pc4_store_half<kVec, 1>(w, ring, fin, lane);
      }
      const uint32_t start = b + 2;  // started in interval b by producer start % 2
      if ((start & 1u) == X && start < nsteps) first_half(start);
      PC_STAMP(t1);
      PC4_SYNC();  // barrier b: steps <= b + 1 complete
      PC_STAMP(t2);
      PC_ACC(1, t0, t1);
      PC_ACC(2, t1, t2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  } else {
    // ---------------- consumer ----------------
    // (No s_setprio here: the consumer is wave 0, the oldest, and priority 3
    // measured 0.3-0.6 % slower; profiles/r03/pc4x2/prio/.)
    Digest s;
    s.init();
    Pc4Sched<kVec> A, B;
    // steps every chain of the workgroup has (inactive lanes count as having all)
    const uint32_t min_steps =
        __builtin_amdgcn_readfirstlane(wave_min(i < p.n ? c.total : 0xFFFFFFFFu));
    if (nsteps > 0) {
      PC4_SYNC();  // barrier 0: steps 0 and 1 complete
      A.load_all(Pc4Sched<kVec>::col(ring, 0, lane));
      // Once, so that the loop's first rounds need no wait on either path into
      // it (otherwise every iteration waits for its own first load).
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0)
    }
    uint32_t k = 0;
    // kUnroll steps per iteration while every chain of the workgroup is running
    // and every step is followed by a barrier: k % 4 == 0, so the slots are
    // compile-time offsets and the steps need no liveness checks.  The two
    // conditions are folded into one bound, so the loop test is one scalar
    // compare (the compiler built the conjunction from 7 scalar ops).
    const uint32_t fast_end = __builtin_amdgcn_readfirstlane(nsteps ? min(min_steps, nsteps - 1) : 0u);
    static_assert(kUnroll % 4 == 0, "the fast loop keeps k % 4 == 0");
    for (; k + kUnroll <= fast_end; k += kUnroll) {
#pragma unroll
      for (int j = 0; j < kUnroll; j += 2) {
        pc4_step(s, A, B, Pc4Sched<kVec>::col(ring, (j + 1) % 4, lane), true, true);
        pc4_barrier(s PC4_ACC);  // barrier k+j+1
        pc4_step(s, B, A, Pc4Sched<kVec>::col(ring, (j + 2) % 4, lane), true, true);
        pc4_barrier(s PC4_ACC);  // barrier k+j+2
      }
    }
    for (; k < nsteps; k += 2) {
      // after barrier k: steps <= k+1 complete; A holds step k
      pc4_step(s, A, B, Pc4Sched<kVec>::col(ring, (k + 1) % kPc4Ring, lane), k < c.total, k < min_steps);
      if (k + 1 >= nsteps) break;
      pc4_barrier(s PC4_ACC);  // barrier k+1
      pc4_step(s, B, A, Pc4Sched<kVec>::col(ring, (k + 2) % kPc4Ring, lane), k + 1 < c.total, k + 1 < min_steps);
      if (k + 2 >= nsteps) break;
      pc4_barrier(s PC4_ACC);  // barrier k+2
    }
    if (i < p.n) write_result(p, i, s);
  }
#ifdef LBF_PC_STAMPS
  if (lane == 0) {
    unsigned long long* o = g_pc_stamps + (blockIdx.x * 3 + wave) * 4;
    o[0] = acc[0];  // consumer: cycles at barriers
    o[1] = acc[1];  // producer: work
    o[2] = acc[2];  // producer: barrier
    o[3] = nsteps;
  }
#endif
#undef PC4_ACC
}

// ---------------------------------------------------------------------------
// Kernel "pc4x2" (variant 12): two pc4 groups in one 6-wave workgroup, for
// 16 K-32 K chains (C4 per GPU).
//
// pcx5 gives each of a CU's two consumers one producer, because the waves of
// a CU must each own a SIMD; one producer cannot add all 80 round constants
// and store 20 KiB per step in time, so pcx5's consumers add K themselves in
// 64 rounds (the two-add3 round, ≈2.65 cycles more each).  Two producers CAN
// share a SIMD: one wave's LDS stores drain while the other issues its VALU,
// so two half steps on one SIMD take ≈1,440 cycles against ≈1,045 for one
// alone (tools/probe_shared_producers.hip).  Waves k and k+4 of a workgroup
// land on the same SIMD, so here waves 2 and 3 are the two consumers, each
// alone on its SIMD, and waves 0, 1 (group 0) and 4, 5 (group 1) are the
// producers, two to a SIMD.  Each group is pc4 unchanged (steps alternate
// between its two producers, the consumer runs W+K rounds and double-buffers
// the next step in registers), except that the W ring has 3 slots instead of
// 4 so that both groups fit 160 KiB of LDS: step s goes into slot s % 3 after
// barrier s-3, and the consumer's loads of step s-3 from that slot were
// issued in its step s-4 and drained by the s_waitcnt lgkmcnt(0) that opens
// barrier s-3 (step 0 is loaded before an extra barrier that ends the
// prologue).  Both groups pass the same barriers, so every wave counts the
// steps of both groups' chains.  LDS 152 KiB: one workgroup per CU.
// The consumers raise their wave priority (s_setprio 3): they are younger than
// the producers of waves 0 and 1, and the CU's arbiter serves older waves
// first -- with the priority C4 went from 13.76-13.80 to 13.10-13.11 ms
// (experimental variant 22 against 12, profiles/r03/pc4x2/prio/).  Group 1's
// producers (waves 4 and 5, the younger of each producer pair on a SIMD) then
// run at priority 1, which breaks the age order between the two producers of
// a SIMD: 13.07 -> 12.92 ms at C4, 1.1-1.5 % at every size (experimental
// variant 25 against 12, profiles/r03/pc4x2/prio/s31_*).
// ---------------------------------------------------------------------------
constexpr int kPc4x2Ring = 3;
constexpr int kPc4x2GroupU4 = kPc4x2Ring * kPcSlotU4 + 2 * kP2Raw * kPcRawU4;
constexpr int kPc4x2LdsBytes = 2 * kPc4x2GroupU4 * 16;

template <int kHalf>
__device__ __forceinline__ void pc4x2_store_half(uint32_t (&w)[16], uint4* ring, uint32_t step, int lane) {
#if defined(LBF_X2_DIAG) && LBF_X2_DIAG == 2
  // diagnostic build (tools/probe_pc.hip): the schedule without its LDS stores
#pragma unroll
  for (int i = 16 * kHalf; i < 16 * kHalf + 16; ++i) {
    w[i & 15] = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]) + round_k(i);
    asm volatile("" ::"v"(w[i & 15]));
  }
  (void)ring, (void)step, (void)lane;
#else
  // The slot's byte offset goes through an empty asm: folded into the lane's
  // address, the compiler addressed the words with negative offsets from a
  // shifted base and left every store unpaired (40 ds_write_b64 per step
  // instead of 20 ds_write2st64_b64), which slowed the consumers' reads by 6 %
  // (C2 with one group, experimental variant 13).
  uint32_t slot_off = (step % kPc4x2Ring) * (kPcSlotU4 * 16);
  asm volatile("" : "+s"(slot_off));
  expand_store_wk2<kHalf>(w, reinterpret_cast<uint2*>(reinterpret_cast<char*>(ring) + slot_off) + lane, kPcLanes);
#endif
}

// kGroups = 1 (experimental variant 13, a diagnostic): one group of three
// waves, 64 chains per workgroup -- pc4 with pc4x2's 3-slot ring and six-step
// loop, to tell the cost of that structure from the cost of a second group.
// kFast = false (experimental variants 14, 15, diagnostics): no six-step loop,
// every step through the generic two-step loop with runtime slot offsets.
// kRawAt (experimental variant 17, a diagnostic): where the raw slots start, in
// W slots from the group's base (pc4's layout has them at 4).
// kFence (experimental variants 18, 19, diagnostics): scheduling barriers
// around the producers' workgroup barrier, as the stamped build has them.
// kUnroll6 (a multiple of 6): steps per fast-loop iteration (12: experimental variant 21).
// kPrio (experimental variants 22, 23, diagnostics): the consumers raise their
// wave priority (s_setprio 3) so the CU's arbiter serves them before producers.
// kPrioG0, kPrioG1: wave priority of group 0's / group 1's producers (0, 1 in
// the shipped kernel since experimental variant 25; variants 26-28 try others).
template <bool kUniform, int kGroups, bool kFast, int kRawAt, bool kFence, int kUnroll6, bool kPrio = false,
          int kPrioG0 = 0, int kPrioG1 = 0>
__device__ __forceinline__ void pc4x2_body(const ChunkParams& p) {
  static_assert(kUnroll6 % 6 == 0, "the fast loop keeps k % 6 == 0");
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // group 0 | group 1: W[3][20][64] | raw[2][2][4][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = wave < 3 ? 0 : 1;
  const uint32_t first = blockIdx.x * (kGroups * kPcLanes);
  const uint32_t i = first + g * kPcLanes + lane;
  const ChainInfo c = chain_info<kUniform>(p, i);
  const uint32_t other = kGroups == 2 ? chain_info<kUniform>(p, first + (1 - g) * kPcLanes + lane).total : 0u;
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane(max(wave_max(c.total), wave_max(other)));
  uint4* ring = lds + g * kPc4x2GroupU4;
#ifdef LBF_PC_STAMPS
  unsigned long long acc[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0, t2 = 0;
#define PC4_ACC , acc
#else
#define PC4_ACC
#endif
#if defined(LBF_X2_DIAG) && LBF_X2_DIAG == 1
  // diagnostic build (tools/probe_pc.hip): group 1 only passes the barriers
  if (g == 1) {
    for (uint32_t b = 0; b < nsteps + (nsteps > 0); ++b) __syncthreads();
    return;
  }
#endif

  if (wave != 2 && wave != 3) {
    // ---------------- producer X of group g: steps X, X+2, ... ----------------
    if (kPrioG0 != 0 && g == 0) __builtin_amdgcn_s_setprio(kPrioG0);
    if (kPrioG1 != 0 && g == 1) __builtin_amdgcn_s_setprio(kPrioG1);
    const uint32_t X = g == 0 ? wave : wave - 4;
    uint4* raw = ring + kRawAt * kPcSlotU4 + X * (kP2Raw * kPcRawU4);
    const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(raw);
    p2_dma(c, X, raw_lds, 0);
    p2_dma(c, X + 2, raw_lds, 1);
    uint32_t w[16];
    auto first_half = [&](uint32_t step) {
      const uint32_t j = (step - X) >> 1;
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");  // block j landed; only j+1's DMAs pending
      p2_block(w, raw + (j & 1u) * kPcRawU4 + lane, c, step);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // raw slot read before it is refilled
      p2_dma(c, step + 4, raw_lds, j & 1u);
      pc4x2_store_half<0>(w, ring, step, lane);
    };
    if (nsteps > 0) {
      // prologue: step X whole, then barrier E (see the consumer)
      if (X < nsteps) {
        first_half(X);
        pc4x2_store_half<1>(w, ring, X, lane);
      }
      PC4_SYNC();  // barrier E: steps 0 and 1 complete
    }
    for (uint32_t b = 0; b < nsteps; ++b) {
      PC_STAMP(t0);
      const uint32_t fin = b + 1;  // finished in interval b by producer fin % 2 (step 1: in the prologue)
      if ((fin & 1u) == X && fin < nsteps && b > 0) pc4x2_store_half<1>(w, ring, fin, lane);
      const uint32_t start = b + 2;  // started in interval b by producer start % 2
      if ((start & 1u) == X && start < nsteps) first_half(start);
      PC_STAMP(t1);
      if (kFence) __builtin_amdgcn_sched_barrier(0);
      PC4_SYNC();  // barrier b: steps <= b + 1 complete
      if (kFence) __builtin_amdgcn_sched_barrier(0);
      PC_STAMP(t2);
      PC_ACC(1, t0, t1);
      PC_ACC(2, t1, t2);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  } else {
    // ---------------- consumer of group g ----------------
    if (kPrio) __builtin_amdgcn_s_setprio(3);
    Digest s;
    s.init();
    Pc4Sched<2> A, B;
    const uint32_t min_steps =
        __builtin_amdgcn_readfirstlane(wave_min(i < p.n ? c.total : 0xFFFFFFFFu));
    if (nsteps > 0) {
      // With 3 slots, step 3's first half goes into slot 0 in interval 1, so
      // step 0 must be loaded out of slot 0 before barrier 0: an extra barrier
      // E ends the prologue, in which the producers build steps 0 and 1 whole.
      PC4_SYNC();  // barrier E: steps 0 and 1 complete
      A.load_all(Pc4Sched<2>::col(ring, 0, lane));
      __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): slot 0 is free from barrier 0 on
      pc4_barrier(s PC4_ACC);  // barrier 0
    }
    uint32_t k = 0;
    // Six steps per iteration (the A/B register sets and the 3-slot ring both
    // come back to where they started), slots as compile-time offsets.
    const uint32_t fast_end = __builtin_amdgcn_readfirstlane(nsteps && kFast ? min(min_steps, nsteps - 1) : 0u);
    for (; k + kUnroll6 <= fast_end; k += kUnroll6) {
#pragma unroll
      for (int j = 0; j < kUnroll6; j += 2) {
        pc4_step(s, A, B, Pc4Sched<2>::col(ring, (j + 1) % kPc4x2Ring, lane), true, true);
        pc4_barrier(s PC4_ACC);  // barrier k+j+1
        pc4_step(s, B, A, Pc4Sched<2>::col(ring, (j + 2) % kPc4x2Ring, lane), true, true);
        pc4_barrier(s PC4_ACC);  // barrier k+j+2
      }
    }
    for (; k < nsteps; k += 2) {
      // after barrier k: steps <= k+1 complete; A holds step k
      pc4_step(s, A, B, Pc4Sched<2>::col(ring, (k + 1) % kPc4x2Ring, lane), k < c.total, k < min_steps);
      if (k + 1 >= nsteps) break;
      pc4_barrier(s PC4_ACC);  // barrier k+1
      pc4_step(s, B, A, Pc4Sched<2>::col(ring, (k + 2) % kPc4x2Ring, lane), k + 1 < c.total, k + 1 < min_steps);
      if (k + 2 >= nsteps) break;
      pc4_barrier(s PC4_ACC);  // barrier k+2
    }
    if (i < p.n) write_result(p, i, s);
  }
#ifdef LBF_PC_STAMPS
  if (lane == 0) {
    unsigned long long* o = g_pc_stamps + (blockIdx.x * 6 + wave) * 4;
    o[0] = acc[0];
    o[1] = acc[1];
    o[2] = acc[2];
    o[3] = nsteps;
  }
#endif
#undef PC4_ACC
}

// The shipped kernel (variant 12).
template <bool kUniform>
__global__ void __launch_bounds__(384) sha1_pc4x2_kernel(ChunkParams p) {
  pc4x2_body<kUniform, 2, true, kPc4x2Ring, false, 6, true, 0, 1>(p);
}

}  // namespace
}  // namespace lbf
