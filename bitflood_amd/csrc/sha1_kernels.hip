// sha1_kernels.hip -- MI355X (gfx950) chunk-hash kernels and their launchers.
//
// Replaces the per-chunk hash of Encoder::EncodeFile
// (/root/reference/cpp/src/Encoder.cpp:54-72 -> Base64Encode :107-120) and the
// verify hashes of Flood.cpp:259-275 / ChunkMethods.cpp:116-123,165-167 with
// one batched launch over many independent chunks.
//
// Kernel "lane" (variant 1): one chunk per lane.  SHA-1 is a serial
// Merkle-Damgard chain, so the only parallelism is across chunks; each lane
// keeps its chain state and the 16-word schedule in VGPRs, streams its chunk
// with 16-byte global loads two blocks ahead of use, and finishes the 0x80/
// length padding in registers.  See DESIGN.md for the roofline discussion.
// Kernel "pc" (variant 2): producer/consumer split for few chains.
// Kernel "lds" (variant 3): variant 1 with LDS-DMA staging, for many chains.
// Kernel "pc2" (variant 4): one consumer + two producers, W+K hand-over, for few chains.
// Kernel "pcx2" (variant 5): two pc pairs in one workgroup pinned to its CU, for 16-32 K chains.
// Kernel "pc4" (variant 6): pc2 with the schedule double-buffered in registers, for <= 16 K chains.
// Kernel "pc4/b64" (variants 7, 8): pc4 with the schedule read as uint2 pairs (8: one ds_read_b64 each).
// Kernel "pcx4" (variant 9): two pc4-style pairs per CU, one producer each, K split, for 16-32 K chains.
// Kernel "pcx5" (variant 10): pcx4 with words 0..15 taken by the consumer from the raw block, for 16-32 K chains.
// Kernel "lds2" (variant 11): lds fetching whole 128-byte lines per lane, for > 32 K chains.
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>

#include "lbf_internal.hpp"
#include "sha1_device.hpp"

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
// Kernel "pc" (variant 2): producer/consumer split for few chains.
//
// With few chunks (C2: 16,384 chains = 256 waves for 1,024 SIMDs) a lone wave
// issues at most one VALU every ~4 cycles (tools/probe_issue.hip), so the time
// per chunk is set by the instruction count of ONE chain.  The 64-word message
// expansion and the byte swaps do not depend on the chain state, so a producer
// wave on another SIMD computes them and hands the 80 expanded words per block
// over in LDS; the consumer wave runs only the 80 rounds (5 VALU each).
//
// One workgroup = 64 chains = 2 waves: wave 0 consumes, wave 1 produces.  The
// LDS ring has 2 slots of [20 uint4][64 lanes] (20 KiB each); one workgroup
// barrier per block step separates "producer writes slot k+1" from "consumer
// reads slot k".  The producer keeps kPcPrefetch blocks of raw chunk bytes in
// flight in registers.  Final (padding/length) blocks are built by the
// producer as ordinary steps, so the consumer loop is uniform.
// ---------------------------------------------------------------------------
constexpr int kPcLanes = 64;
constexpr int kPcQuads = 20;                       // 80 words per block step
constexpr int kPcSlotU4 = kPcQuads * kPcLanes;     // uint4 per W slot (20 KiB)
constexpr int kPcRawSlots = 4;                     // raw blocks in flight: steps k..k+3
constexpr int kPcRawU4 = 4 * kPcLanes;             // uint4 per raw slot (4 KiB)
// LDS: kRing W slots (20 KiB each) then 4 raw slots (4 KiB each).  kRing = 2
// is 56 KiB: at most two workgroups share a CU, i.e. four waves on four SIMDs,
// so a consumer never shares its SIMD with another wave.
template <int kRing>
constexpr int pc_lds_bytes() { return (kRing * kPcSlotU4 + kPcRawSlots * kPcRawU4) * 16; }

#ifdef LBF_PC_STAMPS
// Diagnostic build only (tools/probe_pc.hip): per-workgroup cycle split of the
// two roles.  [wg][wave][0..3] = {wait-a, work, wait-b, steps}.
__device__ unsigned long long g_pc_stamps[8192 * 8];
#define PC_STAMP(var)                                                                 \
  do {                                                                                \
    __builtin_amdgcn_sched_barrier(0);                                                \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(var)::"memory");     \
    __builtin_amdgcn_sched_barrier(0);                                                \
  } while (0)
#define PC_ACC(slot, a, b) acc[slot] += (b) - (a)
#define PC_COPY(dst, src) dst = src
#else
#define PC_COPY(dst, src) \
  do {                    \
  } while (0)
#define PC_STAMP(var) \
  do {                \
  } while (0)
#define PC_ACC(slot, a, b) \
  do {                     \
  } while (0)
#endif

// Valid 64-byte source for lanes with nothing to prefetch (inactive lanes,
// steps past a chain's full blocks, misaligned chains): the raw-block DMA is
// issued by every lane every step so that the vmcnt bookkeeping is static.
__device__ uint4 g_pc_dummy[4];

struct ChainInfo {
  const uint8_t* src;
  uint32_t size;
  uint32_t nfull;   // full 64-byte blocks
  uint32_t total;   // full + final blocks (0 for an inactive lane)
  bool aligned;
};

template <bool kUniform>
__device__ __forceinline__ ChainInfo chain_info(const ChunkParams& p, uint32_t i) {
  ChainInfo c{};
  if (i >= p.n) {
    c.src = p.base;
    return c;
  }
  uint64_t off;
  if (kUniform) {
    off = (p.first_chunk + i) * (uint64_t)p.chunk_size;
    const uint64_t rem = p.len - off;
    c.size = rem < p.chunk_size ? (uint32_t)rem : p.chunk_size;
  } else {
    off = p.offsets[i];
    c.size = p.sizes[i];
  }
  c.src = p.base + off;
  c.nfull = c.size >> 6;
  c.total = c.nfull + ((c.size & 63u) >= 56u ? 2u : 1u);
  c.aligned = (reinterpret_cast<uintptr_t>(c.src) & 15u) == 0;
  return c;
}

__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}

__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, off, 64));
  return v;
}

// 16 bytes per lane, global -> LDS (M0 + lane*16), without a VGPR round trip.
// Inline asm on purpose: with the __builtin_amdgcn_global_load_lds form hipcc
// drains vmcnt(0) before every later ds_read (it cannot tell the staging slots
// apart), which would collapse the prefetch; here the waits are counted by hand
// (pc_wait_raw) and the compiler sees no outstanding VMEM op of ours.
__device__ __forceinline__ void dma16(const void* g, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(g), "s"(lds_addr)
               : "memory");
}

// Raw bytes of block `step` of every chain into raw slot step % 4, laid out
// [16-byte piece j][lane] so both the DMA and the later ds_read_b128 are
// contiguous across lanes.  Always exactly 4 VMEM instructions.
__device__ __forceinline__ void pc_dma_step(const ChainInfo& c, uint32_t step, uint32_t raw_lds) {
  const bool ok = c.aligned && step < c.nfull;
  const uint8_t* src = ok ? c.src + 64ull * step : reinterpret_cast<const uint8_t*>(g_pc_dummy);
  const uint32_t slot = raw_lds + (step % kPcRawSlots) * (kPcRawU4 * 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma16(src + 16 * j, slot + j * (kPcLanes * 16));
}

template <int kRing>
__device__ __forceinline__ void pc_produce(uint4* ring, const ChainInfo& c, uint32_t step, int lane) {
  uint32_t w[16];
  if (step < c.nfull) {
    if (c.aligned) {
      const uint4* raw = ring + kRing * kPcSlotU4 + (step % kPcRawSlots) * kPcRawU4 + lane;
      block_from_vec(w, raw[0], raw[kPcLanes], raw[2 * kPcLanes], raw[3 * kPcLanes]);
    } else {
      load_words_any(w, c.src + 64ull * step, 64);
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap(w[k]);
    }
  } else {
    // step == nfull: block with the tail bytes; step == nfull + 1: zeros + length.
    // Steps past `total` produce don't-care words the consumer never reads.
    final_block(w, c.src + 64ull * c.nfull, c.size & 63u, c.size, step != c.nfull);
  }
  expand_store(w, ring + (step % kRing) * kPcSlotU4 + lane, kPcLanes);
}

// kRing = 2 (the shipped form): the producer writes step k+1 into slot
// (k+1) % 2 while the consumer computes step k from slot k % 2.  A 3-slot ring
// that let the consumer prefetch step k+1 across the barrier measured 6 % slower
// (extra VGPR traffic and LDS instructions inside the round chain).
// kPairs consumer/producer pairs per workgroup (waves 0..kPairs-1 consume,
// kPairs..2*kPairs-1 produce; pair q = wave % kPairs).  kPairs = 2 with 112 KiB
// of LDS pins ONE workgroup per CU, so each of its 4 waves has a SIMD to itself
// -- for 16 K-32 K chains, where two 2- or 3-wave workgroups per CU would put
// a consumer and a producer on one SIMD.
template <bool kUniform, int kRing, int kPairs = 1>
__global__ void __launch_bounds__(128 * kPairs) sha1_pc_kernel(ChunkParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds_all[];  // per pair: W[kRing][20][64] | raw[4][4][64]
  const int lane = threadIdx.x & 63;
  const int wave_id = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave_id % kPairs;
  const int wave = wave_id / kPairs;  // 0 = consumer, 1 = producer
  uint4* ring = lds_all + pair * (pc_lds_bytes<kRing>() / 16);
  const uint32_t i = blockIdx.x * (kPcLanes * kPairs) + pair * kPcLanes + lane;
  const ChainInfo c = chain_info<kUniform>(p, i);
  // Identical in every wave of the workgroup (every wave passes every
  // barrier); readfirstlane keeps the loop bounds scalar.
  uint32_t nsteps = __builtin_amdgcn_readfirstlane(wave_max(c.total));
  if (kPairs > 1) {
    __shared__ uint32_t wg_steps;
    if (threadIdx.x == 0) wg_steps = 0;
    __syncthreads();
    if (lane == 0) atomicMax(&wg_steps, nsteps);
    __syncthreads();
    nsteps = __builtin_amdgcn_readfirstlane(wg_steps);
  }
  const uint32_t nbarriers = nsteps;  // both waves pass exactly nsteps barriers
  constexpr uint32_t kAhead = kRing - 1;  // steps the producer runs ahead
#ifdef LBF_PC_STAMPS
  unsigned long long acc[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0, t2 = 0, t3 = 0;
#endif

  if (wave == 1) {
    // ---------------- producer ----------------
    const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(ring + kRing * kPcSlotU4);
#pragma unroll
    for (uint32_t s = 0; s < kPcRawSlots; ++s) pc_dma_step(c, s, raw_lds);
    // steps 0 .. kAhead-1 before the first barrier, then step k + kAhead in interval k
    for (uint32_t k = 0; k < nbarriers + kAhead - 1; ++k) {
      if (k < nsteps) {
        PC_STAMP(t0);
        // raw block k has landed once at most the 3 younger steps (12 DMAs) are pending
        asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
        PC_STAMP(t1);
        pc_produce<kRing>(ring, c, k, lane);
        pc_dma_step(c, k + kPcRawSlots, raw_lds);  // reuses slot k % 4 (read above)
        PC_STAMP(t2);
        PC_ACC(0, t0, t1);
        PC_ACC(1, t1, t2);
      }
      PC_STAMP(t2);
      if (k + 1 >= kAhead) __syncthreads();       // barrier (k + 1 - kAhead)
      PC_STAMP(t3);
      PC_ACC(2, t2, t3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  } else {
    // ---------------- consumer ----------------
    Digest s;
    s.init();
    const RoundK K;
    for (uint32_t k = 0; k < nsteps; ++k) {
      PC_STAMP(t0);
      __syncthreads();  // barrier k: slot k % 2 complete
      PC_STAMP(t1);
      if (k < c.total) compress_expanded(s, ring + (k % kRing) * kPcSlotU4 + lane, kPcLanes, K);
      PC_STAMP(t2);
      PC_ACC(0, t0, t1);
      PC_ACC(1, t1, t2);
    }
    if (i < p.n) {
      uint32_t be[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) be[k] = bswap(s.h[k]);
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
  }
#ifdef LBF_PC_STAMPS
  if (lane == 0) {
    unsigned long long* o = g_pc_stamps + (blockIdx.x * 2 * kPairs + wave_id) * 4;
    o[0] = acc[0];
    o[1] = acc[1];
    o[2] = acc[2];
    o[3] = nsteps;
  }
#endif
}

// ---------------------------------------------------------------------------
// Kernel "pc2" (variant 4): one consumer, TWO producers per 64 chains.
//
// The consumer's round is cheapest (five VALU ops issued back to back) when
// its schedule word already carries the round constant, leaving one v_add_u32
// and one v_add3_u32 for the sum.  Adding K costs the producer 80 more ops per
// block, more than one producer wave has to spare, so two producers alternate
// blocks: producer X builds steps X, X+2, X+4, ... and spends two barrier
// intervals on each (words 0..39 before the first, 40..79 before the second).
// W ring: 3 slots (step k in slot k % 3): a slot is rewritten only after the
// consumer has passed the barrier that ends its read.  Raw staging: 2 slots of
// 4 KiB per producer.  LDS 76 KiB -> two workgroups per CU.
// ---------------------------------------------------------------------------
constexpr int kP2Ring = 3;
constexpr int kP2Raw = 2;  // raw slots per producer
constexpr int kP2LdsBytes = (kP2Ring * kPcSlotU4 + 2 * kP2Raw * kPcRawU4) * 16;

// Raw bytes of `step` into raw slot `slot` of this producer: 4 DMA ops always.
__device__ __forceinline__ void p2_dma(const ChainInfo& c, uint32_t step, uint32_t raw_lds, uint32_t slot) {
  const bool ok = c.aligned && step < c.nfull;
  const uint8_t* src = ok ? c.src + 64ull * step : reinterpret_cast<const uint8_t*>(g_pc_dummy);
  const uint32_t base = raw_lds + slot * (kPcRawU4 * 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma16(src + 16 * j, base + j * (kPcLanes * 16));
}

// The 16 message words of `step`: full blocks from the raw slot (aligned) or
// global memory (misaligned), final blocks built from the tail.
__device__ __forceinline__ void p2_block(uint32_t (&w)[16], const uint4* raw, const ChainInfo& c, uint32_t step) {
  if (step < c.nfull) {
    if (c.aligned) {
      block_from_vec(w, raw[0], raw[kPcLanes], raw[2 * kPcLanes], raw[3 * kPcLanes]);
    } else {
      load_words_any(w, c.src + 64ull * step, 64);
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap(w[k]);
    }
  } else {
    final_block(w, c.src + 64ull * c.nfull, c.size & 63u, c.size, step != c.nfull);
  }
}

template <bool kUniform>
__global__ void __launch_bounds__(192) sha1_pc2_kernel(ChunkParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 ring[];  // W[3][20][64] | raw[2][2][4][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t i = blockIdx.x * kPcLanes + lane;
  const ChainInfo c = chain_info<kUniform>(p, i);
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane(wave_max(c.total));
#ifdef LBF_PC_STAMPS
  unsigned long long acc[4] = {0, 0, 0, 0}, t0 = 0, t1 = 0, t2 = 0, t3 = 0;
#endif

  if (wave != 0) {
    // ---------------- producer X = wave - 1: steps X, X+2, ... ----------------
    const uint32_t X = wave - 1;
    uint4* raw = ring + kP2Ring * kPcSlotU4 + X * (kP2Raw * kPcRawU4);
    const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(raw);
    p2_dma(c, X, raw_lds, 0);
    p2_dma(c, X + 2, raw_lds, 1);
    uint32_t w[16];
    // Interval b ends at barrier b.  Producer X finishes step b when b % 2 == X
    // and starts step b + 1 otherwise; producer 0 builds step 0 whole.
    for (uint32_t b = 0; b < nsteps; ++b) {
      const bool second = (b & 1u) == X;
      const uint32_t step = second ? b : b + 1;
      const bool first_too = (b == 0 && X == 0);
      PC_STAMP(t0);
      PC_COPY(t1, t0);
      if ((!second || first_too) && step < nsteps) {
        const uint32_t j = (step - X) >> 1;  // this producer's j-th step
        // block j has landed once only block j+1's 4 DMAs may be pending
        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
        PC_STAMP(t1);
        p2_block(w, raw + (j & 1u) * kPcRawU4 + lane, c, step);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // raw slot read before it is refilled
        p2_dma(c, step + 4, raw_lds, j & 1u);
        expand_store_wk<0>(w, ring + (step % kP2Ring) * kPcSlotU4 + lane, kPcLanes);
      }
      if (second && step < nsteps) expand_store_wk<1>(w, ring + (step % kP2Ring) * kPcSlotU4 + lane, kPcLanes);
      PC_STAMP(t2);
      __syncthreads();  // barrier b
      PC_STAMP(t3);
      PC_ACC(0, t0, t1);
      PC_ACC(1, t1, t2);
      PC_ACC(2, t2, t3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  } else {
    // ---------------- consumer ----------------
    Digest s;
    s.init();
    for (uint32_t k = 0; k < nsteps; ++k) {
      PC_STAMP(t0);
      __syncthreads();  // barrier k: slot k % 3 complete
      PC_STAMP(t1);
      if (k < c.total) compress_expanded_wk(s, ring + (k % kP2Ring) * kPcSlotU4 + lane, kPcLanes);
      PC_STAMP(t2);
      PC_ACC(0, t0, t1);
      PC_ACC(1, t1, t2);
    }
    if (i < p.n) {
      uint32_t be[5];
#pragma unroll
      for (int k = 0; k < 5; ++k) be[k] = bswap(s.h[k]);
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
  }
#ifdef LBF_PC_STAMPS
  if (lane == 0) {
    unsigned long long* o = g_pc_stamps + (blockIdx.x * 3 + wave) * 4;
    o[0] = acc[0];
    o[1] = acc[1];
    o[2] = acc[2];
    o[3] = nsteps;
  }
#endif
}

// ---------------------------------------------------------------------------
// Kernel "pc4" (variant 6): pc2 with the schedule double-buffered in the
// consumer's registers.
//
// pc2's consumer loads step k's 80 words after barrier k and its first round
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
__device__ __forceinline__ void write_result(const ChunkParams& p, uint32_t i, const Digest& s) {
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

constexpr int kPc4Ring = 4;
// Diagnostic builds only (tools/probe_pc.hip): LBF_PC4_NOLOADS feeds the
// rounds opaque registers instead of LDS words, LBF_PC4_NOBARRIER drops the
// barriers.  Both give wrong digests; they isolate what loads and barriers cost.
#ifdef LBF_PC4_NOLOADS
#define PC4_LOAD(dst, src) asm volatile("" : "=v"((dst).x), "=v"((dst).y), "=v"((dst).z), "=v"((dst).w))
#else
#define PC4_LOAD(dst, src) (dst) = (src)
#endif
#ifdef LBF_PC4_NOBARRIER
#define PC4_SYNC() do {} while (0)
#else
#define PC4_SYNC() __syncthreads()
#endif
constexpr int kPc4LdsBytes = (kPc4Ring * kPcSlotU4 + 2 * kP2Raw * kPcRawU4) * 16;
constexpr int kPc4Early = 15;  // loads issued before the first round
constexpr int kPc4LateAt = 3;  // the rest after quad 3's rounds

// Step from `cur` (in registers); meanwhile the next step's 20 quads are
// loaded from `next_slot` (this lane's column) into `nxt`.  Every lane runs
// the rounds (no divergent branch around the late loads); a lane whose chain
// has ended (`live` false) keeps its digest.
__device__ __forceinline__ void pc4_compress(Digest& s, const uint4 (&cur)[kPcQuads], uint4 (&nxt)[kPcQuads],
                                             const uint4* next_slot, bool live, bool all_live) {
#pragma unroll
  for (int q = 0; q < kPc4Early; ++q) PC4_LOAD(nxt[q], next_slot[q * kPcLanes]);
  // early loads go first (fenced on the digest, not on copies of it, so the
  // working state needs no register copies)
  asm volatile("" : "+v"(s.h[0]), "+v"(s.h[1]), "+v"(s.h[2]), "+v"(s.h[3]), "+v"(s.h[4])::"memory");
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
  for (int q = 0; q < kPcQuads; ++q) {
    round_step_wk(4 * q + 0, a, b, c, d, e, cur[q].x);
    round_step_wk(4 * q + 1, a, b, c, d, e, cur[q].y);
    round_step_wk(4 * q + 2, a, b, c, d, e, cur[q].z);
    round_step_wk(4 * q + 3, a, b, c, d, e, cur[q].w);
    if (q == kPc4LateAt) {
      // The two fences pin the late loads between quads 3 and 4: rounds are
      // ordered through the state, loads through the memory clobber (left
      // alone, the compiler sinks them to the end of the step, right before
      // the barrier, which then waits for them).
      asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
#pragma unroll
      for (int r = kPc4Early; r < kPcQuads; ++r) PC4_LOAD(nxt[r], next_slot[r * kPcLanes]);
      asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
    }
  }
  if (all_live) {  // wave-uniform: every chain of the workgroup has this step
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

// pc4_compress with the schedule read as 40 ds_read_b64 (variant 7).  A lone
// wave pays ≈96 cycles per block for 20 ds_read_b128 over the same rounds fed
// from registers, and ≈4 for 40 ds_read_b64 (tools/probe_lds_lanes.hip,
// profiles/r01/probe_lds_lanes.log).  The lgkm counter holds 15, so the next
// step's 40 pairs go out in three batches: before round 0, after round 16 and
// after round 40, each pinned by fences like the late loads of pc4_compress.
constexpr int kPc5Pairs = 40;
constexpr int kPc5B1 = 15, kPc5B1At = 7;   // pairs 0..14 first; 15..27 after pair 7's rounds
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

// The consumer's side of one pc4 step in either layout: uint4 quads (kVec 4,
// variant 6) or uint2 pairs (kVec 2, variant 7) of the same 20 KiB slot.
template <int kVec>
struct Pc4Sched;
template <>
struct Pc4Sched<4> {
  uint4 v[kPcQuads];
  static __device__ __forceinline__ const uint4* col(const uint4* ring, int slot, int lane) {
    return ring + slot * kPcSlotU4 + lane;
  }
  __device__ __forceinline__ void load_all(const uint4* src) {
#pragma unroll
    for (int q = 0; q < kPcQuads; ++q) v[q] = src[q * kPcLanes];
  }
};
template <int kVec>
struct Pc4Sched {  // kVec 2: uint2 pairs, loads may pair up; kVec 1: single ds_read_b64 each
  uint2 v[kPc5Pairs];
  static __device__ __forceinline__ const uint2* col(const uint4* ring, int slot, int lane) {
    return reinterpret_cast<const uint2*>(ring + slot * kPcSlotU4) + lane;
  }
  __device__ __forceinline__ void load_all(const uint2* src) {
#pragma unroll
    for (int q = 0; q < kPc5Pairs; ++q) v[q] = src[q * kPcLanes];
  }
};
__device__ __forceinline__ void pc4_step(Digest& s, const Pc4Sched<4>& cur, Pc4Sched<4>& nxt, const uint4* next_slot,
                                         bool live, bool all_live) {
  pc4_compress(s, cur.v, nxt.v, next_slot, live, all_live);
}
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

template <bool kUniform, int kVec>
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
    // Four steps per iteration while every chain of the workgroup is running
    // and every step is followed by a barrier: k % 4 == 0, so the slots are
    // compile-time offsets and the steps need no liveness checks.
    for (; k + 4 <= min_steps && k + 4 < nsteps; k += 4) {
      pc4_step(s, A, B, Pc4Sched<kVec>::col(ring, 1, lane), true, true);
      pc4_barrier(s PC4_ACC);  // barrier k+1
      pc4_step(s, B, A, Pc4Sched<kVec>::col(ring, 2, lane), true, true);
      pc4_barrier(s PC4_ACC);  // barrier k+2
      pc4_step(s, A, B, Pc4Sched<kVec>::col(ring, 3, lane), true, true);
      pc4_barrier(s PC4_ACC);  // barrier k+3
      pc4_step(s, B, A, Pc4Sched<kVec>::col(ring, 0, lane), true, true);
      pc4_barrier(s PC4_ACC);  // barrier k+4
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
constexpr int kPx4PairU4 = kPx4Ring * kPcSlotU4 + kPcRawSlots * kPcRawU4;  // 56 KiB per pair
constexpr int kPx4LdsBytes = 2 * kPx4PairU4 * 16;                           // 112 KiB

template <int kKFrom>
__device__ __forceinline__ void px4_round(int i, uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d, uint32_t& e,
                                          uint32_t x, const RoundK& K) {
  if (i < kKFrom) round_step_kv(i, a, b, c, d, e, x, K);
  else round_step_wk(i, a, b, c, d, e, x);
}

template <int kKFrom>
__device__ __forceinline__ void px4_compress(Digest& s, const uint2 (&cur)[kPc5Pairs], uint2 (&nxt)[kPc5Pairs],
                                             const uint2* next_slot, const RoundK& K, bool live, bool all_live) {
#pragma unroll
  for (int q = 0; q < kPc5B1; ++q) nxt[q] = next_slot[q * kPcLanes];
  asm volatile("" : "+v"(s.h[0]), "+v"(s.h[1]), "+v"(s.h[2]), "+v"(s.h[3]), "+v"(s.h[4])::"memory");
  uint32_t a = s.h[0], b = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
  for (int q = 0; q < kPc5Pairs; ++q) {
    px4_round<kKFrom>(2 * q + 0, a, b, c, d, e, cur[q].x, K);
    px4_round<kKFrom>(2 * q + 1, a, b, c, d, e, cur[q].y, K);
    if (q == kPc5B1At || q == kPc5B2At) {
      asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d), "+v"(e)::"memory");
      const int lo = q == kPc5B1At ? kPc5B1 : kPc5B2;
      const int hi = q == kPc5B1At ? kPc5B2 : kPc5Pairs;
#pragma unroll
      for (int r = lo; r < hi; ++r) nxt[r] = next_slot[r * kPcLanes];
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

// One whole step of this producer's 64 chains into ring slot step % 2; the
// raw slot it read is refilled with block step + 4.
template <int kKFrom>
__device__ __forceinline__ void px4_produce(uint4* ring, uint32_t raw_lds, const ChainInfo& c, uint32_t step,
                                            int lane) {
  uint32_t w[16];
  asm volatile("s_waitcnt vmcnt(12)" ::: "memory");  // block `step` landed; steps +1..+3 pending
  const uint4* raw = ring + kPx4Ring * kPcSlotU4 + (step % kPcRawSlots) * kPcRawU4 + lane;
  if (step < c.nfull) {
    if (c.aligned) {
      block_from_vec(w, raw[0], raw[kPcLanes], raw[2 * kPcLanes], raw[3 * kPcLanes]);
    } else {
      load_words_any(w, c.src + 64ull * step, 64);
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap(w[k]);
    }
  } else {
    final_block(w, c.src + 64ull * c.nfull, c.size & 63u, c.size, step != c.nfull);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // raw slot read before it is refilled
  pc_dma_step(c, step + kPcRawSlots, raw_lds);
  expand_store_split<kKFrom>(w, reinterpret_cast<uint2*>(ring + (step % kPx4Ring) * kPcSlotU4) + lane, kPcLanes);
}

template <bool kUniform, int kKFrom>
__global__ void __launch_bounds__(256) sha1_pcx4_kernel(ChunkParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds_all[];  // per pair: W[2][20][64] | raw[4][4][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int pair = wave & 1;
  uint4* ring = lds_all + pair * kPx4PairU4;
  const uint32_t i = blockIdx.x * (2 * kPcLanes) + pair * kPcLanes + lane;
  const ChainInfo c = chain_info<kUniform>(p, i);
  // every wave passes every barrier: the step count is the workgroup's maximum
  __shared__ uint32_t wg_steps;
  if (threadIdx.x == 0) wg_steps = 0;
  __syncthreads();
  const uint32_t mine = __builtin_amdgcn_readfirstlane(wave_max(c.total));
  if (lane == 0) atomicMax(&wg_steps, mine);
  __syncthreads();
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane(wg_steps);
  if (nsteps == 0) return;  // uniform over the workgroup: no barrier is left waiting

  if (wave >= 2) {
    // ---------------- producer ----------------
    const uint32_t raw_lds = (uint32_t)reinterpret_cast<uintptr_t>(ring + kPx4Ring * kPcSlotU4);
#pragma unroll
    for (uint32_t r = 0; r < (uint32_t)kPcRawSlots; ++r) pc_dma_step(c, r, raw_lds);
    px4_produce<kKFrom>(ring, raw_lds, c, 0, lane);
    if (nsteps > 1) px4_produce<kKFrom>(ring, raw_lds, c, 1, lane);
    __syncthreads();  // barrier P: steps 0 and 1 complete
    __syncthreads();  // barrier 0: the consumers hold step 0, slot 0 is free
    for (uint32_t k = 0; k + 1 < nsteps; ++k) {
      // interval k+1: step k+2 into slot k % 2
      if (k + 2 < nsteps) px4_produce<kKFrom>(ring, raw_lds, c, k + 2, lane);
      __syncthreads();  // barrier k+1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  } else {
    // ---------------- consumer ----------------
    Digest s;
    s.init();
    const RoundK K;
    Pc4Sched<2> A, B;
#ifdef LBF_PC_STAMPS
    unsigned long long acc[4] = {0, 0, 0, 0};
#define PX4_ACC , acc
#else
#define PX4_ACC
#endif
    const uint32_t min_steps = __builtin_amdgcn_readfirstlane(wave_min(i < p.n ? c.total : 0xFFFFFFFFu));
    __syncthreads();  // barrier P
    A.load_all(Pc4Sched<2>::col(ring, 0, lane));
    __syncthreads();  // barrier 0 (its fence completes the loads)
    uint32_t k = 0;
    // two steps per iteration while every chain of the pair runs and each step
    // is followed by a barrier: k % 2 == 0, so the slot offsets are immediates
    for (; k + 2 <= min_steps && k + 2 < nsteps; k += 2) {
      px4_compress<kKFrom>(s, A.v, B.v, Pc4Sched<2>::col(ring, 1, lane), K, true, true);
      pc4_barrier(s PX4_ACC);  // barrier k+1
      px4_compress<kKFrom>(s, B.v, A.v, Pc4Sched<2>::col(ring, 0, lane), K, true, true);
      pc4_barrier(s PX4_ACC);  // barrier k+2
    }
    for (; k < nsteps; k += 2) {
      px4_compress<kKFrom>(s, A.v, B.v, Pc4Sched<2>::col(ring, (k + 1) % kPx4Ring, lane), K, k < c.total,
                           k < min_steps);
      if (k + 1 >= nsteps) break;
      pc4_barrier(s PX4_ACC);  // barrier k+1
      px4_compress<kKFrom>(s, B.v, A.v, Pc4Sched<2>::col(ring, k % kPx4Ring, lane), K, k + 1 < c.total,
                           k + 1 < min_steps);
      if (k + 2 >= nsteps) break;
      pc4_barrier(s PX4_ACC);  // barrier k+2
    }
    if (i < p.n) write_result(p, i, s);
#undef PX4_ACC
  }
}

// K split: the consumer adds K in rounds 0..39.  Splitting at 20 or 0 ran 5 %
// slower at every chain count (profiles/r01/sweep_v5_pcx4_ksplit.log).
constexpr int kPx4KFrom = 40;

template <int kKFrom>
void launch_pcx4(const ChunkParams& p, hipStream_t stream) {
  static std::once_flag once;
  std::call_once(once, [] {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pcx4_kernel<false, kKFrom>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kPx4LdsBytes);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pcx4_kernel<true, kKFrom>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kPx4LdsBytes);
  });
  const uint32_t blocks = (p.n + 2 * kPcLanes - 1) / (2 * kPcLanes);
  if (p.offsets) hipLaunchKernelGGL((sha1_pcx4_kernel<false, kKFrom>), dim3(blocks), dim3(256), kPx4LdsBytes, stream, p);
  else hipLaunchKernelGGL((sha1_pcx4_kernel<true, kKFrom>), dim3(blocks), dim3(256), kPx4LdsBytes, stream, p);
}

// ---------------------------------------------------------------------------
// Kernel "pcx5" (variant 10): pcx4 with the producer's first 16 words left in
// the raw block.
//
// pcx4 is producer-bound (≈2,170 cycles per step); ≈690 of a producer's
// cycles are its 20 KiB of stores.  Words 0..15 of a step are the chunk's own
// 64 bytes, already in LDS from the DMA, so the consumer reads them there
// (4 ds_read_b128 of the raw slot) and swaps their bytes itself (16 v_perm);
// the producer stores only words 16..79 (16 KiB).  The consumer's load count
// stays at 20 instructions per step.  For final and misaligned blocks the
// producer writes the little-endian words it built into the raw slot, so the
// consumer's read is the same for every step.
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
  uint4 raw[4];  // words 0..15, little-endian
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
    px4_round<kKFrom>(4 * j + 0, a, b, c, d, e, bswap(cur.raw[j].x), K);
    px4_round<kKFrom>(4 * j + 1, a, b, c, d, e, bswap(cur.raw[j].y), K);
    px4_round<kKFrom>(4 * j + 2, a, b, c, d, e, bswap(cur.raw[j].z), K);
    px4_round<kKFrom>(4 * j + 3, a, b, c, d, e, bswap(cur.raw[j].w), K);
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
  } else {
    if (step < c.nfull) {
      load_words_any(w, c.src + 64ull * step, 64);
#pragma unroll
      for (int k = 0; k < 16; ++k) w[k] = bswap(w[k]);
    } else {
      final_block(w, c.src + 64ull * c.nfull, c.size & 63u, c.size, step != c.nfull);
    }
    // the consumer reads words 0..15 of every step from the raw slot
#pragma unroll
    for (int j = 0; j < 4; ++j)
      raw[j * kPcLanes] = make_uint4(bswap(w[4 * j]), bswap(w[4 * j + 1]), bswap(w[4 * j + 2]), bswap(w[4 * j + 3]));
  }
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
      if (k + 2 < nsteps) px5_produce<kKFrom>(ring, raw_lds, c, k + 2, lane);
      __syncthreads();  // barrier k+1
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the workgroup
  } else {
    // ---------------- consumer ----------------
    Digest s;
    s.init();
    const RoundK K;
    Px5Sched A, B;
#ifdef LBF_PC_STAMPS
    unsigned long long acc[4] = {0, 0, 0, 0};
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
}

// K split for pcx5: the consumer adds K in rounds 0..63.  With the producer's
// stores down to 16 KiB the two sides balance near there: splitting at 40 ran
// 2 % slower, 48 and 56 within 0.5 % (profiles/r01/sweep_v9_pcx5_k40_k48.log,
// sweep_pcx5_k48_k56_k64.log); 72 ran 1.5 % and 80 (no K in the producer)
// 5 % slower (sweep_pcx5_k64_k72_k80.log).
constexpr int kPx5KFrom = 64;

template <int kKFrom>
void launch_pcx5(const ChunkParams& p, hipStream_t stream) {
  static std::once_flag once;
  std::call_once(once, [] {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pcx5_kernel<false, kKFrom>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kPx5LdsBytes);
    hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pcx5_kernel<true, kKFrom>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kPx5LdsBytes);
  });
  const uint32_t blocks = (p.n + 2 * kPcLanes - 1) / (2 * kPcLanes);
  if (p.offsets) hipLaunchKernelGGL((sha1_pcx5_kernel<false, kKFrom>), dim3(blocks), dim3(256), kPx5LdsBytes, stream, p);
  else hipLaunchKernelGGL((sha1_pcx5_kernel<true, kKFrom>), dim3(blocks), dim3(256), kPx5LdsBytes, stream, p);
}

// ---------------------------------------------------------------------------
// Kernel "lds" (variant 3): one chunk per lane for MANY chains.
//
// With >= 4 waves per SIMD the VALU itself is the limit (≈2,040 SIMD cycles per
// 64-byte block) and what is left to win is memory stall: in the
// lane kernel the compiler sinks every 16-byte load next to its use, so each
// block waits a full HBM round trip.  Here each wave streams its 64 chains'
// next kStages blocks global -> LDS with DMA (no VGPRs in flight, so the
// compiler cannot move them) and waits by count.  LDS per wave: kStages x 4 KiB.
// ---------------------------------------------------------------------------
template <int kStages>
__device__ __forceinline__ void lds_dma_step(const ChainInfo& c, uint32_t step, uint32_t wave_lds) {
  const bool ok = c.aligned && step < c.nfull;
  const uint8_t* src = ok ? c.src + 64ull * step : reinterpret_cast<const uint8_t*>(g_pc_dummy);
  const uint32_t slot = wave_lds + (step % kStages) * (kPcRawU4 * 16);
#pragma unroll
  for (int j = 0; j < 4; ++j) dma16(src + 16 * j, slot + j * (kPcLanes * 16));
}

template <bool kUniform, int kStages>
__global__ void __launch_bounds__(256) sha1_lds_kernel(ChunkParams p) {
  extern __shared__ __attribute__((aligned(16))) uint4 stage[];  // [wave][kStages][4][64]
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const ChainInfo c = chain_info<kUniform>(p, i);
  uint4* mine = stage + wave * (kStages * kPcRawU4);
  const uint32_t wave_lds = (uint32_t)reinterpret_cast<uintptr_t>(mine);
  const uint32_t nsteps = __builtin_amdgcn_readfirstlane(wave_max(c.nfull));
  const bool any_unaligned = __builtin_amdgcn_readfirstlane(
      (uint32_t)(__ballot(c.total != 0 && !c.aligned) != 0));
  Digest s;
  s.init();
#pragma unroll
  for (uint32_t k = 0; k < (uint32_t)kStages; ++k) lds_dma_step<kStages>(c, k, wave_lds);
  for (uint32_t k = 0; k < nsteps; ++k) {
    // block k has landed once at most the (kStages-1) younger steps are pending
    asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * (kStages - 1)) : "memory");
    const uint4* raw = mine + (k % kStages) * kPcRawU4 + lane;
    uint32_t w[16];
    block_from_vec(w, raw[0], raw[kPcLanes], raw[2 * kPcLanes], raw[3 * kPcLanes]);
    if (any_unaligned && !c.aligned && k < c.nfull) {
      load_words_any(w, c.src + 64ull * k, 64);
#pragma unroll
      for (int q = 0; q < 16; ++q) w[q] = bswap(w[q]);
    }
    // the slot is refilled below: its ds_reads must have returned first
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    lds_dma_step<kStages>(c, k + kStages, wave_lds);
    if (k < c.nfull) compress(s, w);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no DMA outlives the wave
  if (i >= p.n) return;
  finish(s, c.src + 64ull * c.nfull, c.size & 63u, c.size);
  uint32_t be[5];
#pragma unroll
  for (int k = 0; k < 5; ++k) be[k] = bswap(s.h[k]);
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
constexpr int kLdsStages = 2;

// ---------------------------------------------------------------------------
// Kernel "lds2" (variant 11): `lds` fetching each chain's bytes a whole 128-B
// line at a time.
//
// `lds` DMAs one 64-byte block per lane per step, so the two halves of a 128-B
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

// Counter-mode splitmix64 fill, 16 bytes per thread per step.
__global__ void __launch_bounds__(256) fill_synth_kernel(uint8_t* dst, uint64_t len, uint64_t seed,
                                                         uint64_t start_word) {
  const uint64_t nwords = len >> 3;
  const uint64_t npairs = (nwords + 1) >> 1;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < npairs; t += stride) {
    const uint64_t k = 2 * t;
    const uint64_t w0 = synth_word(seed, start_word + k);
    if (k + 1 < nwords) {
      const uint64_t w1 = synth_word(seed, start_word + k + 1);
      uint4 v;
      v.x = (uint32_t)w0; v.y = (uint32_t)(w0 >> 32);
      v.z = (uint32_t)w1; v.w = (uint32_t)(w1 >> 32);
      *reinterpret_cast<uint4*>(dst + 8 * k) = v;
    } else {
      *reinterpret_cast<uint64_t*>(dst + 8 * k) = w0;
    }
  }
  if (blockIdx.x == 0 && threadIdx.x == 0 && (len & 7)) {
    const uint64_t w = synth_word(seed, start_word + nwords);
    for (uint32_t j = 0; j < (len & 7); ++j) dst[8 * nwords + j] = (uint8_t)(w >> (8 * j));
  }
}

std::atomic<int> g_variant{0};
// Chain counts up to which pc4 / pcx2 are chosen automatically (tuned on
// MI355X, see DESIGN.md "kernel selection"): 64 chains per CU, 128 per CU.
constexpr uint32_t kPc4MaxChains = 16384;
constexpr uint32_t kPcMaxChains = 32768;

}  // namespace

int pick_variant(uint64_t n) {
  int variant = g_variant.load();
  if (variant == 0) {
    // Few chains: the per-chain instruction count bounds the time.  Up to one
    // 64-chain workgroup per CU, the schedule (round constants folded in) comes
    // from two producer waves and is double-buffered in the consumer's
    // registers, read as 8-byte pairs in three batches per step (7; 1-2 %
    // ahead of the uint4 form 6, profiles/r01/sweep_v678.log).  Up to two per
    // CU, two such pairs with one producer each share a workgroup pinned to its
    // CU, so every wave owns a SIMD, split the round constants between
    // consumer and producer, and the consumer takes words 0..15 from the raw
    // block so the producer stores 16 KiB per step instead of 20 (10; 8 % ahead
    // of pcx4 (9), which was 0-4 % ahead of the plain pairs of pcx2 (5);
    // profiles/r01/sweep_v5_pcx4_ksplit.log, sweep_v9_pcx5_k40_k48.log,
    // sweep_pcx5_k48_k56_k64.log).  Many chains: every SIMD is busy
    // and the fused one-chunk-per-lane kernel issues the fewest instructions in
    // total, LDS-staged and fetching whole 128-byte lines (11; 2 % ahead of the
    // per-block DMA of 3 at C3, traffic 1.14 -> 1.001 x, sweep_v3_v11_lds2.log).
    // Crossovers from tools/sweep_variants.py (profiles/r01/sweep_v123.log,
    // sweep_v245.log, sweep_v46_pc4.log).
    variant = n <= kPc4MaxChains ? 7 : (n <= kPcMaxChains ? 10 : 11);
  }
  return variant;
}

int launch_chunks(const ChunkParams& p, hipStream_t stream) {
  if (p.n == 0) return LBF_OK;
  const int variant = pick_variant(p.n);
  if (variant == 2) {
    const uint32_t blocks = (p.n + kPcLanes - 1) / kPcLanes;
    constexpr int lds = pc_lds_bytes<2>();
    if (p.offsets) hipLaunchKernelGGL((sha1_pc_kernel<false, 2>), dim3(blocks), dim3(128), lds, stream, p);
    else hipLaunchKernelGGL((sha1_pc_kernel<true, 2>), dim3(blocks), dim3(128), lds, stream, p);
  } else if (variant == 5) {
    constexpr int lds = 2 * pc_lds_bytes<2>();
    static std::once_flag once;
    std::call_once(once, [] {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pc_kernel<false, 2, 2>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pc_kernel<true, 2, 2>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    });
    const uint32_t blocks = (p.n + 2 * kPcLanes - 1) / (2 * kPcLanes);
    if (p.offsets) hipLaunchKernelGGL((sha1_pc_kernel<false, 2, 2>), dim3(blocks), dim3(256), lds, stream, p);
    else hipLaunchKernelGGL((sha1_pc_kernel<true, 2, 2>), dim3(blocks), dim3(256), lds, stream, p);
  } else if (variant == 4) {
    static std::once_flag once;
    std::call_once(once, [] {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pc2_kernel<false>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kP2LdsBytes);
      hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pc2_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kP2LdsBytes);
    });
    const uint32_t blocks = (p.n + kPcLanes - 1) / kPcLanes;
    if (p.offsets) hipLaunchKernelGGL(sha1_pc2_kernel<false>, dim3(blocks), dim3(192), kP2LdsBytes, stream, p);
    else hipLaunchKernelGGL(sha1_pc2_kernel<true>, dim3(blocks), dim3(192), kP2LdsBytes, stream, p);
  } else if (variant == 6 || variant == 7 || variant == 8) {
    static std::once_flag once;
    std::call_once(once, [] {
      for (const void* f : {reinterpret_cast<const void*>(&sha1_pc4_kernel<false, 4>),
                            reinterpret_cast<const void*>(&sha1_pc4_kernel<true, 4>),
                            reinterpret_cast<const void*>(&sha1_pc4_kernel<false, 2>),
                            reinterpret_cast<const void*>(&sha1_pc4_kernel<true, 2>),
                            reinterpret_cast<const void*>(&sha1_pc4_kernel<false, 1>),
                            reinterpret_cast<const void*>(&sha1_pc4_kernel<true, 1>)})
        hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, kPc4LdsBytes);
    });
    const uint32_t blocks = (p.n + kPcLanes - 1) / kPcLanes;
    const dim3 g(blocks), b(192);
    if (variant == 6) {
      if (p.offsets) hipLaunchKernelGGL((sha1_pc4_kernel<false, 4>), g, b, kPc4LdsBytes, stream, p);
      else hipLaunchKernelGGL((sha1_pc4_kernel<true, 4>), g, b, kPc4LdsBytes, stream, p);
    } else if (variant == 7) {
      if (p.offsets) hipLaunchKernelGGL((sha1_pc4_kernel<false, 2>), g, b, kPc4LdsBytes, stream, p);
      else hipLaunchKernelGGL((sha1_pc4_kernel<true, 2>), g, b, kPc4LdsBytes, stream, p);
    } else {
      if (p.offsets) hipLaunchKernelGGL((sha1_pc4_kernel<false, 1>), g, b, kPc4LdsBytes, stream, p);
      else hipLaunchKernelGGL((sha1_pc4_kernel<true, 1>), g, b, kPc4LdsBytes, stream, p);
    }
  } else if (variant == 9) {
    launch_pcx4<kPx4KFrom>(p, stream);
  } else if (variant == 10) {
    launch_pcx5<kPx5KFrom>(p, stream);
  } else if (variant == 11) {
    static std::once_flag once;
    std::call_once(once, [] {
      hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_lds2_kernel<false>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kLds2Bytes);
      hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_lds2_kernel<true>),
                          hipFuncAttributeMaxDynamicSharedMemorySize, kLds2Bytes);
    });
    const uint32_t blocks = (p.n + 255) / 256;
    if (p.offsets) hipLaunchKernelGGL(sha1_lds2_kernel<false>, dim3(blocks), dim3(256), kLds2Bytes, stream, p);
    else hipLaunchKernelGGL(sha1_lds2_kernel<true>, dim3(blocks), dim3(256), kLds2Bytes, stream, p);
  } else if (variant == 3) {
    const uint32_t blocks = (p.n + 255) / 256;
    constexpr int lds = 4 * kLdsStages * kPcRawU4 * 16;
    if (p.offsets) hipLaunchKernelGGL((sha1_lds_kernel<false, kLdsStages>), dim3(blocks), dim3(256), lds, stream, p);
    else hipLaunchKernelGGL((sha1_lds_kernel<true, kLdsStages>), dim3(blocks), dim3(256), lds, stream, p);
  } else {
    // 64-thread workgroups while waves are scarce so they spread over every CU.
    const uint32_t threads = p.n <= 65536u ? 64u : 256u;
    const uint32_t blocks = (p.n + threads - 1) / threads;
    if (p.offsets) {
      hipLaunchKernelGGL(sha1_lane_kernel<false>, dim3(blocks), dim3(threads), 0, stream, p);
    } else {
      hipLaunchKernelGGL(sha1_lane_kernel<true>, dim3(blocks), dim3(threads), 0, stream, p);
    }
  }
  LBF_HIP_TRY(hipGetLastError());
  return LBF_OK;
}

}  // namespace lbf

using lbf::fail;

static int check_out_alignment(const uint8_t* d_digests, const uint8_t* d_expected) {
  if ((reinterpret_cast<uintptr_t>(d_digests) & 3u) || (reinterpret_cast<uintptr_t>(d_expected) & 3u))
    return fail(LBF_ERR_INVALID, "digest/expected arrays must be 4-byte aligned");
  return LBF_OK;
}

extern "C" int lbf_sha1_launch(const uint8_t* d_base, const uint64_t* d_offsets, const uint32_t* d_sizes,
                               uint64_t n, uint8_t* d_digests, const uint8_t* d_expected,
                               uint8_t* d_verdicts, void* stream) {
  if (n == 0) return LBF_OK;
  if (!d_base || !d_offsets || !d_sizes) return fail(LBF_ERR_INVALID, "lbf_sha1_launch: null input");
  if (n > 0xFFFFFFFFull) return fail(LBF_ERR_INVALID, "lbf_sha1_launch: n exceeds 2^32-1 per launch");
  if (!d_digests && !d_verdicts) return fail(LBF_ERR_INVALID, "lbf_sha1_launch: no output");
  if ((d_verdicts != nullptr) != (d_expected != nullptr))
    return fail(LBF_ERR_INVALID, "lbf_sha1_launch: expected and verdicts go together");
  if (int rc = check_out_alignment(d_digests, d_expected)) return rc;
  lbf::ChunkParams p{};
  p.base = d_base;
  p.offsets = d_offsets;
  p.sizes = d_sizes;
  p.n = (uint32_t)n;
  p.digests = d_digests;
  p.expected = d_expected;
  p.verdicts = d_verdicts;
  return lbf::launch_chunks(p, (hipStream_t)stream);
}

extern "C" int lbf_sha1_uniform_launch(const uint8_t* d_base, uint64_t len, uint32_t chunk_size,
                                       uint64_t first_chunk, uint64_t n, uint8_t* d_digests,
                                       const uint8_t* d_expected, uint8_t* d_verdicts, void* stream) {
  if (n == 0) return LBF_OK;
  if (!d_base || chunk_size == 0) return fail(LBF_ERR_INVALID, "lbf_sha1_uniform_launch: bad region");
  const uint64_t total_chunks = (len + chunk_size - 1) / chunk_size;
  if (first_chunk > total_chunks || n > total_chunks - first_chunk)
    return fail(LBF_ERR_INVALID, "lbf_sha1_uniform_launch: chunk range outside region");
  if (n > 0xFFFFFFFFull) return fail(LBF_ERR_INVALID, "lbf_sha1_uniform_launch: n too large");
  if (!d_digests && !d_verdicts) return fail(LBF_ERR_INVALID, "lbf_sha1_uniform_launch: no output");
  if ((d_verdicts != nullptr) != (d_expected != nullptr))
    return fail(LBF_ERR_INVALID, "lbf_sha1_uniform_launch: expected and verdicts go together");
  if (int rc = check_out_alignment(d_digests, d_expected)) return rc;
  lbf::ChunkParams p{};
  p.base = d_base;
  p.len = len;
  p.first_chunk = first_chunk;
  p.chunk_size = chunk_size;
  p.n = (uint32_t)n;
  p.digests = d_digests;
  p.expected = d_expected;
  p.verdicts = d_verdicts;
  return lbf::launch_chunks(p, (hipStream_t)stream);
}

extern "C" int lbf_set_kernel_variant(int variant) {
  if (variant < 0 || variant > 11) return fail(LBF_ERR_INVALID, "unknown kernel variant");
  lbf::g_variant.store(variant);
  return LBF_OK;
}

extern "C" int lbf_get_kernel_variant(void) { return lbf::g_variant.load(); }

extern "C" int lbf_kernel_for(uint64_t n_chunks) { return lbf::pick_variant(n_chunks); }

extern "C" int lbf_fill_synthetic(uint8_t* d_buf, uint64_t len, uint64_t seed, uint64_t start, void* stream) {
  if (len == 0) return LBF_OK;
  if (!d_buf || (start & 7u) || (reinterpret_cast<uintptr_t>(d_buf) & 15u))
    return fail(LBF_ERR_INVALID, "lbf_fill_synthetic: need start%8==0 and a 16-byte aligned buffer");
  const uint64_t pairs = ((len >> 3) + 1) >> 1;
  uint64_t blocks = (pairs + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks == 0) blocks = 1;
  hipLaunchKernelGGL(lbf::fill_synth_kernel, dim3((uint32_t)blocks), dim3(256), 0, (hipStream_t)stream,
                     d_buf, len, seed, start >> 3);
  LBF_HIP_TRY(hipGetLastError());
  return LBF_OK;
}

extern "C" int lbf_time_uniform(const uint8_t* d_base, uint64_t len, uint32_t chunk_size, uint64_t first_chunk,
                                uint64_t n, uint8_t* d_digests, int reps, void* stream,
                                float* out_ms_per_launch) {
  if (reps <= 0 || !out_ms_per_launch) return fail(LBF_ERR_INVALID, "lbf_time_uniform: bad reps/out");
  hipStream_t s = (hipStream_t)stream;
  struct Events {  // destroyed on every return path
    hipEvent_t e0 = nullptr, e1 = nullptr;
    ~Events() {
      if (e0) (void)hipEventDestroy(e0);
      if (e1) (void)hipEventDestroy(e1);
    }
  } ev;
  LBF_HIP_TRY(hipEventCreate(&ev.e0));
  LBF_HIP_TRY(hipEventCreate(&ev.e1));
  int rc = LBF_OK;
  LBF_HIP_TRY(hipEventRecord(ev.e0, s));
  for (int r = 0; r < reps && rc == LBF_OK; ++r)
    rc = lbf_sha1_uniform_launch(d_base, len, chunk_size, first_chunk, n, d_digests, nullptr, nullptr, stream);
  LBF_HIP_TRY(hipEventRecord(ev.e1, s));
  LBF_HIP_TRY(hipEventSynchronize(ev.e1));
  float ms = 0.f;
  LBF_HIP_TRY(hipEventElapsedTime(&ms, ev.e0, ev.e1));
  if (rc != LBF_OK) return rc;
  *out_ms_per_launch = ms / (float)reps;
  return LBF_OK;
}
