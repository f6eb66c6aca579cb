// kern_common.hpp -- shared pieces of the chunk-hash kernels: LDS slot
// geometry, s_memtime stamps (diagnostic builds), chain descriptors, the LDS-DMA
// primitive and the digest/verdict write-back.
//
// Part of the single translation unit sha1_kernels.hip (included from there);
// DESIGN.md §4 has the measurements behind each kernel.
#pragma once

#include <hip/hip_runtime.h>

#include "lbf_internal.hpp"
#include "sha1_device.hpp"

namespace lbf {
namespace {

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
    // A lane past the end of the table runs a copy of its wave's first chain
    // (no result is ever written for it).  The producer waves then take one
    // branch per step for the whole wave, instead of building a padding block
    // for the idle lanes next to the live lanes' full blocks: a wave with
    // idle lanes -- one chunk through Base64Encode, the last wave of a batch
    // -- ran at ≈2,380 rather than ≈1,810 cycles per block.
    const uint32_t first = i & ~63u;
    if (first >= p.n) {
      c.src = p.base;
      return c;
    }
    i = first;
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
// M0 is declared clobbered.  M0 is a reserved register, so clang warns that
// the clobber "may not be preserved", but the clobber is what stops the
// compiler from reusing an M0 value it set before the asm: without it, two
// __builtin_amdgcn_global_load_lds with the same LDS base around a dma16 share
// one `s_mov_b32 m0` and the second lands at the dma16's address
// (tests/c/m0_clobber_probe.hip, pinned by tests/test_isa.py).
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ void dma16(const void* g, uint32_t lds_addr) {
  asm volatile("s_mov_b32 m0, %1\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %0, off"
               :
               : "v"(g), "s"(lds_addr)
               : "memory", "m0");
}
#pragma clang diagnostic pop

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

}  // namespace
}  // namespace lbf
