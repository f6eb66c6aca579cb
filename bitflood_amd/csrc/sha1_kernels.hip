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

#include "kern_common.hpp"
#include "kern_lane.hpp"
#include "kern_pc.hpp"
#include "kern_pcx.hpp"

namespace lbf {

namespace {

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
