// sha1_kernels.hip -- MI355X (gfx950) chunk-hash kernels and their launchers.
//
// Replaces the per-chunk hash of Encoder::EncodeFile
// (/root/reference/cpp/src/Encoder.cpp:54-72 -> Base64Encode :107-120) and the
// verify hashes of Flood.cpp:259-275 / ChunkMethods.cpp:116-123,165-167 with
// one batched launch over many independent chunks.
//
// Also the receiver's base64 decode (kern_b64.hpp, lbf_b64_verify_batch).
//
// Shipped kernels (lbf_kernel_for picks one by chain count):
//   "lane" (variant 1): one chunk per lane, the simple baseline.  SHA-1 is a
//     serial Merkle-Damgard chain, so the only parallelism is across chunks;
//     each lane keeps its chain state and the 16-word schedule in VGPRs.
//   "pc4/b64" (variant 7): one consumer + two producer waves per 64 chains, the
//     W+K schedule handed over in LDS and double-buffered in the consumer's
//     registers as 8-byte pairs -- few chains (<= 16 K, C2).
//   "pc4x2" (variant 12): two pc4 groups per CU in one 6-wave workgroup, the
//     producers two to a SIMD -- the 16 K-32 K chain kernel since round 3.
//   "pcx5" (variant 10): two consumer/producer pairs per CU, K split between
//     them, words 0..15 read by the consumer from the raw block -- the 16-32 K
//     chain kernel (C4 per GPU) until round 3, kept for A/B.
//   "lds2" (variant 11): one chunk per lane with LDS-DMA staging of whole
//     128-byte lines -- many chains (C3).
// The superseded variants (2 pc, 3 lds, 4 pc2, 5 pcx2, 6 pc4/uint4, 8 pc4/b64
// single loads, 9 pcx4) and the diagnostic forms (13-33) are not in this
// library: tools/experimental/ builds them into an A/B library of its own,
// which registers them through g_extra_variants (lbf_internal.hpp).
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>

#include "lbf_internal.hpp"
#include "sha1_device.hpp"

#include "kern_common.hpp"
#include "kern_lane.hpp"
#include "kern_pc.hpp"
#include "kern_pcx.hpp"
#include "kern_b64.hpp"

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

bool shipped_variant(int v) { return v == 1 || v == 7 || v == 10 || v == 11 || v == 12; }
// Chain counts up to which pc4 / pcx2 are chosen automatically (tuned on
// MI355X, see DESIGN.md "kernel selection"): 64 chains per CU, 128 per CU.
constexpr uint32_t kPc4MaxChains = 16384;
constexpr uint32_t kPcMaxChains = 32768;

}  // namespace

const ExtraVariants* g_extra_variants = nullptr;

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
    // Since round 3, 16 K-32 K chains go to pc4x2 (12): two pc4 groups per CU,
    // their producers two to a SIMD.  Level with or ahead of pcx5 at every
    // count measured, and far ahead on ragged counts (20,000 chains: 3.45
    // against 4.83 ms at 256 KiB; profiles/r03/pc4x2/).
    variant = n <= kPc4MaxChains ? 7 : (n <= kPcMaxChains ? 12 : 11);
  }
  return variant;
}

template <bool kUniform>
void launch_pc4(const ChunkParams& p, hipStream_t stream) {
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pc4_kernel<kUniform, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kPc4LdsBytes);
  });
  hipLaunchKernelGGL((sha1_pc4_kernel<kUniform, 2>), dim3((p.n + kPcLanes - 1) / kPcLanes), dim3(192), kPc4LdsBytes,
                     stream, p);
}

template <bool kUniform>
void launch_pc4x2(const ChunkParams& p, hipStream_t stream) {
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_pc4x2_kernel<kUniform>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, kPc4x2LdsBytes);
  });
  hipLaunchKernelGGL(sha1_pc4x2_kernel<kUniform>, dim3((p.n + 2 * kPcLanes - 1) / (2 * kPcLanes)), dim3(384),
                     kPc4x2LdsBytes, stream, p);
}

template <bool kUniform>
void launch_lds2(const ChunkParams& p, hipStream_t stream) {
  static std::once_flag once;
  std::call_once(once, [] {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&sha1_lds2_kernel<kUniform>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, kLds2Bytes);
  });
  hipLaunchKernelGGL(sha1_lds2_kernel<kUniform>, dim3((p.n + 255) / 256), dim3(256), kLds2Bytes, stream, p);
}

template <bool kUniform>
void launch_lane(const ChunkParams& p, hipStream_t stream) {
  // 64-thread workgroups while waves are scarce so they spread over every CU.
  const uint32_t threads = p.n <= 65536u ? 64u : 256u;
  hipLaunchKernelGGL(sha1_lane_kernel<kUniform>, dim3((p.n + threads - 1) / threads), dim3(threads), 0, stream, p);
}


int launch_chunks(const ChunkParams& p, hipStream_t stream) {
  if (p.n == 0) return LBF_OK;
  const int variant = pick_variant(p.n);
  const bool uniform = p.offsets == nullptr;
  if (!shipped_variant(variant)) {
    // a variant only an A/B library registers (lbf_set_kernel_variant accepted it)
    if (!g_extra_variants || !g_extra_variants->launch(variant, p, stream))
      return fail(LBF_ERR_INVALID, "kernel variant " + std::to_string(variant) + " has no launcher");
    LBF_HIP_TRY(hipGetLastError());
    return LBF_OK;
  }
  if (variant == 7) {
    if (uniform) launch_pc4<true>(p, stream);
    else launch_pc4<false>(p, stream);
  } else if (variant == 10) {
    launch_pcx5<kPx5KFrom>(p, stream);
  } else if (variant == 12) {
    if (uniform) launch_pc4x2<true>(p, stream);
    else launch_pc4x2<false>(p, stream);
  } else if (variant == 11) {
    if (uniform) launch_lds2<true>(p, stream);
    else launch_lds2<false>(p, stream);
  } else {  // 1
    if (uniform) launch_lane<true>(p, stream);
    else launch_lane<false>(p, stream);
  }
  LBF_HIP_TRY(hipGetLastError());
  return LBF_OK;
}

// grid = (groups of kDecTilesPerGroup / kEncTilesPerGroup tiles, chunks), in launches of at most 65,535 chunks (grid.y)
template <class F>
static int b64_tiled_launch(uint32_t n, uint32_t tiles, F launch) {
  constexpr uint32_t kPer = 65535;
  for (uint32_t c0 = 0; c0 < n; c0 += kPer) {
    launch(dim3(tiles, std::min(kPer, n - c0)), c0);
    LBF_HIP_TRY(hipGetLastError());
  }
  return LBF_OK;
}

int launch_b64_decode(const B64Launch& b, hipStream_t stream) {
  if (b.n == 0) return LBF_OK;
  // the one-pass decode of canonically laid-out text, tile by tile (each
  // chunk's tiles cover its text and its output slot); then the general
  // two-pass decode of whatever it handed back (a workgroup per chunk, most
  // exit at once)
  const uint32_t tiles = std::max<uint32_t>(
      1u, std::max((b.max_text_len + kDecText - 1) / kDecText, (b.max_cap + kDecBytes - 1) / kDecBytes));
  if (int rc = b64_tiled_launch(b.n, (tiles + kDecTilesPerGroup - 1) / kDecTilesPerGroup, [&](dim3 grid, uint32_t c0) {
        hipLaunchKernelGGL(b64_decode_canon_kernel, grid, dim3(kB64Threads), 0, stream, b.text, b.text_off, b.text_len,
                           b.out, b.out_off, b.cap, b.sizes, b.over, b.redo, tiles, c0);
      }))
    return rc;
  hipLaunchKernelGGL(b64_decode_kernel, dim3(b.n), dim3(kB64Threads), 0, stream, b.text, b.scratch, b.text_off,
                     b.sext_off, b.text_len, b.out, b.out_off, b.cap, b.sizes, b.over, (const uint8_t*)b.redo);
  LBF_HIP_TRY(hipGetLastError());
  return LBF_OK;
}

int launch_b64_encode(const uint8_t* data, const uint64_t* data_off, const uint32_t* size, uint8_t* text,
                      const uint64_t* text_off, uint32_t n, uint32_t max_size, hipStream_t stream) {
  if (n == 0) return LBF_OK;
  const uint32_t tiles = std::max<uint32_t>(1u, (uint32_t)((b64_put_length(max_size) + kB64TileText - 1) / kB64TileText));
  return b64_tiled_launch(n, (tiles + kEncTilesPerGroup - 1) / kEncTilesPerGroup, [&](dim3 grid, uint32_t c0) {
    hipLaunchKernelGGL(b64_encode_kernel, grid, dim3(kB64Threads), 0, stream, data, data_off, size, text, text_off, tiles,
                       c0);
  });
}

}  // namespace lbf

using lbf::fail;

// A device array the caller passed must fit in the allocation it points into:
// a launch that would run past one (a digest array sized for fewer chunks than
// the launch writes) is refused before the kernel runs, since an out-of-bounds
// write is a GPU fault.  Memory HIP cannot place (an allocator it does not
// track) is not checked; the chunk bytes of a table launch are not either (the
// offsets are on the device).
static int check_fits(const void* p, uint64_t bytes, const char* what) {
  if (!p || bytes == 0) return LBF_OK;
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  if (hipMemGetAddressRange(&base, &size, const_cast<void*>(p)) != hipSuccess) {
    (void)hipGetLastError();
    return LBF_OK;
  }
  const uintptr_t b = reinterpret_cast<uintptr_t>(base), q = reinterpret_cast<uintptr_t>(p);
  if (q < b || q - b > size || bytes > size - (q - b))
    return fail(LBF_ERR_INVALID, std::string(what) + ": " + std::to_string(bytes) + " bytes from this pointer run past " +
                                     "its allocation (" + std::to_string(size - std::min<uintptr_t>(q - b, size)) +
                                     " bytes left)");
  return LBF_OK;
}

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
  if (int rc = check_fits(d_offsets, 8 * n, "lbf_sha1_launch: offsets")) return rc;
  if (int rc = check_fits(d_sizes, 4 * n, "lbf_sha1_launch: sizes")) return rc;
  if (int rc = check_fits(d_digests, 20 * n, "lbf_sha1_launch: digests")) return rc;
  if (int rc = check_fits(d_expected, 20 * n, "lbf_sha1_launch: expected")) return rc;
  if (int rc = check_fits(d_verdicts, n, "lbf_sha1_launch: verdicts")) return rc;
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
  if (int rc = check_fits(d_base, len, "lbf_sha1_uniform_launch: region")) return rc;
  if (int rc = check_fits(d_digests, 20 * n, "lbf_sha1_uniform_launch: digests")) return rc;
  if (int rc = check_fits(d_expected, 20 * n, "lbf_sha1_uniform_launch: expected")) return rc;
  if (int rc = check_fits(d_verdicts, n, "lbf_sha1_uniform_launch: verdicts")) return rc;
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
  const bool known = variant == 0 || lbf::shipped_variant(variant) ||
                     (lbf::g_extra_variants && lbf::g_extra_variants->known(variant));
  if (!known) return fail(LBF_ERR_INVALID, "unknown kernel variant (shipped: 0 auto, 1, 7, 10, 11, 12)");
  lbf::g_variant.store(variant);
  return LBF_OK;
}

extern "C" int lbf_get_kernel_variant(void) { return lbf::g_variant.load(); }

extern "C" int lbf_kernel_for(uint64_t n_chunks) { return lbf::pick_variant(n_chunks); }

extern "C" int lbf_fill_synthetic(uint8_t* d_buf, uint64_t len, uint64_t seed, uint64_t start, void* stream) {
  if (len == 0) return LBF_OK;
  if (!d_buf || (start & 7u) || (reinterpret_cast<uintptr_t>(d_buf) & 15u))
    return fail(LBF_ERR_INVALID, "lbf_fill_synthetic: need start%8==0 and a 16-byte aligned buffer");
  if (int rc = check_fits(d_buf, len, "lbf_fill_synthetic")) return rc;
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
