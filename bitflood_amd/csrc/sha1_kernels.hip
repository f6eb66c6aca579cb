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
#include <hip/hip_runtime.h>

#include <atomic>

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

}  // namespace

int launch_chunks(const ChunkParams& p, hipStream_t stream) {
  if (p.n == 0) return LBF_OK;
  // Few chains (C2: 16,384) -> 64-thread workgroups so the waves spread over
  // every CU; many chains -> 256-thread workgroups.
  const uint32_t threads = p.n <= 65536u ? 64u : 256u;
  const uint32_t blocks = (p.n + threads - 1) / threads;
  if (p.offsets) {
    hipLaunchKernelGGL(sha1_lane_kernel<false>, dim3(blocks), dim3(threads), 0, stream, p);
  } else {
    hipLaunchKernelGGL(sha1_lane_kernel<true>, dim3(blocks), dim3(threads), 0, stream, p);
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
  if (variant < 0 || variant > 1) return fail(LBF_ERR_INVALID, "unknown kernel variant");
  lbf::g_variant.store(variant);
  return LBF_OK;
}

extern "C" int lbf_get_kernel_variant(void) { return lbf::g_variant.load(); }

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
  hipEvent_t e0, e1;
  LBF_HIP_TRY(hipEventCreate(&e0));
  LBF_HIP_TRY(hipEventCreate(&e1));
  int rc = LBF_OK;
  LBF_HIP_TRY(hipEventRecord(e0, s));
  for (int r = 0; r < reps && rc == LBF_OK; ++r)
    rc = lbf_sha1_uniform_launch(d_base, len, chunk_size, first_chunk, n, d_digests, nullptr, nullptr, stream);
  LBF_HIP_TRY(hipEventRecord(e1, s));
  LBF_HIP_TRY(hipEventSynchronize(e1));
  float ms = 0.f;
  LBF_HIP_TRY(hipEventElapsedTime(&ms, e0, e1));
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  if (rc != LBF_OK) return rc;
  *out_ms_per_launch = ms / (float)reps;
  return LBF_OK;
}
