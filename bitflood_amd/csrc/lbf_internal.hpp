// lbf_internal.hpp -- shared internals of liblbfhash.so (not part of the ABI).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "lbf_hash.h"

namespace lbf {

// Thread-local last-error slot behind lbf_last_error().
void set_error(const std::string& msg);
int fail(int status, const std::string& msg);
int hip_fail(hipError_t e, const char* what);

#define LBF_HIP_TRY(expr)                                   \
  do {                                                      \
    hipError_t lbf_e_ = (expr);                             \
    if (lbf_e_ != hipSuccess) return ::lbf::hip_fail(lbf_e_, #expr); \
  } while (0)

// Kernel-side parameter block shared by every chunk-hash kernel variant.
struct ChunkParams {
  const uint8_t* base;
  const uint64_t* offsets;   // null => uniform chunking of [0, len)
  const uint32_t* sizes;
  uint64_t len;              // uniform: region length
  uint64_t first_chunk;      // uniform: index of chunk 0 of this launch
  uint32_t chunk_size;       // uniform
  uint32_t n;                // chunks in this launch
  uint8_t* digests;          // n*20 bytes or null
  const uint8_t* expected;   // n*20 bytes or null
  uint8_t* verdicts;         // n bytes or null
};

int pick_variant(uint64_t n);
int launch_chunks(const ChunkParams& p, hipStream_t stream);

// Device base64 decode (kern_b64.hpp): n chunks' text -> bytes, on `stream`.
struct B64Launch {
  const uint8_t* text;
  uint8_t* scratch;
  const uint64_t* text_off;
  const uint64_t* sext_off;
  const uint32_t* text_len;
  uint8_t* out;
  const uint64_t* out_off;
  const uint32_t* cap;
  uint32_t* sizes;
  uint8_t* over;
  uint8_t* redo;  // n bytes, zero on entry: the chunks the one-pass decode hands to the general one
  uint32_t n;
  uint32_t max_text_len;  // the longest text and the largest cap: the one-pass decode's tiles per chunk
  uint32_t max_cap;
};
int launch_b64_decode(const B64Launch& b, hipStream_t stream);
// Device base64 encode (kern_b64.hpp): n chunks' bytes -> their SendChunk text.
// max_size: the largest chunk (sets the tiles per chunk).
int launch_b64_encode(const uint8_t* data, const uint64_t* data_off, const uint32_t* size, uint8_t* text,
                      const uint64_t* text_off, uint32_t n, uint32_t max_size, hipStream_t stream);

// Kernel variants beyond the shipped ones (1, 7, 10, 11, 12).  Null in the
// shipped library; the A/B library of tools/experimental/ points it at its
// superseded and diagnostic variants when it loads.
struct ExtraVariants {
  bool (*known)(int variant);
  bool (*launch)(int variant, const ChunkParams& p, hipStream_t stream);
};
extern const ExtraVariants* g_extra_variants;

}  // namespace lbf
