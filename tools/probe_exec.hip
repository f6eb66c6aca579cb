// tools/probe_exec.hip -- diagnostic microbenchmark (not product code).
//
// Does a wave whose EXEC mask holds only some lanes issue its VALU stream any
// faster?  Each lane runs an in-register SHA-1 chain (sha1_device.hpp's
// compress, no global loads) of `nblk` blocks; lanes at or above `active` in
// each wave skip the loop.  Launches of W waves of 64 threads, timed with HIP
// events: the time is one chain's (all chains run side by side), so if a
// half-active wave issued in half the cycles the time would halve.
// Build: hipcc --offload-arch=gfx950 -O3 -Ibitflood_amd/csrc -Iinclude tools/probe_exec.hip -o tools/build/probe_exec
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "sha1_device.hpp"

using namespace lbf;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

__global__ void __launch_bounds__(256) chains(uint32_t nblk, uint32_t active, uint32_t* out) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  Digest s;
  s.init();
  if ((threadIdx.x & 63) < active) {
    uint32_t w[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) w[k] = i * 0x9E3779B9u + k;
    for (uint32_t b = 0; b < nblk; ++b) {
      uint32_t x[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) x[k] = w[k] ^ s.h[k % 5];
      compress(s, x);
    }
  }
  out[i] = s.h[0] ^ s.h[1] ^ s.h[2] ^ s.h[3] ^ s.h[4];
}

int main(int argc, char** argv) {
  const uint32_t nblk = argc > 1 ? (uint32_t)atoi(argv[1]) : 1024;
  uint32_t* out = nullptr;
  const uint32_t max_waves = 4096;
  CK(hipMalloc(&out, (size_t)max_waves * 64 * 4));
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  struct Case {
    uint32_t waves, threads, active;
  } cases[] = {{256, 64, 64},   {256, 64, 32},   {256, 64, 16},   {256, 64, 1},    {1024, 64, 64},
               {1024, 64, 32},  {1024, 64, 16},  {1024, 256, 64}, {1024, 256, 32}, {2048, 256, 32},
               {2048, 256, 64}, {512, 256, 32},  {512, 256, 64}};
  for (const Case& c : cases) {
    const uint32_t blocks = c.waves * 64 / c.threads;
    hipLaunchKernelGGL(chains, dim3(blocks), dim3(c.threads), 0, 0, nblk / 8, c.active, out);  // warm
    CK(hipDeviceSynchronize());
    float best = 1e30f;
    for (int r = 0; r < 3; ++r) {
      CK(hipEventRecord(a, 0));
      hipLaunchKernelGGL(chains, dim3(blocks), dim3(c.threads), 0, 0, nblk, c.active, out);
      CK(hipEventRecord(b, 0));
      CK(hipEventSynchronize(b));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, a, b));
      if (ms < best) best = ms;
    }
    const double chains_n = (double)c.waves * c.active;
    printf("{\"waves\": %u, \"threads_per_block\": %u, \"active_lanes\": %u, \"chains\": %.0f, \"nblk\": %u, "
           "\"ms\": %.4f, \"ns_per_block_per_chain\": %.2f, \"chain_bytes_per_ns\": %.2f}\n",
           c.waves, c.threads, c.active, chains_n, nblk, best, best * 1e6 / nblk, chains_n * nblk * 64 / (best * 1e6));
    fflush(stdout);
  }
  CK(hipFree(out));
  return 0;
}
