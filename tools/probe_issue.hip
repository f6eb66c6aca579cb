// tools/probe_issue.hip -- diagnostic microbenchmark (not product code).
//
// Separates the chunk-hash kernel's time into issue-bound compute and memory:
//   P-compute: SHA-1 compressions of an in-register block (no global loads),
//              4096 blocks per lane, at several chain counts;
//   clock:     s_memtime / s_memrealtime (100 MHz) inside the same kernel.
// Build: hipcc --offload-arch=gfx950 -O3 -I../bitflood_amd/csrc -I../include probe_issue.hip -o build/probe_issue
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

__global__ void __launch_bounds__(256) compute_only(uint32_t nblk, uint32_t* out, unsigned long long* clk) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  Digest s;
  s.init();
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = i * 0x9E3779B9u + k;
  for (uint32_t b = 0; b < nblk; ++b) {
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = w[k] ^ s.h[k % 5];  // cheap per-block variation
    compress(s, x);
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  unsigned long long r1 = __builtin_amdgcn_s_memrealtime();
  out[i] = s.h[0] ^ s.h[1] ^ s.h[2] ^ s.h[3] ^ s.h[4];
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = t1 - t0;
    clk[2 * blockIdx.x + 1] = r1 - r0;
  }
}

int main(int argc, char** argv) {
  const uint32_t nblk = argc > 1 ? atoi(argv[1]) : 4096;
  const uint32_t chains_list[] = {16384, 32768, 65536, 131072, 262144};
  uint32_t* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, 262144 * 4));
  CK(hipMalloc(&clk, 2 * 262144 * 8));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (uint32_t tpb : {64u, 256u}) {
    for (uint32_t chains : chains_list) {
      const uint32_t blocks = chains / tpb;
      hipLaunchKernelGGL(compute_only, dim3(blocks), dim3(tpb), 0, 0, nblk, out, clk);  // warm
      CK(hipDeviceSynchronize());
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(compute_only, dim3(blocks), dim3(tpb), 0, 0, nblk, out, clk);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      unsigned long long* h = (unsigned long long*)malloc(2 * blocks * 8);
      CK(hipMemcpy(h, clk, 2 * blocks * 8, hipMemcpyDeviceToHost));
      double cyc = 0, real = 0;
      for (uint32_t b = 0; b < blocks; ++b) {
        cyc += h[2 * b];
        real += h[2 * b + 1];
      }
      cyc /= blocks;
      real /= blocks;
      const double ghz = cyc / (real * 10.0);  // memrealtime ticks at 100 MHz
      const double bytes = (double)chains * nblk * 64.0;
      printf("tpb=%3u chains=%6u waves=%5u  %8.3f ms  %7.1f GB/s-equiv  clk=%.3f GHz  cyc/blk/wave=%.0f\n",
             tpb, chains, chains / 64, ms, bytes / ms / 1e6, ghz, cyc / nblk);
      free(h);
    }
  }
  return 0;
}
