// tools/probe_rounds.hip -- diagnostic (not product code): cycles per 80-round
// step of the consumer's round chain alone (schedule words in registers), at
// one wave per SIMD, to separate the chain's own issue/latency cost from LDS
// and producer interference.
//   R: rounds only (compress_quads), 1 chain/lane
//   P: producer work only (expand 16 -> 80 words, no LDS stores)
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "sha1_device.hpp"

using namespace lbf;

__global__ void __launch_bounds__(64) rounds_only(uint32_t nsteps, uint32_t* out, unsigned long long* clk) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  uint4 w[20];
#pragma unroll
  for (int q = 0; q < 20; ++q) w[q] = make_uint4(i + q, i * 3 + q, i ^ q, i * 7);
  Digest s;
  s.init();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t k = 0; k < nsteps; ++k) {
    compress_quads(s, w);
    w[k % 20].x ^= s.h[0];  // keep the schedule live and varying
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[i] = s.h[0] ^ s.h[4];
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

__global__ void __launch_bounds__(64) expand_only(uint32_t nsteps, uint32_t* out, unsigned long long* clk) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  uint32_t acc = 0;
  uint32_t base[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) base[k] = i * 0x9E3779B9u + k;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t k = 0; k < nsteps; ++k) {
    uint32_t w[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) w[j] = bswap(base[j] ^ k);
#pragma unroll
    for (int r = 16; r < 80; ++r) {
      const uint32_t x = sched(w[(r + 13) & 15], w[(r + 8) & 15], w[(r + 2) & 15], w[r & 15]);
      w[r & 15] = x;
      acc += x;
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[i] = acc;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <typename K>
static void run(const char* name, K kern, uint32_t waves) {
  uint32_t* out;
  unsigned long long* clk;
  hipMalloc(&out, waves * 64 * 4);
  hipMalloc(&clk, waves * 8);
  const uint32_t nsteps = 2048;
  hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, nsteps, out, clk);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(kern, dim3(waves), dim3(64), 0, 0, nsteps, out, clk);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  unsigned long long* h = new unsigned long long[waves];
  hipMemcpy(h, clk, waves * 8, hipMemcpyDeviceToHost);
  double c = 0;
  for (uint32_t b = 0; b < waves; ++b) c += h[b];
  c /= waves;
  printf("%-12s waves=%5u  %.3f ms  cycles/step=%.0f\n", name, waves, ms, c / nsteps);
  delete[] h;
  hipFree(out);
  hipFree(clk);
}

int main() {
  for (uint32_t w : {256u, 1024u}) {
    run("rounds_only", rounds_only, w);
    run("expand_only", expand_only, w);
  }
  return 0;
}
