// tools/probe_producer.hip -- diagnostic microbenchmark (not product code).
//
// Where does a producer wave's time go?  In pc4 a producer spends ≈1,280
// cycles per half step (tools/probe_pc.hip, profiles/r01/probe_pc4_diag.log)
// for ≈170 instructions, twice its issue floor.  One wave per CU runs the
// half-step loop of expand_store_wk on its own, with the stores and the round
// constants in several forms:
//   mode 0  expand_store_wk<1> as shipped: ds_write_b128, K as a literal
//   mode 1  same arithmetic, stores into an asm sink (no LDS traffic)
//   mode 2  ds_write_b64 pairs instead of ds_write_b128
//   mode 3  K from VGPRs (v_add_u32 with no literal), ds_write_b128
//   mode 4  first half as shipped: raw block from LDS + byte swaps + words 0..39
//   mode 5  mode 0 with the ten stores issued at the end of the half
// Build: hipcc --offload-arch=gfx950 -O3 -I../bitflood_amd/csrc -I../include probe_producer.hip -o build/probe_producer
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "sha1_device.hpp"

using namespace lbf;

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e = (x);                                                                 \
    if (e != hipSuccess) {                                                              \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

constexpr int kSlotU4 = 20 * 64;

template <int kMode>
__device__ __forceinline__ void half(uint32_t (&w)[16], uint4* out, const uint4* raw, const RoundK& K) {
  if (kMode == 4) {
    block_from_vec(w, raw[0], raw[64], raw[128], raw[192]);
    expand_store_wk<0>(w, out, 64);
    return;
  }
  uint4 keep[10];
#pragma unroll
  for (int q = 10; q < 20; ++q) {
    uint32_t x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * q + j;
      x[j] = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]);
      w[i & 15] = x[j];
      x[j] += (kMode == 3) ? K.k[i / 20] : round_k(i);
    }
    const uint4 v = make_uint4(x[0], x[1], x[2], x[3]);
    if (kMode == 0 || kMode == 3) {
      out[q * 64] = v;
    } else if (kMode == 1) {
      asm volatile("" ::"v"(v.x), "v"(v.y), "v"(v.z), "v"(v.w));
    } else if (kMode == 2) {
      uint2* o2 = reinterpret_cast<uint2*>(out + q * 64);
      o2[0] = make_uint2(v.x, v.y);
      o2[1] = make_uint2(v.z, v.w);
    } else {
      keep[q - 10] = v;
    }
  }
  if (kMode == 5) {
#pragma unroll
    for (int q = 10; q < 20; ++q) out[q * 64] = keep[q - 10];
  }
}

template <int kMode>
__global__ void __launch_bounds__(64) producer(uint32_t iters, uint32_t* out, unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];  // W slot | raw slot
  const int lane = threadIdx.x;
  uint4* slot = lds;
  uint4* raw = lds + kSlotU4;
  for (int q = 0; q < 4; ++q) raw[q * 64 + lane] = make_uint4(lane * q, lane + q, lane ^ q, q);
  __syncthreads();
  const RoundK K;
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = lane * 0x9E3779B9u + k;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
    half<kMode>(w, slot + lane, raw + lane, K);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) x ^= w[k];
  out[blockIdx.x * 64 + lane] = x ^ slot[lane].x;
  if (lane == 0) clk[blockIdx.x] = t1 - t0;
}

template <int kMode>
static void run(const char* name, uint32_t* out, unsigned long long* clk) {
  const int lds_bytes = 100 * 1024;  // one wave per CU
  CK(hipFuncSetAttribute((const void*)producer<kMode>, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
  const uint32_t iters = 20000;
  const int wgs = 256;
  hipLaunchKernelGGL(producer<kMode>, dim3(wgs), dim3(64), lds_bytes, 0, iters, out, clk);
  hipLaunchKernelGGL(producer<kMode>, dim3(wgs), dim3(64), lds_bytes, 0, iters, out, clk);
  CK(hipDeviceSynchronize());
  unsigned long long h[256];
  CK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
  double sum = 0;
  for (int b = 0; b < wgs; ++b) sum += (double)h[b];
  // s_memtime counts shader-clock cycles
  printf("%-28s cycles/half=%7.1f\n", name, sum / wgs / iters);
}

int main() {
  uint32_t* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, 256 * 64 * 4));
  CK(hipMalloc(&clk, 256 * 8));
  run<0>("0 b128 literal-K", out, clk);
  run<1>("1 no stores", out, clk);
  run<2>("2 b64 stores", out, clk);
  run<3>("3 b128 vgpr-K", out, clk);
  run<4>("4 first half (raw+bswap)", out, clk);
  run<5>("5 b128 stores at end", out, clk);
  return 0;
}
