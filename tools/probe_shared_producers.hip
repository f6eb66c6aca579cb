// tools/probe_shared_producers.hip -- diagnostic microbenchmark (not product code).
//
// Question: can two producer waves share one SIMD and still each finish a
// half step of W+K (40 schedule words with K, ten 1 KiB ds_write_b128) in well
// under twice the time one producer alone takes?  A lone producer spends
// ≈1,045 cycles per half, ≈345 of them on its stores (probe_producer.hip).  If
// one wave's stores drain while the other issues VALU, two producers per SIMD
// would fit the half-step budget of a pc4-style pair (≈1,800 cycles), and a
// 6-wave workgroup (two consumers alone on their SIMDs, four producers two to
// a SIMD) could give C4's 32 K chains pc4's consumer.
//
// One workgroup per CU (LDS), `waves` waves; the waves listed in `mask` run the
// producer loop, the others exit at once.  Each wave reports its SIMD (HW_ID)
// and cycles per half (s_memtime).
// Build: hipcc --offload-arch=gfx950 -O3 -I../bitflood_amd/csrc -I../include probe_shared_producers.hip -o build/probe_shared_producers
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

constexpr int kSlotU4 = 20 * 64;  // one W slot: 20 quads x 64 lanes (20 KiB)

__device__ __forceinline__ void half(uint32_t (&w)[16], uint4* out) {
#pragma unroll
  for (int q = 10; q < 20; ++q) {
    uint32_t x[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * q + j;
      x[j] = sched(w[(i + 13) & 15], w[(i + 8) & 15], w[(i + 2) & 15], w[i & 15]);
      w[i & 15] = x[j];
      x[j] += round_k(i);
    }
    out[q * 64] = make_uint4(x[0], x[1], x[2], x[3]);
  }
}

__global__ void __launch_bounds__(512) producers(uint32_t iters, uint32_t mask, uint32_t* out,
                                                 unsigned long long* clk, uint32_t* simd) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  const int wave = threadIdx.x / 64, lane = threadIdx.x % 64;
  const int slot_of = __popc(mask & ((1u << wave) - 1));  // this producer's own slot
  uint32_t id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
  const int rec = blockIdx.x * 8 + wave;
  if (lane == 0) simd[rec] = (id >> 4) & 3;
  if (!(mask >> wave & 1)) {
    if (lane == 0) clk[rec] = 0;
    return;
  }
  uint4* slot = lds + slot_of * kSlotU4 + lane;
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = lane * 0x9E3779B9u + k + wave;
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; ++it) {
    half(w, slot);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 16; ++k) x ^= w[k];
  out[rec * 64 + lane] = x ^ slot[0].x;
  if (lane == 0) clk[rec] = t1 - t0;
}

static void run(const char* name, int waves, uint32_t mask, uint32_t* out, unsigned long long* clk, uint32_t* simd) {
  const int lds_bytes = 140 * 1024;  // one workgroup per CU; up to 6 slots of 20 KiB
  CK(hipFuncSetAttribute((const void*)producers, hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes));
  const uint32_t iters = 20000;
  const int wgs = 256;
  hipLaunchKernelGGL(producers, dim3(wgs), dim3(64 * waves), lds_bytes, 0, iters, mask, out, clk, simd);
  hipLaunchKernelGGL(producers, dim3(wgs), dim3(64 * waves), lds_bytes, 0, iters, mask, out, clk, simd);
  CK(hipDeviceSynchronize());
  static unsigned long long h[256 * 8];
  static uint32_t s[256 * 8];
  CK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
  CK(hipMemcpy(s, simd, sizeof(s), hipMemcpyDeviceToHost));
  // per wave slot: mean cycles/half over the workgroups, and how often it shared its SIMD with another producer
  printf("%-34s", name);
  for (int wv = 0; wv < waves; ++wv) {
    if (!(mask >> wv & 1)) continue;
    double sum = 0;
    int shared = 0;
    for (int b = 0; b < wgs; ++b) {
      sum += (double)h[b * 8 + wv];
      for (int o = 0; o < waves; ++o)
        if (o != wv && (mask >> o & 1) && s[b * 8 + o] == s[b * 8 + wv]) {
          ++shared;
          break;
        }
    }
    printf(" w%d=%7.1f(shared %3d/256)", wv, sum / wgs / iters, shared);
  }
  printf("\n");
  // SIMD pattern of the first workgroup
  printf("%-34s simd of each wave in wg0:", "");
  for (int wv = 0; wv < waves; ++wv) printf(" %u", s[wv]);
  printf("\n");
}

int main() {
  uint32_t *out, *simd;
  unsigned long long* clk;
  CK(hipMalloc(&out, 256 * 8 * 64 * 4));
  CK(hipMalloc(&clk, 256 * 8 * 8));
  CK(hipMalloc(&simd, 256 * 8 * 4));
  run("1 wave, producer alone", 1, 0x1, out, clk, simd);
  run("4 waves, 4 producers (one per SIMD)", 4, 0xF, out, clk, simd);
  run("5 waves, producers w0 + w4", 5, 0x11, out, clk, simd);
  run("6 waves, producers w0 w1 w4 w5", 6, 0x33, out, clk, simd);
  run("6 waves, all six producers", 6, 0x3F, out, clk, simd);
  return 0;
}
