// tools/probe_latency.hip -- diagnostic (not product code): dependent-chain
// latency of the VALU ops on SHA-1's critical path, one wave alone on its SIMD.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define N 4096

template <int kOp>
__global__ void __launch_bounds__(64) chain(uint32_t seed, uint32_t* out, unsigned long long* clk) {
  uint32_t x = seed + threadIdx.x, y = seed * 3 + threadIdx.x, z = seed ^ threadIdx.x;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
#pragma unroll 64
  for (int i = 0; i < N; ++i) {
    if (kOp == 0) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x));
    if (kOp == 1) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
    if (kOp == 2) asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(x) : "v"(y));
    if (kOp == 3) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(y), "v"(z));
    if (kOp == 4) asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(y), "v"(z));
    if (kOp == 5) asm volatile("v_alignbit_b32 %0, %0, %0, 27\n\tv_add_u32_e32 %0, %0, %1" : "+v"(x) : "v"(y));
    // independent stream of the same ops (issue rate, not latency)
    if (kOp == 6) asm volatile("v_alignbit_b32 %0, %2, %2, 27\n\tv_add3_u32 %1, %2, %3, %2" : "+v"(x), "+v"(y) : "v"(z), "v"(seed));
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + threadIdx.x] = x ^ y;
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <int kOp>
static void run(const char* name, int ops_per_iter) {
  uint32_t* out;
  unsigned long long* clk;
  hipMalloc(&out, 256 * 64 * 4);
  hipMalloc(&clk, 256 * 8);
  hipLaunchKernelGGL(chain<kOp>, dim3(256), dim3(64), 0, 0, 7u, out, clk);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(chain<kOp>, dim3(256), dim3(64), 0, 0, 7u, out, clk);
  hipDeviceSynchronize();
  unsigned long long h[256];
  hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost);
  double c = 0;
  for (int b = 0; b < 256; ++b) c += h[b];
  c /= 256;
  printf("%-28s %.2f cycles per op\n", name, c / ((double)N * ops_per_iter));
  hipFree(out);
  hipFree(clk);
}

int main() {
  run<0>("alignbit chain", 1);
  run<1>("add3 chain", 1);
  run<2>("add_u32 (VOP2) chain", 1);
  run<3>("bitop3 chain", 1);
  run<4>("alignbit->add3 chain", 2);
  run<5>("alignbit->add_u32 chain", 2);
  run<6>("independent alignbit+add3", 2);
  return 0;
}
