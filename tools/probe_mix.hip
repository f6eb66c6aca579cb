#include <hip/hip_runtime.h>
#include <stdio.h>
#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)
__global__ void __launch_bounds__(64) k_mix4_1(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_xor_b32 v10, v10, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_xor_b32 v10, v10, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_xor_b32 v10, v10, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_xor_b32 v10, v10, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_xor_b32 v10, v10, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_xor_b32 v10, v10, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_xor_b32 v10, v10, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_xor_b32 v10, v10, v1\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v1","v2");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_align_add3_1(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_add3_u32 v10, v10, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_add3_u32 v10, v10, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_add3_u32 v10, v10, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_add3_u32 v10, v10, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_add3_u32 v10, v10, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_add3_u32 v10, v10, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_add3_u32 v10, v10, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_add3_u32 v10, v10, v1, v2\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v1","v2");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_mix4_2(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_bitop3_b32 v11, v11, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_xor_b32 v10, v10, v1\n v_xor_b32 v11, v11, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_bitop3_b32 v11, v11, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_xor_b32 v10, v10, v1\n v_xor_b32 v11, v11, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_bitop3_b32 v11, v11, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_xor_b32 v10, v10, v1\n v_xor_b32 v11, v11, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_bitop3_b32 v11, v11, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_xor_b32 v10, v10, v1\n v_xor_b32 v11, v11, v1\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v1","v2");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_align_add3_2(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v1","v2");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_mix4_4(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_bitop3_b32 v11, v11, v1, v2 bitop3:0x96\n v_bitop3_b32 v12, v12, v1, v2 bitop3:0x96\n v_bitop3_b32 v13, v13, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_add3_u32 v12, v12, v1, v2\n v_add3_u32 v13, v13, v1, v2\n v_xor_b32 v10, v10, v1\n v_xor_b32 v11, v11, v1\n v_xor_b32 v12, v12, v1\n v_xor_b32 v13, v13, v1\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_bitop3_b32 v11, v11, v1, v2 bitop3:0x96\n v_bitop3_b32 v12, v12, v1, v2 bitop3:0x96\n v_bitop3_b32 v13, v13, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_add3_u32 v12, v12, v1, v2\n v_add3_u32 v13, v13, v1, v2\n v_xor_b32 v10, v10, v1\n v_xor_b32 v11, v11, v1\n v_xor_b32 v12, v12, v1\n v_xor_b32 v13, v13, v1\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v1","v2");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_align_add3_4(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_add3_u32 v12, v12, v1, v2\n v_add3_u32 v13, v13, v1, v2\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_add3_u32 v12, v12, v1, v2\n v_add3_u32 v13, v13, v1, v2\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v1","v2");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_mix4_8(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_alignbit_b32 v14, v14, v14, 27\n v_alignbit_b32 v15, v15, v15, 27\n v_alignbit_b32 v16, v16, v16, 27\n v_alignbit_b32 v17, v17, v17, 27\n v_bitop3_b32 v10, v10, v1, v2 bitop3:0x96\n v_bitop3_b32 v11, v11, v1, v2 bitop3:0x96\n v_bitop3_b32 v12, v12, v1, v2 bitop3:0x96\n v_bitop3_b32 v13, v13, v1, v2 bitop3:0x96\n v_bitop3_b32 v14, v14, v1, v2 bitop3:0x96\n v_bitop3_b32 v15, v15, v1, v2 bitop3:0x96\n v_bitop3_b32 v16, v16, v1, v2 bitop3:0x96\n v_bitop3_b32 v17, v17, v1, v2 bitop3:0x96\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_add3_u32 v12, v12, v1, v2\n v_add3_u32 v13, v13, v1, v2\n v_add3_u32 v14, v14, v1, v2\n v_add3_u32 v15, v15, v1, v2\n v_add3_u32 v16, v16, v1, v2\n v_add3_u32 v17, v17, v1, v2\n v_xor_b32 v10, v10, v1\n v_xor_b32 v11, v11, v1\n v_xor_b32 v12, v12, v1\n v_xor_b32 v13, v13, v1\n v_xor_b32 v14, v14, v1\n v_xor_b32 v15, v15, v1\n v_xor_b32 v16, v16, v1\n v_xor_b32 v17, v17, v1\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v1","v2");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_align_add3_8(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_alignbit_b32 v14, v14, v14, 27\n v_alignbit_b32 v15, v15, v15, 27\n v_alignbit_b32 v16, v16, v16, 27\n v_alignbit_b32 v17, v17, v17, 27\n v_add3_u32 v10, v10, v1, v2\n v_add3_u32 v11, v11, v1, v2\n v_add3_u32 v12, v12, v1, v2\n v_add3_u32 v13, v13, v1, v2\n v_add3_u32 v14, v14, v1, v2\n v_add3_u32 v15, v15, v1, v2\n v_add3_u32 v16, v16, v1, v2\n v_add3_u32 v17, v17, v1, v2\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v1","v2");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <typename K> static double run(K kern, int w, int per) {
  unsigned long long* clk; const int blocks = 256 * 4 * w; hipMalloc(&clk, blocks * 8);
  const int iters = 32;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, iters, clk); hipDeviceSynchronize();
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, iters, clk); hipDeviceSynchronize();
  unsigned long long* h = new unsigned long long[blocks]; hipMemcpy(h, clk, blocks * 8, hipMemcpyDeviceToHost);
  double c = 0; for (int b = 0; b < blocks; ++b) c += h[b]; c /= blocks; delete[] h; hipFree(clk);
  return c / (iters * 32.0 * per) / w;
}
int main() {
  printf("%-12s %6s %8s %8s %8s   (cycles per wave-instruction per SIMD)\n", "pattern", "chains", "w=1", "w=2", "w=4");
  printf("%-12s %6d %8.2f %8.2f %8.2f\n", "mix4", 1, run(k_mix4_1, 1, 32), run(k_mix4_1, 2, 32), run(k_mix4_1, 4, 32));
  printf("%-12s %6d %8.2f %8.2f %8.2f\n", "align_add3", 1, run(k_align_add3_1, 1, 16), run(k_align_add3_1, 2, 16), run(k_align_add3_1, 4, 16));
  printf("%-12s %6d %8.2f %8.2f %8.2f\n", "mix4", 2, run(k_mix4_2, 1, 32), run(k_mix4_2, 2, 32), run(k_mix4_2, 4, 32));
  printf("%-12s %6d %8.2f %8.2f %8.2f\n", "align_add3", 2, run(k_align_add3_2, 1, 16), run(k_align_add3_2, 2, 16), run(k_align_add3_2, 4, 16));
  printf("%-12s %6d %8.2f %8.2f %8.2f\n", "mix4", 4, run(k_mix4_4, 1, 32), run(k_mix4_4, 2, 32), run(k_mix4_4, 4, 32));
  printf("%-12s %6d %8.2f %8.2f %8.2f\n", "align_add3", 4, run(k_align_add3_4, 1, 16), run(k_align_add3_4, 2, 16), run(k_align_add3_4, 4, 16));
  printf("%-12s %6d %8.2f %8.2f %8.2f\n", "mix4", 8, run(k_mix4_8, 1, 32), run(k_mix4_8, 2, 32), run(k_mix4_8, 4, 32));
  printf("%-12s %6d %8.2f %8.2f %8.2f\n", "align_add3", 8, run(k_align_add3_8, 1, 16), run(k_align_add3_8, 2, 16), run(k_align_add3_8, 4, 16));
  return 0;
}
