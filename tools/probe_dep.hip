// per-op VALU throughput with k interleaved dependent chains per wave
#include <hip/hip_runtime.h>
#include <stdio.h>
#define REP8(x) x x x x x x x x
#define REP32(x) REP8(x) REP8(x) REP8(x) REP8(x)
__global__ void __launch_bounds__(64) k_xor_1(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_xor_b32 v10, v10, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v10, v10, v0\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_xor_2(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_xor_b32 v10, v10, v0\n v_xor_b32 v11, v11, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v11, v11, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v11, v11, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v11, v11, v0\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_xor_4(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_xor_b32 v10, v10, v0\n v_xor_b32 v11, v11, v0\n v_xor_b32 v12, v12, v0\n v_xor_b32 v13, v13, v0\n v_xor_b32 v10, v10, v0\n v_xor_b32 v11, v11, v0\n v_xor_b32 v12, v12, v0\n v_xor_b32 v13, v13, v0\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_xor_8(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_xor_b32 v10, v10, v0\n v_xor_b32 v11, v11, v0\n v_xor_b32 v12, v12, v0\n v_xor_b32 v13, v13, v0\n v_xor_b32 v14, v14, v0\n v_xor_b32 v15, v15, v0\n v_xor_b32 v16, v16, v0\n v_xor_b32 v17, v17, v0\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_alignbit_1(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v10, v10, v10, 27\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_alignbit_2(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_alignbit_4(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_alignbit_8(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_alignbit_b32 v10, v10, v10, 27\n v_alignbit_b32 v11, v11, v11, 27\n v_alignbit_b32 v12, v12, v12, 27\n v_alignbit_b32 v13, v13, v13, 27\n v_alignbit_b32 v14, v14, v14, 27\n v_alignbit_b32 v15, v15, v15, 27\n v_alignbit_b32 v16, v16, v16, 27\n v_alignbit_b32 v17, v17, v17, 27\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_add3_1(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v10, v10, v0, v1\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_add3_2(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v11, v11, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v11, v11, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v11, v11, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v11, v11, v0, v1\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_add3_4(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v11, v11, v0, v1\n v_add3_u32 v12, v12, v0, v1\n v_add3_u32 v13, v13, v0, v1\n v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v11, v11, v0, v1\n v_add3_u32 v12, v12, v0, v1\n v_add3_u32 v13, v13, v0, v1\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_add3_8(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_add3_u32 v10, v10, v0, v1\n v_add3_u32 v11, v11, v0, v1\n v_add3_u32 v12, v12, v0, v1\n v_add3_u32 v13, v13, v0, v1\n v_add3_u32 v14, v14, v0, v1\n v_add3_u32 v15, v15, v0, v1\n v_add3_u32 v16, v16, v0, v1\n v_add3_u32 v17, v17, v0, v1\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_bitop3_1(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_bitop3_2(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v11, v11, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v11, v11, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v11, v11, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v11, v11, v0, v1 bitop3:0x96\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_bitop3_4(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v11, v11, v0, v1 bitop3:0x96\n v_bitop3_b32 v12, v12, v0, v1 bitop3:0x96\n v_bitop3_b32 v13, v13, v0, v1 bitop3:0x96\n v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v11, v11, v0, v1 bitop3:0x96\n v_bitop3_b32 v12, v12, v0, v1 bitop3:0x96\n v_bitop3_b32 v13, v13, v0, v1 bitop3:0x96\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}
__global__ void __launch_bounds__(64) k_bitop3_8(int iters, unsigned long long* clk) {
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < iters; ++i) {
    asm volatile(REP32("v_bitop3_b32 v10, v10, v0, v1 bitop3:0x96\n v_bitop3_b32 v11, v11, v0, v1 bitop3:0x96\n v_bitop3_b32 v12, v12, v0, v1 bitop3:0x96\n v_bitop3_b32 v13, v13, v0, v1 bitop3:0x96\n v_bitop3_b32 v14, v14, v0, v1 bitop3:0x96\n v_bitop3_b32 v15, v15, v0, v1 bitop3:0x96\n v_bitop3_b32 v16, v16, v0, v1 bitop3:0x96\n v_bitop3_b32 v17, v17, v0, v1 bitop3:0x96\n ") ::: "v10","v11","v12","v13","v14","v15","v16","v17","v0","v1");
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;
}

template <typename K> static double run(K kern, int w) {
  unsigned long long* clk; const int blocks = 256 * 4 * w; hipMalloc(&clk, blocks * 8);
  const int iters = 64;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, iters, clk); hipDeviceSynchronize();
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, iters, clk); hipDeviceSynchronize();
  unsigned long long* h = new unsigned long long[blocks]; hipMemcpy(h, clk, blocks * 8, hipMemcpyDeviceToHost);
  double c = 0; for (int b = 0; b < blocks; ++b) c += h[b]; c /= blocks; delete[] h; hipFree(clk);
  return c / (iters * 32.0 * 8) / w;  // cycles per instruction per SIMD
}
int main() {
  printf("%-10s %6s %8s %8s %8s   (cycles per wave-instruction per SIMD)\n", "op", "chains", "w=1", "w=2", "w=4");
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "xor", 1, run(k_xor_1, 1), run(k_xor_1, 2), run(k_xor_1, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "xor", 2, run(k_xor_2, 1), run(k_xor_2, 2), run(k_xor_2, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "xor", 4, run(k_xor_4, 1), run(k_xor_4, 2), run(k_xor_4, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "xor", 8, run(k_xor_8, 1), run(k_xor_8, 2), run(k_xor_8, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "alignbit", 1, run(k_alignbit_1, 1), run(k_alignbit_1, 2), run(k_alignbit_1, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "alignbit", 2, run(k_alignbit_2, 1), run(k_alignbit_2, 2), run(k_alignbit_2, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "alignbit", 4, run(k_alignbit_4, 1), run(k_alignbit_4, 2), run(k_alignbit_4, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "alignbit", 8, run(k_alignbit_8, 1), run(k_alignbit_8, 2), run(k_alignbit_8, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "add3", 1, run(k_add3_1, 1), run(k_add3_1, 2), run(k_add3_1, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "add3", 2, run(k_add3_2, 1), run(k_add3_2, 2), run(k_add3_2, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "add3", 4, run(k_add3_4, 1), run(k_add3_4, 2), run(k_add3_4, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "add3", 8, run(k_add3_8, 1), run(k_add3_8, 2), run(k_add3_8, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "bitop3", 1, run(k_bitop3_1, 1), run(k_bitop3_1, 2), run(k_bitop3_1, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "bitop3", 2, run(k_bitop3_2, 1), run(k_bitop3_2, 2), run(k_bitop3_2, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "bitop3", 4, run(k_bitop3_4, 1), run(k_bitop3_4, 2), run(k_bitop3_4, 4));
  printf("%-10s %6d %8.2f %8.2f %8.2f\n", "bitop3", 8, run(k_bitop3_8, 1), run(k_bitop3_8, 2), run(k_bitop3_8, 4));
  return 0;
}
