// tools/probe_banks.hip -- diagnostic (not product code): single-wave issue cost
// of independent VALU streams by instruction form and VGPR bank pattern
// (register numbers fixed in the asm; values are don't-care).
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(x) x x x x x x x x
#define REP64(x) REP8(REP8(x))

#define KERNEL(name, body)                                                              \
  __global__ void __launch_bounds__(64) name(int iters, unsigned long long* clk) {     \
    unsigned long long t0 = __builtin_amdgcn_s_memtime();                              \
    for (int i = 0; i < iters; ++i) {                                                  \
      asm volatile(REP64(body) ::: "v10", "v11", "v12", "v13", "v20", "v21", "v22", "v23", \
                   "v0", "v1", "v2", "v3", "v4", "v5", "v6", "v7", "v8", "v9");          \
    }                                                                                  \
    unsigned long long t1 = __builtin_amdgcn_s_memtime();                              \
    if (threadIdx.x == 0) clk[blockIdx.x] = t1 - t0;                                   \
  }

// 4 independent destinations per group so no instruction waits on the previous
KERNEL(k_xor, "v_xor_b32 v10, v0, v1\n v_xor_b32 v11, v2, v3\n v_xor_b32 v12, v4, v5\n v_xor_b32 v13, v6, v7\n")
KERNEL(k_align_same, "v_alignbit_b32 v10, v0, v0, 27\n v_alignbit_b32 v11, v1, v1, 27\n v_alignbit_b32 v12, v2, v2, 27\n v_alignbit_b32 v13, v3, v3, 27\n")
KERNEL(k_align_diff, "v_alignbit_b32 v10, v0, v1, 27\n v_alignbit_b32 v11, v1, v2, 27\n v_alignbit_b32 v12, v2, v3, 27\n v_alignbit_b32 v13, v3, v4, 27\n")
KERNEL(k_add3_banks3, "v_add3_u32 v10, v0, v1, v2\n v_add3_u32 v11, v1, v2, v3\n v_add3_u32 v12, v2, v3, v4\n v_add3_u32 v13, v3, v4, v5\n")
KERNEL(k_add3_bank1, "v_add3_u32 v10, v0, v4, v8\n v_add3_u32 v11, v1, v5, v9\n v_add3_u32 v12, v0, v4, v8\n v_add3_u32 v13, v1, v5, v9\n")
KERNEL(k_add3_sgpr, "v_add3_u32 v10, v0, v1, s4\n v_add3_u32 v11, v1, v2, s4\n v_add3_u32 v12, v2, v3, s4\n v_add3_u32 v13, v3, v4, s4\n")
KERNEL(k_bitop3, "v_bitop3_b32 v10, v0, v1, v2 bitop3:0x96\n v_bitop3_b32 v11, v1, v2, v3 bitop3:0x96\n v_bitop3_b32 v12, v2, v3, v4 bitop3:0x96\n v_bitop3_b32 v13, v3, v4, v5 bitop3:0x96\n")
KERNEL(k_mix, "v_alignbit_b32 v10, v0, v0, 27\n v_add3_u32 v11, v1, v2, v3\n v_bitop3_b32 v12, v4, v5, v6 bitop3:0xca\n v_xor_b32 v13, v7, v8\n")

template <typename K>
static void run(const char* name, K kern, int waves_per_cu_simd) {
  unsigned long long* clk;
  const int blocks = 256 * waves_per_cu_simd;
  hipMalloc(&clk, blocks * 8);
  const int iters = 256;
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, iters, clk);
  hipDeviceSynchronize();
  hipLaunchKernelGGL(kern, dim3(blocks), dim3(64), 0, 0, iters, clk);
  hipDeviceSynchronize();
  unsigned long long* h = new unsigned long long[blocks];
  hipMemcpy(h, clk, blocks * 8, hipMemcpyDeviceToHost);
  double c = 0;
  for (int b = 0; b < blocks; ++b) c += h[b];
  c /= blocks;
  printf("%-16s blocks=%5d  %.2f cycles per instruction per wave\n", name, blocks, c / (iters * 64.0 * 4));
  delete[] h;
  hipFree(clk);
}

int main() {
  for (int w : {1, 8}) {
    run("xor(VOP2)", k_xor, w);
    run("alignbit a,a", k_align_same, w);
    run("alignbit a,b", k_align_diff, w);
    run("add3 3banks", k_add3_banks3, w);
    run("add3 1bank", k_add3_bank1, w);
    run("add3 +sgpr", k_add3_sgpr, w);
    run("bitop3", k_bitop3, w);
    run("mix", k_mix, w);
  }
  return 0;
}
