// tools/probe_valu_rate.hip -- diagnostic microbenchmark (not product code).
//
// Issue throughput of single VALU instructions on one SIMD at 1, 2 and 4 waves
// per SIMD: eight independent accumulators, each instruction written in asm so
// the compiler cannot pick another form.  The SHA-1 kernels are built from
// v_add_u32 / v_add3_u32 / v_alignbit_b32 / v_bitop3_b32 (3-input xor too) / v_perm;
// v_fma_f32 is the reference the guide documents (2 cycles per wave-instruction
// on a SIMD with two waves, 4 for one wave alone).  Output: ns per
// wave-instruction per SIMD, and that ratio to v_fma_f32's.
// Build: hipcc --offload-arch=gfx950 -O3 tools/probe_valu_rate.hip -o tools/build/probe_valu_rate
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

#define ACC8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)

#define DEFINE_KERNEL(NAME, BODY)                                                          \
  __global__ void __launch_bounds__(256) NAME(uint32_t iters, uint32_t* out, unsigned long long* clk) { \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,       \
             a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;                                    \
    const uint32_t b = blockIdx.x | 1, c = blockIdx.x * 7 + 3;                             \
    for (uint32_t i = 0; i < iters; ++i) {                                                 \
      ACC8(BODY) ACC8(BODY) ACC8(BODY) ACC8(BODY)                                          \
    }                                                                                      \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;  \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                             \
      clk[0] = __builtin_amdgcn_s_memtime() - t0;                                          \
      clk[1] = __builtin_amdgcn_s_memrealtime() - r0;                                      \
    }                                                                                      \
  }

#define OP_ADD(x) asm volatile("v_add_u32 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_XOR(x) asm volatile("v_xor_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_ADD3(x) asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_ALIGN(x) asm volatile("v_alignbit_b32 %0, %0, %0, 27" : "+v"(x));
#define OP_BFI(x) asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_BITOP3(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xe8" : "+v"(x) : "v"(b), "v"(c));
#define OP_PERM(x) asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_LSHLADD(x) asm volatile("v_lshl_add_u32 %0, %0, 5, %1" : "+v"(x) : "v"(b));
#define OP_AND(x) asm volatile("v_and_b32 %0, %0, %1" : "+v"(x) : "v"(b));
#define OP_LSHL(x) asm volatile("v_lshlrev_b32 %0, 5, %0" : "+v"(x));
#define OP_BITOP3X(x) asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x96" : "+v"(x) : "v"(b), "v"(c));
#define OP_ANDOR(x) asm volatile("v_and_or_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_OR3(x) asm volatile("v_or3_b32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));
#define OP_FMA(x) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(x) : "v"(b), "v"(c));

DEFINE_KERNEL(k_add, OP_ADD)
DEFINE_KERNEL(k_xor, OP_XOR)
DEFINE_KERNEL(k_add3, OP_ADD3)
DEFINE_KERNEL(k_align, OP_ALIGN)
DEFINE_KERNEL(k_bfi, OP_BFI)
DEFINE_KERNEL(k_bitop3, OP_BITOP3)
DEFINE_KERNEL(k_perm, OP_PERM)
DEFINE_KERNEL(k_lshladd, OP_LSHLADD)
#define OP_MIX_AX(x) OP_ALIGN(x) OP_XOR(x)
#define OP_MIX_A3A(x) OP_ADD3(x) OP_ADD(x)
#define OP_MIX_AB(x) OP_ALIGN(x) OP_BITOP3X(x)
#define HALF8(OP) OP(a0) OP(a1) OP(a2) OP(a3) OP(a4) OP(a5) OP(a6) OP(a7)
// 32 instructions per iteration like the others: 16 slow + 16 fast, interleaved
#define DEFINE_MIX(NAME, PAIR)                                                               \
  __global__ void __launch_bounds__(256) NAME(uint32_t iters, uint32_t* out, unsigned long long* clk) { \
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime(); \
    uint32_t a0 = threadIdx.x, a1 = a0 * 3, a2 = a0 * 5, a3 = a0 * 7, a4 = a0 * 11,         \
             a5 = a0 * 13, a6 = a0 * 17, a7 = a0 * 19;                                      \
    const uint32_t b = blockIdx.x | 1, c = blockIdx.x * 7 + 3;                               \
    for (uint32_t i = 0; i < iters; ++i) {                                                   \
      HALF8(PAIR) HALF8(PAIR)                                                                \
    }                                                                                        \
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 ^ a1 ^ a2 ^ a3 ^ a4 ^ a5 ^ a6 ^ a7;    \
    if (blockIdx.x == 0 && threadIdx.x == 0) {                                               \
      clk[0] = __builtin_amdgcn_s_memtime() - t0;                                            \
      clk[1] = __builtin_amdgcn_s_memrealtime() - r0;                                        \
    }                                                                                        \
  }

DEFINE_KERNEL(k_fma, OP_FMA)
DEFINE_KERNEL(k_and, OP_AND)
DEFINE_KERNEL(k_lshl, OP_LSHL)
DEFINE_KERNEL(k_bitop3x, OP_BITOP3X)
DEFINE_KERNEL(k_andor, OP_ANDOR)
DEFINE_KERNEL(k_or3, OP_OR3)
DEFINE_MIX(k_mix_ax, OP_MIX_AX)
DEFINE_MIX(k_mix_a3a, OP_MIX_A3A)
DEFINE_MIX(k_mix_ab, OP_MIX_AB)

typedef void (*Kern)(uint32_t, uint32_t*, unsigned long long*);

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const uint32_t iters = 65536, ops_per_iter = 32;  // ~5 ms per launch: the clock has ramped
  uint32_t* out = nullptr;
  CK(hipMalloc(&out, (size_t)cus * 4 * 256 * 4));
  unsigned long long* clk = nullptr;
  CK(hipMalloc(&clk, 2 * sizeof(unsigned long long)));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  struct K {
    const char* name;
    Kern k;
  } ks[] = {{"v_fma_f32", k_fma},         {"v_add_u32", k_add},       {"v_xor_b32", k_xor},
            {"v_and_b32", k_and},         {"v_lshlrev_b32", k_lshl},  {"v_add3_u32", k_add3},
            {"v_alignbit_b32", k_align},  {"v_bfi_b32", k_bfi},       {"v_bitop3_b32 (maj)", k_bitop3},
            {"v_bitop3_b32 (xor3)", k_bitop3x}, {"v_and_or_b32", k_andor}, {"v_or3_b32", k_or3},
            {"v_perm_b32", k_perm}, {"v_lshl_add_u32", k_lshladd},
            // mixed streams: is a slow instruction's cost added to a fast one's, or do they overlap?
            {"mix alignbit+xor", k_mix_ax}, {"mix add3+add", k_mix_a3a}, {"mix alignbit+bitop3", k_mix_ab}};
  double fma_ns[5] = {0, 0, 0, 0, 0};
  for (const K& k : ks) {
    for (int wps : {1, 2, 4}) {  // waves per SIMD: 4 * wps waves per CU
      const uint32_t blocks = (uint32_t)cus * wps;  // 256 threads = 4 waves, one per SIMD
      hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, 16, out, clk);
      CK(hipDeviceSynchronize());
      float best = 1e30f;
      for (int r = 0; r < 3; ++r) {
        CK(hipEventRecord(e0, 0));
        hipLaunchKernelGGL(k.k, dim3(blocks), dim3(256), 0, 0, iters, out, clk);
        CK(hipEventRecord(e1, 0));
        CK(hipEventSynchronize(e1));
        float ms = 0;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (ms < best) best = ms;
      }
      unsigned long long hc[2];
      CK(hipMemcpy(hc, clk, sizeof(hc), hipMemcpyDeviceToHost));
      const double ghz = hc[1] ? (double)hc[0] / ((double)hc[1] * 10.0) : 0.0;  // s_memrealtime ticks at 100 MHz
      const double ns_per = best * 1e6 / ((double)iters * ops_per_iter * wps);  // per wave-instruction per SIMD
      if (k.k == k_fma) fma_ns[wps] = ns_per;
      printf("{\"op\": \"%s\", \"waves_per_simd\": %d, \"ms\": %.4f, \"ns_per_wave_inst_per_simd\": %.4f, "
             "\"vs_fma\": %.3f, \"block0_ghz\": %.3f, \"cycles_per_wave_inst_per_simd\": %.3f}\n",
             k.name, wps, best, ns_per, ns_per / fma_ns[wps], ghz, ns_per * ghz);
      fflush(stdout);
    }
  }
  CK(hipFree(out));
  CK(hipFree(clk));
  return 0;
}
