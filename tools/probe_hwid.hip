// tools/probe_hwid.hip -- diagnostic (not product code): which SIMD does each
// wave of a workgroup land on?  Reads HW_ID (hwreg 4) in every wave of
// 256 workgroups of W waves with L KiB of LDS and prints the SIMD pattern.
// Build: hipcc --offload-arch=gfx950 -O3 probe_hwid.hip -o build/probe_hwid
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include <map>
#include <string>

__global__ void hwid_kernel(unsigned* out, unsigned spin) {
  extern __shared__ unsigned lds[];
  unsigned id;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
  // keep every wave resident for a while so that the workgroups coexist
  unsigned x = threadIdx.x;
  for (unsigned i = 0; i < spin; ++i) x = x * 1664525u + 1013904223u;
  if ((threadIdx.x & 63) == 0) {
    out[blockIdx.x * 16 + (threadIdx.x >> 6)] = id;
    lds[threadIdx.x >> 6] = x;
  }
}

int main() {
  unsigned* d;
  hipMalloc(&d, 1024 * 16 * 4);
  for (int waves : {2, 3, 4}) {
    for (int lds_kib : {60, 96, 144}) {
      hipFuncSetAttribute((const void*)hwid_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, lds_kib * 1024);
      hipMemset(d, 0xff, 1024 * 16 * 4);
      hipLaunchKernelGGL(hwid_kernel, dim3(256), dim3(64 * waves), lds_kib * 1024, 0, d, 200000u);
      hipDeviceSynchronize();
      unsigned h[256 * 16];
      hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
      std::map<std::string, int> pat;
      std::map<unsigned, int> cu_use;
      for (int b = 0; b < 256; ++b) {
        std::string s;
        for (int w = 0; w < waves; ++w) {
          const unsigned id = h[b * 16 + w];
          const unsigned simd = (id >> 4) & 3, cu = (id >> 8) & 15, sh = (id >> 12) & 1, se = (id >> 13) & 7;
          s += std::to_string(simd);
          if (w == 0) cu_use[(se << 8) | (sh << 4) | cu]++;
        }
        pat[s]++;
      }
      printf("waves=%d lds=%dKiB: distinct CUs %zu; SIMD patterns:", waves, lds_kib, cu_use.size());
      for (auto& kv : pat) printf(" %s x%d", kv.first.c_str(), kv.second);
      printf("\n");
    }
  }
  return 0;
}
