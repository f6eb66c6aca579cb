// tools/probe_placement.hip -- diagnostic (not product code): where and when
// the waves of a compute-bound chunk-hash launch run.  Each wave records its
// start/end (s_memrealtime, 100 MHz) and HW_ID (SIMD/CU/SE) + XCC_ID; the host
// reports waves per SIMD and the launch timeline.
#include <hip/hip_runtime.h>
#include <stdio.h>

#include <algorithm>
#include <map>
#include <vector>

#include "sha1_device.hpp"

using namespace lbf;

struct WaveRec {
  unsigned long long t0, t1;
  uint32_t hw_id, xcc;
};

template <int kRotate>
__device__ __forceinline__ void rotate_prio(uint32_t b, uint32_t slot) {
  if (kRotate == 0) return;
  // every kRotate blocks the top priority moves to the next of 4 waves
  const uint32_t p = __builtin_amdgcn_readfirstlane(((b / kRotate) + slot) & 3);
  if (p == 0) __builtin_amdgcn_s_setprio(3);
  else if (p == 1) __builtin_amdgcn_s_setprio(2);
  else if (p == 2) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}

template <int kRotate>
__global__ void __launch_bounds__(256) compute_only(uint32_t nblk, uint32_t* out, WaveRec* rec) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
  Digest s;
  s.init();
  uint32_t w[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) w[k] = i * 0x9E3779B9u + k;
  uint32_t hwid;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hwid));
  const uint32_t slot = hwid & 3;  // wave slot within its SIMD
  for (uint32_t b = 0; b < nblk; ++b) {
    if (kRotate && (b % kRotate) == 0) rotate_prio<kRotate>(b, slot);
    uint32_t x[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) x[k] = w[k] ^ s.h[k % 5];
    compress(s, x);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
  out[i] = s.h[0] ^ s.h[1] ^ s.h[2] ^ s.h[3] ^ s.h[4];
  if ((threadIdx.x & 63) == 0) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    WaveRec r{t0, t1, hw, xcc};
    rec[i / 64] = r;
  }
}

template <int kRotate>
static int run(uint32_t chains, uint32_t tpb) {
  const uint32_t nblk = 1024;
  const uint32_t waves = chains / 64;
  uint32_t* out;
  WaveRec* rec;
  hipMalloc(&out, chains * 4);
  hipMalloc(&rec, waves * sizeof(WaveRec));
  hipLaunchKernelGGL(compute_only<kRotate>, dim3(chains / tpb), dim3(tpb), 0, 0, nblk, out, rec);
  hipDeviceSynchronize();
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(compute_only<kRotate>, dim3(chains / tpb), dim3(tpb), 0, 0, nblk, out, rec);
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms;
  hipEventElapsedTime(&ms, e0, e1);
  std::vector<WaveRec> h(waves);
  hipMemcpy(h.data(), rec, waves * sizeof(WaveRec), hipMemcpyDeviceToHost);
  unsigned long long t_min = ~0ull, t_max = 0;
  for (auto& r : h) {
    t_min = std::min(t_min, r.t0);
    t_max = std::max(t_max, r.t1);
  }
  // HW_ID (gfx9): wave_id[3:0] simd_id[5:4] pipe_id[7:6] cu_id[11:8] sh_id[12] se_id[15:13]
  std::map<uint64_t, std::vector<const WaveRec*>> per_simd;
  std::map<uint64_t, int> per_cu;
  for (auto& r : h) {
    const uint32_t simd = (r.hw_id >> 4) & 3, cu = (r.hw_id >> 8) & 15, sh = (r.hw_id >> 12) & 1,
                   se = (r.hw_id >> 13) & 7;
    const uint64_t cu_key = ((uint64_t)r.xcc << 16) | (se << 8) | (sh << 4) | cu;
    per_simd[(cu_key << 2) | simd].push_back(&r);
    per_cu[cu_key]++;
  }
  std::map<int, int> hist_simd, hist_cu;
  for (auto& kv : per_simd) hist_simd[(int)kv.second.size()]++;
  for (auto& kv : per_cu) hist_cu[kv.second]++;
  double dur_sum = 0;
  for (auto& r : h) dur_sum += (double)(r.t1 - r.t0);
  printf("rotate=%d chains=%u tpb=%u nblk=%u: kernel %.3f ms, span %.3f ms, mean wave %.3f ms, SIMDs used %zu, CUs used %zu\n",
         kRotate, chains, tpb, nblk, ms, (t_max - t_min) / 1e5, dur_sum / h.size() / 1e5, per_simd.size(), per_cu.size());
  printf("  waves per SIMD histogram:");
  for (auto& kv : hist_simd) printf(" %d:%d", kv.first, kv.second);
  printf("\n  waves per CU histogram:");
  for (auto& kv : hist_cu) printf(" %d:%d", kv.first, kv.second);
  // start-time spread: fraction of waves that started > 10% of the span after the first
  int late = 0;
  for (auto& r : h)
    if (r.t0 - t_min > (t_max - t_min) / 10) ++late;
  printf("\n  waves starting after 10%% of the span: %d of %u\n", late, waves);
  int shown = 0;
  for (auto& kv : per_simd) {
    if (shown++ >= 3) break;
    printf("  simd %llx:", (unsigned long long)kv.first);
    for (const WaveRec* r : kv.second)
      printf(" [slot %u %.2f-%.2f]", r->hw_id & 15, (r->t0 - t_min) / 1e5, (r->t1 - t_min) / 1e5);
    printf("\n");
  }
  hipFree(out);
  hipFree(rec);
  return 0;
}

int main(int argc, char** argv) {
  const uint32_t chains = argc > 1 ? atoi(argv[1]) : 262144;
  const uint32_t tpb = argc > 2 ? atoi(argv[2]) : 256;
  const int which = argc > 3 ? atoi(argv[3]) : -1;
  if (which < 0 || which == 0) run<0>(chains, tpb);
  if (which < 0 || which == 8) run<8>(chains, tpb);
  if (which < 0 || which == 32) run<32>(chains, tpb);
  if (which < 0 || which == 128) run<128>(chains, tpb);
  return 0;
}
