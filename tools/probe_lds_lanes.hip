// tools/probe_lds_lanes.hip -- diagnostic microbenchmark (not product code).
//
// Does the consumer's schedule read (one ds_read_b128 per 4 rounds) cost less
// issue time when fewer lanes of the wave are active?  One wave per CU runs the
// pc2 consumer loop (compress_expanded_wk over an LDS slot) with L active lanes,
// and, as the floor, the same rounds fed from registers.
// Build: hipcc --offload-arch=gfx950 -O3 -I../bitflood_amd/csrc -I../include probe_lds_lanes.hip -o build/probe_lds_lanes
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdlib.h>

#include "sha1_device.hpp"

using namespace lbf;

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e)); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int kSlotU4 = 20 * 64;

// mode 0: schedule from LDS (pc2 consumer); mode 1: from registers (floor);
// mode 2: from LDS, two ds_read_b64 per 4 rounds; modes 3/4: two-add3 rounds from registers
// with the round constant in an SGPR (3) or a VGPR (4); modes 5/6: the two-add3 round (5) and
// the W+K round (6) from registers with rotl5(a) forced into the last add
template <int kMode>
__global__ void __launch_bounds__(64) consumer(uint32_t nblk, uint32_t lanes, uint32_t* out,
                                               unsigned long long* clk) {
  extern __shared__ __attribute__((aligned(16))) uint4 slot[];
  const int lane = threadIdx.x;
  for (int q = 0; q < 20; ++q) slot[q * 64 + lane] = make_uint4(lane * q, lane + q, lane ^ q, q);
  __syncthreads();
  uint4 r[20];
#pragma unroll
  for (int q = 0; q < 20; ++q) r[q] = slot[q * 64 + lane];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  Digest s;
  s.init();
  if ((uint32_t)lane < lanes) {
    for (uint32_t b = 0; b < nblk; ++b) {
      if (kMode == 0) {
        compress_expanded_wk(s, slot + lane, 64);
      } else if (kMode == 1) {
        uint32_t a = s.h[0], bb = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
        for (int q = 0; q < 20; ++q) {
          round_step_wk(4 * q + 0, a, bb, c, d, e, r[q].x);
          round_step_wk(4 * q + 1, a, bb, c, d, e, r[q].y);
          round_step_wk(4 * q + 2, a, bb, c, d, e, r[q].z);
          round_step_wk(4 * q + 3, a, bb, c, d, e, r[q].w);
        }
        s.h[0] += a; s.h[1] += bb; s.h[2] += c; s.h[3] += d; s.h[4] += e;
      } else if (kMode == 5 || kMode == 6) {
        // the sum associated as written: the late operand rotl5(a) enters the
        // LAST add (an empty asm keeps the compiler from reassociating);
        // 5: t = add3(e, W, K) with K in VGPRs, 6: s = e + (W+K)
        uint32_t kv[4] = {kK1, kK2, kK3, kK4};
#pragma unroll
        for (int j = 0; j < 4; ++j) asm volatile("v_mov_b32 %0, %1" : "=v"(kv[j]) : "s"(kv[j]));
        uint32_t a = s.h[0], bb = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
        for (int q = 0; q < 20; ++q) {
          const uint32_t x4[4] = {r[q].x, r[q].y, r[q].z, r[q].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 4 * q + j;
            const uint32_t f = i < 20 ? f_choose(bb, c, d) : (i >= 40 && i < 60 ? f_major(bb, c, d) : f_parity(bb, c, d));
            uint32_t t = kMode == 5 ? e + x4[j] + kv[i / 20] : e + x4[j];
            asm("" : "+v"(t));
            const uint32_t n = rotl(a, 5) + f + t;
            e = d; d = c; c = rotl(bb, 30); bb = a; a = n;
          }
        }
        s.h[0] += a; s.h[1] += bb; s.h[2] += c; s.h[3] += d; s.h[4] += e;
      } else if (kMode == 3 || kMode == 4) {
        // two-add3 rounds (t = rotl5(a) + f + (e + W + K)) fed from registers,
        // K from an SGPR (3) or from VGPRs (4)
        uint32_t kv[4] = {kK1, kK2, kK3, kK4};
        if (kMode == 4) {
#pragma unroll
          for (int j = 0; j < 4; ++j) asm volatile("v_mov_b32 %0, %1" : "=v"(kv[j]) : "s"(kv[j]));
        }
        uint32_t a = s.h[0], bb = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
        for (int q = 0; q < 20; ++q) {
          const uint32_t x4[4] = {r[q].x, r[q].y, r[q].z, r[q].w};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int i = 4 * q + j;
            const uint32_t f = i < 20 ? f_choose(bb, c, d) : (i >= 40 && i < 60 ? f_major(bb, c, d) : f_parity(bb, c, d));
            const uint32_t t = rotl(a, 5) + f + (e + x4[j] + kv[i / 20]);
            e = d; d = c; c = rotl(bb, 30); bb = a; a = t;
          }
        }
        s.h[0] += a; s.h[1] += bb; s.h[2] += c; s.h[3] += d; s.h[4] += e;
      } else {
        const uint2* w2 = reinterpret_cast<const uint2*>(slot);
        uint32_t a = s.h[0], bb = s.h[1], c = s.h[2], d = s.h[3], e = s.h[4];
#pragma unroll
        for (int q = 0; q < 40; ++q) {
          const uint2 v = w2[q * 64 + lane];
          round_step_wk(2 * q + 0, a, bb, c, d, e, v.x);
          round_step_wk(2 * q + 1, a, bb, c, d, e, v.y);
        }
        s.h[0] += a; s.h[1] += bb; s.h[2] += c; s.h[3] += d; s.h[4] += e;
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * 64 + lane] = s.h[0] ^ s.h[1] ^ s.h[2] ^ s.h[3] ^ s.h[4];
  if (lane == 0) clk[blockIdx.x] = t1 - t0;
}

template <int kMode>
static void run(const char* name, uint32_t nblk, uint32_t lanes, uint32_t* out, unsigned long long* clk) {
  const int wgs = 256;
  const size_t lds = 100 * 1024;  // one workgroup per CU
  CK(hipFuncSetAttribute((const void*)consumer<kMode>, hipFuncAttributeMaxDynamicSharedMemorySize, lds));
  hipLaunchKernelGGL(consumer<kMode>, dim3(wgs), dim3(64), lds, 0, nblk, lanes, out, clk);
  CK(hipDeviceSynchronize());
  hipLaunchKernelGGL(consumer<kMode>, dim3(wgs), dim3(64), lds, 0, nblk, lanes, out, clk);
  CK(hipDeviceSynchronize());
  unsigned long long h[256];
  CK(hipMemcpy(h, clk, sizeof(h), hipMemcpyDeviceToHost));
  double cyc = 0;
  for (int b = 0; b < wgs; ++b) cyc += (double)h[b];
  cyc /= wgs;
  printf("%-10s lanes=%2u  cycles/block=%7.1f  cycles/round=%5.2f\n", name, lanes, cyc / nblk, cyc / nblk / 80.0);
}

int main(int argc, char** argv) {
  const uint32_t nblk = argc > 1 ? atoi(argv[1]) : 2048;
  uint32_t* out;
  unsigned long long* clk;
  CK(hipMalloc(&out, 256 * 64 * 4));
  CK(hipMalloc(&clk, 256 * 8));
  for (uint32_t lanes : {64u, 32u}) {
    run<0>("lds_b128", nblk, lanes, out, clk);
    run<2>("lds_b64", nblk, lanes, out, clk);
    run<1>("regs", nblk, lanes, out, clk);
    run<3>("2add3_sK", nblk, lanes, out, clk);
    run<4>("2add3_vK", nblk, lanes, out, clk);
    run<5>("2add3_vK_late", nblk, lanes, out, clk);
    run<6>("wk_late", nblk, lanes, out, clk);
  }
  return 0;
}
