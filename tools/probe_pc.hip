// tools/probe_pc.hip -- diagnostic build of the pc kernel with s_memtime stamps
// (not product code).  Compiles the product sources with LBF_PC_STAMPS and
// prints, per role, the mean cycles per block step spent waiting vs working.
// Build: hipcc --offload-arch=gfx950 -O3 -DLBF_PC_STAMPS -I../include -I../bitflood_amd/csrc \
//          probe_pc.hip -o build/probe_pc -L/opt/rocm/lib -lhsa-runtime64
#include "../bitflood_amd/csrc/lbf_capi.cpp"
#include "../bitflood_amd/csrc/sha1_kernels.hip"
#include "experimental/sha1_superseded.hip"  // variants 4, 6, 13

#include <stdio.h>
#include <vector>

static void run(int variant, uint8_t* buf, uint64_t len, uint32_t cs, uint8_t* dig) {
  const uint64_t n = len / cs;
  lbf_set_kernel_variant(variant);
  float ms = 0;
  lbf_time_uniform(buf, len, cs, 0, n, dig, 1, nullptr, &ms);
  if (lbf_time_uniform(buf, len, cs, 0, n, dig, 3, nullptr, &ms)) {
    printf("error: %s\n", lbf_last_error());
    return;
  }
  const bool px = variant == 10;  // two pairs per workgroup: waves 0,1 consume, 2,3 produce
  const bool x2 = variant == 12;   // pc4x2: waves 2,3 consume; 0,4 are producer 0 and 1,5 producer 1 of each group
  const bool x1 = variant == 13;   // pc4x2's structure, one group: wave 2 consumes, 0 and 1 produce (stamps at wg * 6)
  const int wgs = (int)((n + (px || x2 ? 127 : 63)) / (px || x2 ? 128 : 64));
  const int nw = (variant == 4 || variant == 6 || variant == 7) ? 3 : px ? 4 : x2 || x1 ? 6 : 2;  // waves per workgroup
  std::vector<unsigned long long> h(wgs * nw * 4);
  hipMemcpyFromSymbol(h.data(), HIP_SYMBOL(lbf::g_pc_stamps), wgs * nw * 4 * 8, 0, hipMemcpyDeviceToHost);
  double a[3][3] = {{0}};
  double steps = 0;
  // roles: 0 = consumer(s), 1.. = producer(s); pcx5's two pairs fold into one consumer and one producer
  const int roles = px ? 2 : x2 || x1 ? 3 : nw;
  for (int w = 0; w < wgs; ++w)
    for (int r = 0; r < nw; ++r) {
      if (x1 && r > 2) continue;
      const int role = px ? (r >= 2 ? 1 : 0) : x2 ? (r == 2 || r == 3 ? 0 : r == 0 || r == 4 ? 1 : 2)
                     : x1 ? (r == 2 ? 0 : r + 1) : r;
      for (int j = 0; j < 3; ++j) a[role][j] += (double)h[(w * nw + r) * 4 + j] / (px || x2 ? 2 : 1);
      if (r == 0) steps += (double)h[(w * nw) * 4 + 3];
    }
  steps /= wgs;
  for (int r = 0; r < roles; ++r)
    for (int j = 0; j < 3; ++j) a[r][j] /= wgs * steps;
  printf("variant %d cs=%u n=%lu: %.3f ms (%.1f GiB/s)  steps=%.0f  cycles/step: consumer[wait %.0f work %.0f]",
         variant, cs, (unsigned long)n, ms, len / (ms * 1e-3) / (1 << 30), steps, a[0][0], a[0][1]);
  for (int r = 1; r < roles; ++r)
    printf(" producer%d[vmwait %.0f work %.0f barrier %.0f]", r - 1, a[r][0], a[r][1], a[r][2]);
  printf("\n");
  if (x2) {
    // pc4x2: the two consumers (waves 2 and 3) separately, and how often each
    // is the one the barrier waits for (its wait below the other's)
    double cw[2] = {0, 0};
    long later[2] = {0, 0};
    for (int w = 0; w < wgs; ++w) {
      const double c0 = (double)h[(w * nw + 2) * 4 + 0], c1 = (double)h[(w * nw + 3) * 4 + 0];
      cw[0] += c0;
      cw[1] += c1;
      later[c0 < c1 ? 0 : 1]++;
    }
    printf("  pc4x2 consumers: wave 2 waits %.0f, wave 3 waits %.0f cycles/step; arrives last in %ld / %ld of %d workgroups\n",
           cw[0] / (wgs * steps), cw[1] / (wgs * steps), later[0], later[1], wgs);
  }
}

int main(int argc, char** argv) {
  // default: pcx5 at the C4 shape (32,768 x 1 MiB, 32 GiB) and at 32,768 x 256 KiB, pc4 at C2
  const uint64_t len = 32ull << 30;
  uint8_t *buf, *dig;
  if (hipMalloc(&buf, len) != hipSuccess || hipMalloc(&dig, (len / 65536) * 20) != hipSuccess) {
    printf("hipMalloc failed\n");
    return 1;
  }
  lbf_fill_synthetic(buf, len, 0x5EED, 0, nullptr);
  hipDeviceSynchronize();
  const bool all = argc > 1;
  run(10, buf, len, 1 << 20, dig);
  run(12, buf, len, 1 << 20, dig);
  run(10, buf, 8ull << 30, 262144, dig);
  run(12, buf, 8ull << 30, 262144, dig);
  run(7, buf, 4ull << 30, 262144, dig);
  run(13, buf, 4ull << 30, 262144, dig);
  if (all)
    for (int v : {4, 6}) run(v, buf, 4ull << 30, 262144, dig);
  hipFree(buf);
  hipFree(dig);
  return 0;
}
