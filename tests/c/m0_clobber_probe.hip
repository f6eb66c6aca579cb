// m0_clobber_probe.hip -- compile-only regression probe for the shipped LDS-DMA
// primitive dma16 (bitflood_amd/csrc/kern_common.hpp).
//
// Two compiler-generated LDS DMAs with the same LDS base (M0 = 0) sit around
// one dma16 that writes M0 itself.  If dma16 did not declare M0 clobbered, the
// compiler would set M0 = 0 once and the third DMA would land at dma16's LDS
// address.  tests/test_isa.py compiles this for gfx950 and checks that M0 is
// set again after the asm.  Never launched.
#include "kern_common.hpp"

__global__ void m0_clobber_probe(const uint4* g, uint32_t lds_addr, uint4* out) {
  extern __shared__ uint4 s[];
  auto* lds = (__attribute__((address_space(3))) void*)s;
  __builtin_amdgcn_global_load_lds((const void*)(g + threadIdx.x), lds, 16, 0, 0);
  lbf::dma16(g + 64 + threadIdx.x, lds_addr);
  __builtin_amdgcn_global_load_lds((const void*)(g + 128 + threadIdx.x), lds, 16, 0, 0);
  __syncthreads();
  out[threadIdx.x] = s[threadIdx.x];
}
