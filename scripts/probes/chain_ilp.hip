// chain_ilp.hip -- PROBE (not product): does a LONE wave per SIMD leave
// issue slots a second independent MD5 chain per lane can fill?  BALANCED
// (md5_desc_balanced_t, one wave per SIMD) spends 9.4 % of its wave cycles
// in SQ_WAIT_INST_ANY (issue stall) against 85 % VALU (PMC, round 5, call
// r05d).  Here each lane runs `iters` MD5 compressions of register data
// (md5_core.h compress, the product's step code) on C chains interleaved
// (C = 1, 2, 3), one 4-wave workgroup per CU (96 KiB of LDS reserved, so a
// CU holds one: one wave per SIMD), or W waves per SIMD (W workgroups per
// CU, 40 KiB each).  Time per compression per chain says whether the
// chains overlap.  Built by scripts/probes/chain_ilp.py --build.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../sproxy_amd/csrc/md5_core.h"

using namespace md5hip;

template <int C>
__global__ void __launch_bounds__(256) chains(uint32_t iters, uint32_t seed, uint4* __restrict__ out) {
  extern __shared__ uint8_t hog[];
  State st[C];
  uint4 w[C][4];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    st[c] = initial_state();
    const uint32_t x = seed ^ (threadIdx.x * 0x9E3779B9u) ^ (blockIdx.x << 8) ^ (c * 0x85EBCA6Bu);
#pragma unroll
    for (int q = 0; q < 4; ++q) w[c][q] = make_uint4(x + q, x * 3u + q, x ^ (q << 9), x + 77u * q);
  }
  for (uint32_t it = 0; it < iters; ++it) {
#pragma unroll
    for (int c = 0; c < C; ++c) {
      compress_regs<true, true>(st[c], w[c]);
      // every message word depends on the chain (16 adds per compression,
      // the same for every C): no M + K is hoisted out of the loop
#pragma unroll
      for (int q = 0; q < 4; ++q)
        w[c][q] = make_uint4(w[c][q].x + st[c].a, w[c][q].y + st[c].b, w[c][q].z + st[c].c, w[c][q].w + st[c].d);
    }
  }
  uint4 r = make_uint4(0, 0, 0, 0);
#pragma unroll
  for (int c = 0; c < C; ++c) r.x ^= st[c].a, r.y ^= st[c].b, r.z ^= st[c].c, r.w ^= st[c].d;
  if (hog[threadIdx.x] == 0xFF && r.x == 0x12345678u) r.y ^= 1;   // keep the LDS reservation live
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = r;
}

extern "C" int chain_ilp(int C, uint32_t iters, uint32_t wgs, uint32_t lds, uint4* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const dim3 g(wgs), b(256);
  switch (C) {
    case 1: hipLaunchKernelGGL(chains<1>, g, b, lds, s, iters, 7u, out); break;
    case 2: hipLaunchKernelGGL(chains<2>, g, b, lds, s, iters, 7u, out); break;
    case 3: hipLaunchKernelGGL(chains<3>, g, b, lds, s, iters, 7u, out); break;
    default: return -22;
  }
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
