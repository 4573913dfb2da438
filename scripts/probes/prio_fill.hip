// prio_fill.hip -- PROBE (not product): can a low-priority wave fill the
// issue slots a lone MD5 chain wave leaves (9.4 % of its cycles,
// SQ_WAIT_INST_ANY) without slowing it?  One 8-wave workgroup
// per CU = two waves per SIMD (96 KiB of LDS reserved).  Waves 0-3 run
// `iters` compressions of one chain per lane at s_setprio `hi`; waves 4-7 run
// compressions at s_setprio 0 until waves 0-3 are done (an LDS flag), and
// count them.  mode 0: the filler waves exit at once (the chain waves alone).
// Built by scripts/probes/prio_fill.py --build.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../sproxy_amd/csrc/md5_core.h"

using namespace md5hip;

__device__ __forceinline__ void step(State& st, uint4 (&w)[4]) {
  compress_regs<true, true>(st, w);
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = make_uint4(w[q].x + st.a, w[q].y + st.b, w[q].z + st.c, w[q].w + st.d);
}

__global__ void __launch_bounds__(512) prio_fill(uint32_t iters, int mode, int hi, uint32_t* __restrict__ fills,
                                                 uint4* __restrict__ out) {
  extern __shared__ uint32_t lds[];
  const uint32_t wave = threadIdx.x >> 6;
  if (threadIdx.x == 0) lds[0] = 0;
  __syncthreads();
  State st = initial_state();
  const uint32_t x = (threadIdx.x * 0x9E3779B9u) ^ (blockIdx.x << 8);
  uint4 w[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) w[q] = make_uint4(x + q, x * 3u + q, x ^ (q << 9), x + 77u * q);
  if (wave < 4) {
    if (hi == 3) __builtin_amdgcn_s_setprio(3);
    else if (hi == 2) __builtin_amdgcn_s_setprio(2);
    else if (hi == 1) __builtin_amdgcn_s_setprio(1);
    for (uint32_t it = 0; it < iters; ++it) step(st, w);
    if ((threadIdx.x & 63) == 0) atomicAdd(&lds[0], 1u);
  } else if (mode) {
    __builtin_amdgcn_s_setprio(0);
    uint32_t n = 0;
    while (__atomic_load_n(&lds[0], __ATOMIC_RELAXED) < 4u) {
      step(st, w);
      ++n;
    }
    if ((threadIdx.x & 63) == 0) fills[blockIdx.x * 4 + (wave - 4)] = n;
  }
  out[(size_t)blockIdx.x * blockDim.x + threadIdx.x] = make_uint4(st.a, st.b, st.c, st.d);
}

extern "C" int prio_fill_run(uint32_t iters, int mode, int hi, uint32_t wgs, uint32_t* fills, uint4* out,
                             void* stream) {
  hipLaunchKernelGGL(prio_fill, dim3(wgs), dim3(512), 96 << 10, (hipStream_t)stream, iters, mode, hi, fills, out);
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
