// window_read.hip -- PROBE (not product): the HBM access pattern of fastcrc
// (blk_make_crc's head and tail windows of F bytes per block,
// blk_io.c:408-424) with no CRC arithmetic: per block, F bytes at its start
// and F bytes at its end are read (16 B per lane, F/16 lanes per window) and
// XOR-folded into one 4-byte word written per block.  Its rate is the
// ceiling the access pattern leaves crc32_fast_pipe.
// Built by scripts/probes/window_read.py --build (hipcc, gfx950).
#include <hip/hip_runtime.h>
#include <stdint.h>

template <int F, bool NT>
__global__ void __launch_bounds__(256) windows(const uint8_t* __restrict__ base, uint64_t n, uint32_t len,
                                               uint64_t stride, uint32_t* __restrict__ out) {
  constexpr int LPW = F / 16;                 // lanes per window
  constexpr int LPB = 2 * LPW;                // lanes per block
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t blk = t / LPB;
  const int k = (int)(t % LPB);
  uint32_t v = 0;
  if (blk < n) {
    const uint8_t* p = base + blk * stride + (k < LPW ? 16u * k : (uint64_t)len - F + 16u * (k - LPW));
    typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
    const u32x4* q = reinterpret_cast<const u32x4*>(p);
    const u32x4 x = NT ? __builtin_nontemporal_load(q) : *q;
    v = x.x ^ x.y ^ x.z ^ x.w;
  }
#pragma unroll
  for (int o = 1; o < LPB; o <<= 1) v ^= __shfl_xor(v, o, 64);
  if (blk < n && k == 0) out[blk] = v;
}

extern "C" int window_read(const void* base, uint64_t n, uint32_t len, uint64_t stride, uint32_t F, int nt,
                           uint32_t* out, void* stream) {
  const uint64_t threads = n * (2 * F / 16);
  const dim3 grid((unsigned)((threads + 255) / 256)), blk(256);
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)base;
  if (F == 128 && nt) hipLaunchKernelGGL((windows<128, true>), grid, blk, 0, s, b, n, len, stride, out);
  else if (F == 128) hipLaunchKernelGGL((windows<128, false>), grid, blk, 0, s, b, n, len, stride, out);
  else if (F == 64 && nt) hipLaunchKernelGGL((windows<64, true>), grid, blk, 0, s, b, n, len, stride, out);
  else if (F == 64) hipLaunchKernelGGL((windows<64, false>), grid, blk, 0, s, b, n, len, stride, out);
  else return -22;
  return hipGetLastError() == hipSuccess ? 0 : -5;
}
