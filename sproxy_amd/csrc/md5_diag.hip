// md5_diag.hip -- DIAGNOSTIC kernels (libmd5hip_diag.so), never used by the
// product.  They split the batched-MD5 kernel's time into its two ceilings:
//
//   kind 0  compute only: the same 64-step compression over message words
//           re-read from LDS each block (as the LDS variants do), no HBM reads
//   kind 1..4  load only: the product's loaders (direct2, direct4, lds64,
//           lds128) with the compression replaced by a 16-word xor fold
//   kind 5  ideal coalesced read: each wave-instruction reads 1 KiB contiguous
//
// C ABI: int md5diag_run(int kind, const void *base, uint64_t n, uint32_t len,
//                        uint64_t stride, void *out, void *stream)
#include <errno.h>

#include "md5_kernels.h"

namespace md5hip {

template __global__ void md5_fixed_direct<2, 1>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void md5_fixed_direct<4, 1>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);

__global__ void __launch_bounds__(256)
diag_lds64_load(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                uint4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  fixed_lds_body<64, 1>(base, n, len, stride, out, lds_dyn);
}

__global__ void __launch_bounds__(256)
diag_lds128_load(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  fixed_lds_body<128, 1>(base, n, len, stride, out, lds_dyn);
}

__global__ void __launch_bounds__(256)
diag_xpose1_load(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<1, 1>(base, n, len, stride, out, img);
}

__global__ void __launch_bounds__(256)
diag_xpose2_load(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<2, 1>(base, n, len, stride, out, img);
}

// Compute only: lane L hashes `nblocks` blocks whose words it re-reads from its
// own 64-B LDS row every block (ds_read_b128 x4, like lds64), then the pad block.
__global__ void __launch_bounds__(256)
diag_compute(uint64_t n, uint32_t nblocks, uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t rows[256 * 64];
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  uint32_t* my = reinterpret_cast<uint32_t*>(rows + threadIdx.x * 64);
#pragma unroll
  for (int k = 0; k < 16; ++k) my[k] = (uint32_t)i * 2654435761u + (uint32_t)k;
  __builtin_amdgcn_wave_barrier();
  State st = initial_state();
  for (uint32_t b = 0; b < nblocks; ++b) {
    uint4 w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      // rotate the slot each block so the reads cannot be hoisted
      const uint32_t q = ((uint32_t)k + b) & 3u;
      w[k] = *reinterpret_cast<const uint4*>(rows + threadIdx.x * 64 + q * 16);
    }
    compress_regs(st, w);
  }
  compress_pad_only(st, nblocks * 512u, 0u);
  if (i < n) out[i] = make_uint4(st.a, st.b, st.c, st.d);
}

// Ideal streaming read of n*len bytes: grid-stride, 16 B per lane, consecutive
// lanes consecutive addresses; xor-fold per lane.
__global__ void __launch_bounds__(256)
diag_stream_read(const uint4* __restrict__ src, uint64_t n16, uint4* __restrict__ out) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  uint4 acc = make_uint4(0, 0, 0, 0);
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n16; j += stride) {
    const uint4 v = ld16(src + j);
    acc.x ^= v.x; acc.y ^= v.y; acc.z ^= v.z; acc.w ^= v.w;
  }
  out[(uint64_t)blockIdx.x * blockDim.x + threadIdx.x] = acc;
}

}  // namespace md5hip

using namespace md5hip;

extern "C" int md5diag_run(int kind, const void* base, uint64_t n, uint32_t len, uint64_t stride,
                           void* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)base;
  uint4* o = (uint4*)out;
  const uint32_t grid = (uint32_t)((n + 255) / 256);
  switch (kind) {
    case 0:
      hipLaunchKernelGGL(diag_compute, dim3(grid), dim3(256), 0, s, n, len >> 6, o);
      break;
    case 1:
      hipLaunchKernelGGL((md5_fixed_direct<2, 1>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 2:
      hipLaunchKernelGGL((md5_fixed_direct<4, 1>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 3: {
      const size_t lds = 4 * 2 * 64 * 64;
      hipLaunchKernelGGL(diag_lds64_load, dim3(grid), dim3(256), lds, s, b, n, len, stride, o);
      break;
    }
    case 4: {
      const size_t lds = 4 * 2 * 64 * 128;
      (void)hipFuncSetAttribute(reinterpret_cast<const void*>(diag_lds128_load),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
      hipLaunchKernelGGL(diag_lds128_load, dim3(grid), dim3(256), lds, s, b, n, len, stride, o);
      break;
    }
    case 5: {
      // `out` must hold 8192*256 uint4
      hipLaunchKernelGGL(diag_stream_read, dim3(8192), dim3(256), 0, s,
                         (const uint4*)b, n * (uint64_t)len / 16, o);
      break;
    }
    case 6:
      hipLaunchKernelGGL(diag_xpose1_load, dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 7:
      hipLaunchKernelGGL(diag_xpose2_load, dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    default:
      return -EINVAL;
  }
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
