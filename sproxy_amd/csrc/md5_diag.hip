// md5_diag.hip -- DIAGNOSTIC kernels (libmd5hip_diag.so), never used by the
// product.  They split the batched-MD5 kernel's time into its two ceilings:
//
//   kind 0  compute only: the same 64-step compression over message words
//           re-read from LDS each block (as the LDS variants do), no HBM reads
//   kind 1..4  load only: the product's loaders (direct2, direct4, lds64,
//           lds128) with the compression replaced by a 16-word xor fold
//   kind 5  ideal coalesced read: each wave-instruction reads 1 KiB contiguous
//   kind 6,7  load only for the xpose1 / xpose2 loaders
//   kind 12   compute only with the latency-form step (md5_core.h kLat)
//   kind 13,14 single-chain latency: few lanes, long chunks (kLat off / on)
//   kind 20-26 xpose1 with buffer-load aux 0, 1, 2, 3, 16, 18, 19 (cache policy A/B)
//   kind 8,9  load only, direct2 / direct4 with paired (whole-line) ring refill
//   kind 10,11 MD5 direct2 / direct4 with paired refill
//   kind 27   CRC-32 lane32 with the unpaired ring (out = u32 per chunk)
//   kind 34-37 product xpose1nt at 20 / 16 / 12 / 8 waves per CU (LDS-capped)
//   kind 38,39 64-B stages through VGPRs at 8 waves/SIMD (nt / default policy)
//   kind 44,45 64-B stages by LDS-DMA, single 4 KiB image (nt / default)
//   kind 40-43 compute only at 32 / 24 / 20 / 16 waves per CU
//   kind 46,47 xpose2 with paired 256-B refill (nt / default)
//   kind 48,49 xpose1nt / compute only with per-wave clock stamps after the digests
//   kind 50   load only (xpose1nt loader, xor fold) with clock stamps
//   kind 51   CRC-32 product body (crc32_fixed_xpose) with clock stamps
//   kind 52,53 xpose1nt on a persistent grid with a work counter (5 / 4 WGs per CU)
//   kind 54   xpose1nt without the peeled last stage (clamped re-read)
//   kind 55,56 xpose1nt / compute only with the PLAIN round-3 form (kX3 off; A/B)
//   kind 57,58 xpose image filled by LDS-DMA, one image per wave (nt / default)
//   kind 28-33 serial-chain latency with 64/32/16/1 active lanes (28-31), and
//             64/32 with the latency-form step (32,33); n = waves, len = bytes
//   kind 100+K VALU issue-rate probes (instruction K of diag_valu_rate)
//
// C ABI: int md5diag_run(int kind, const void *base, uint64_t n, uint32_t len,
//                        uint64_t stride, void *out, void *stream)
#include <errno.h>

#include "md5_kernels.h"
#include "md5_kernels_ab.h"

namespace md5hip {

// ---- experimental loaders (measured, not shipped: DESIGN.md §4) ----

// ---------------------------------------------------------------------------
// Fixed-length, 64-B stages at full occupancy ("x64").
// The MD5 stream issues fastest with 8 waves per SIMD (the VALU issue rate of
// the step's instructions rises from 4 to 8 waves per SIMD), which needs
// <= 64 VGPRs and <= 5 KiB of LDS per wave.  A stage is one 64-B block for the
// wave's 64 chunks (4 KiB): 4 buffer_load_dwordx4 wave-instructions of
// 16 chunks x 64 B (4 lanes per run), a 4 KiB per-wave LDS image, one stage of
// register prefetch.  kDma: the stage goes HBM -> LDS by LDS-DMA
// (global_load_lds_dwordx4) instead of through VGPRs; the single image is
// re-filled only after this lane's ds_reads have returned.
// Same source swizzle as fixed_lds_body<64>: row L's 16-B slot q holds part
// q ^ ((L >> 2) & 3), so every ds_read_b128 lane group is conflict-free.
// Requires 64 * stride < 2^31 (checked by the launcher).
// ---------------------------------------------------------------------------
template <int CP, bool kDma = false, class H = Md5Hasher<false>>
__device__ __forceinline__ void fixed_x64_body(const uint8_t* __restrict__ base, uint64_t n,
                                               uint32_t len, uint64_t stride,
                                               typename H::Out* __restrict__ out, uint8_t* lds) {
  H h;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + (size_t)wave * 4096;
  const uint64_t wave_first = ((uint64_t)blockIdx.x * blockDim.x) + wave * 64u;
  if (wave_first >= n) return;
  const uint64_t left = n - wave_first;
  const uint32_t rows = left < 64 ? (uint32_t)left : 64u;
  const uint8_t* wbase = base + wave_first * stride;
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(wbase);
  uint32_t voff[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const uint32_t row = (uint32_t)r * 16u + (lane >> 2);
    const uint32_t rc = row < rows ? row : rows - 1u;          // ragged last wave
    const uint32_t part = (lane & 3u) ^ ((row >> 2) & 3u);       // source swizzle
    voff[r] = rc * (uint32_t)stride + part * 16u;
  }
  const uint32_t g = (lane >> 2) & 3u;
  const uint32_t nfull = len >> 6;
  typename H::State st = h.init();

  auto read_row = [&](uint4 (&w)[4]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(img + lane * 64 + ((q ^ g) * 16));
      w[q] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };

  if (nfull) {
    const uint32_t lastb = nfull - 1;
    if constexpr (kDma) {
      // buffer_load_dwordx4 ... lds: per-lane voffset fixed, the stage offset
      // in soffset, so the refill spends no VALU on addresses
      auto issue = [&](uint32_t blk) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, img + r * 1024, 16, voff[r], blk * 64u, 0, CP);
      };
      issue(0);
      for (uint32_t blk = 0; blk < nfull; ++blk) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        uint4 w[4];
        read_row(w);
        // the DMA below overwrites the image: this wave's reads must be done
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (blk < lastb) issue(blk + 1);
        h.block(st, w);
      }
    } else {
      auto load_stage = [&](u32x4 (&R)[4], uint32_t blk) __attribute__((always_inline)) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          R[r] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)voff[r], (int)(blk * 64u), CP);
      };
      u32x4 R[4];
      load_stage(R, 0);
      for (uint32_t blk = 0; blk < nfull; ++blk) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<u32x4*>(img + r * 1024 + lane * 16) = R[r];
        __builtin_amdgcn_wave_barrier();
        uint4 w[4];
        read_row(w);
        __builtin_amdgcn_wave_barrier();
        load_stage(R, min(blk + 1, lastb));
        __builtin_amdgcn_sched_barrier(0);
        h.block(st, w);
      }
    }
  }
  const uint64_t i = wave_first + lane;
  const uint64_t ci = lane < rows ? i : n - 1;
  const uint8_t* chunk = base + ci * stride;
  h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
  if (lane < rows) h.store(out, i, st);
}

// Dynamic variant: a persistent grid whose waves take 64-chunk groups from a
// global counter (zeroed by the launcher), so XCDs that run faster under the
// power cap take more groups instead of idling at the end.
template <int D, class H = Md5Hasher<false>, int CP = 0>
__device__ __forceinline__ void fixed_xpose_dyn_body(const uint8_t* __restrict__ base, uint64_t n,
                                                     uint32_t len, uint64_t stride,
                                                     typename H::Out* __restrict__ out,
                                                     uint8_t* lds, uint32_t* counter) {
  H h;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + (size_t)wave * 8192;
  const uint64_t ngroups = (n + 63) / 64;
  for (;;) {
    uint32_t g = 0;
    if ((threadIdx.x & 63u) == 0) g = atomicAdd(counter, 1u);
    g = __builtin_amdgcn_readfirstlane(g);
    if (g >= ngroups) break;
    fixed_xpose_group<D, H, CP>(h, base, n, len, stride, out, img, (uint64_t)g * 64u);
  }
}


template __global__ void md5_fixed_direct<2, FoldHasher>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void md5_fixed_direct<4, FoldHasher>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void md5_fixed_direct<2, FoldHasher, true>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void md5_fixed_direct<4, FoldHasher, true>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void md5_fixed_direct<2, Md5Hasher<false>, true>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void md5_fixed_direct<4, Md5Hasher<false>, true>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void md5_desc<false, true, true, 8, true>(const uint8_t*, const uint64_t*, const uint32_t*,
                                                              const uint32_t*, uint64_t, uint64_t, uint32_t, uint4*);
template __global__ void md5_desc<false, true, true, 8, false, true>(const uint8_t*, const uint64_t*, const uint32_t*,
                                                                     const uint32_t*, uint64_t, uint64_t, uint32_t, uint4*);

// CRC-32 lane-private tables with the unpaired ring (A/B of the paired default)
__global__ void __launch_bounds__(1024)
diag_crc_lane32_unpaired(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                         uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t tabs[Crc32LaneHasher<32>::kLdsBytes];
  crc32_fixed_lane_body<32, 4, false>(base, n, len, stride, out, tabs);
}
#define DESC_INST(L, P, D)                                                                  \
  template __global__ void md5_desc<false, L, P, D>(const uint8_t*, const uint64_t*,       \
                                                    const uint32_t*, const uint32_t*, uint64_t, \
                                                    uint64_t, uint32_t, uint4*);
DESC_INST(false, false, 2) DESC_INST(true, true, 2) DESC_INST(true, true, 4)
DESC_INST(true, true, 8) DESC_INST(true, false, 8) DESC_INST(true, true, 12)
#undef DESC_INST

__global__ void __launch_bounds__(256)
diag_lds64_load(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                uint4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  fixed_lds_body<64, FoldHasher>(base, n, len, stride, out, lds_dyn);
}

__global__ void __launch_bounds__(256)
diag_lds128_load(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  fixed_lds_body<128, FoldHasher>(base, n, len, stride, out, lds_dyn);
}

__global__ void __launch_bounds__(256)
diag_xpose1_load(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<1, FoldHasher>(base, n, len, stride, out, img);
}

__global__ void __launch_bounds__(256)
diag_xpose2_load(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<2, FoldHasher>(base, n, len, stride, out, img);
}

// Cache-policy A/B for the product loader (xpose1): aux bits of the buffer
// loads (gfx950 CPol: sc0 = 1, nt = 2, sc1 = 16).
template <int CP>
__global__ void __launch_bounds__(256)
diag_xpose1_cp(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
               uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<1, Md5Hasher<false>, CP>(base, n, len, stride, out, img);
}

// Compute only: lane L hashes `nblocks` blocks whose words it re-reads from its
// own 64-B LDS row every block (ds_read_b128 x4, like lds64), then the pad block.
template <bool kLat>
__device__ __forceinline__ void diag_compute_body(uint64_t n, uint32_t nblocks, uint4* __restrict__ out) {
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
    compress_regs<kLat>(st, w);
  }
  compress_pad_only(st, nblocks * 512u, 0u);
  if (i < n) out[i] = make_uint4(st.a, st.b, st.c, st.d);
}

template <bool kLat>
__global__ void __launch_bounds__(256)
diag_compute(uint64_t n, uint32_t nblocks, uint4* __restrict__ out) {
  diag_compute_body<kLat>(n, nblocks, out);
}

__global__ void __launch_bounds__(256)
diag_compute_clk(uint64_t n, uint32_t nblocks, uint4* __restrict__ out) {
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  diag_compute_body<false>(n, nblocks, out);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    uint64_t* clk = reinterpret_cast<uint64_t*>(out + n);
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    clk[2 * w] = t1 - t0;
    clk[2 * w + 1] = r1 - r0;
  }
}

// Serial-chain latency with ACT active lanes per wave (the others exit at
// once): does a partly-masked wave64 finish a dependent MD5 chain sooner?
// Message words live in registers (xor with the block index, off the chain).
template <int ACT, bool kLat>
__global__ void __launch_bounds__(64)
diag_chain(uint32_t nblocks, uint4* __restrict__ out) {
  if ((threadIdx.x & 63u) >= (uint32_t)ACT) return;
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  uint4 w0[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    w0[k] = make_uint4(i * 2654435761u + 4 * k, i * 40503u + 4 * k + 1, i ^ (0x9E37u * k), i + 77u * k);
  State st = initial_state();
  for (uint32_t b = 0; b < nblocks; ++b) {
    uint4 w[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = make_uint4(w0[k].x ^ b, w0[k].y ^ b, w0[k].z ^ b, w0[k].w ^ b);
    compress_regs<kLat>(st, w);
  }
  out[i] = make_uint4(st.a, st.b, st.c, st.d);
}

// The same chain with pre-summed addends (md5_core.h compress_fed): 4 VALU
// per step, the 64 addends of a block read from LDS (16 ds_read_b128 per
// block from one of four 16 KiB tables).  kind 80.
__global__ void __launch_bounds__(64)
diag_chain_fed(uint32_t nblocks, uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint4 tab[4][16][64];
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t i = blockIdx.x * 64u + lane;
  for (int b = 0; b < 4; ++b)
    for (int t = 0; t < 16; ++t)
      tab[b][t][lane] = make_uint4(i * 2654435761u + 4 * t + b, i * 40503u + t, i ^ (0x9E37u * t), i + 77u * t);
  __syncthreads();
  State st = initial_state();
  for (uint32_t b = 0; b < nblocks; ++b) {
    uint4 q[16];
#pragma unroll
    for (int t = 0; t < 16; ++t) q[t] = tab[b & 3][t][lane];
    compress_fed(st, q);
  }
  out[i] = make_uint4(st.a, st.b, st.c, st.d);
}

// Lone-chain step mixes (round 3, kinds 84-87).  The product step is
// v_add / v_bitop3 / v_add3 / v_alignbit / v_add; v_add3 and v_alignbit cost
// ~4.4 cycles per wave-instruction at full occupancy, v_add / v_bitop3 ~3.
// Here every addition is a separate v_add_u32_e32 (pinned, so hipcc cannot form
// v_add3; an asm volatile add would make hipcc pad with s_nop): kind 84 = 6 VALU per step (w+M, +K, f, +f, rotate, +x), kind 85
// the fed step as 5 (w+W, f, +f, rotate, +x), against kinds 32 / 80.
__device__ __forceinline__ uint32_t vadd(uint32_t a, uint32_t b) {
  uint32_t r = a + b;
  asm("" : "+v"(r));      // an empty pin (as md5_core.h kLat): no v_add3, no s_nop
  return r;
}
__device__ __forceinline__ uint32_t vaddk(uint32_t a, uint32_t k) { return vadd(a, k); }
template <bool kFed>
__device__ __forceinline__ void compress_adds(State& st, const uint32_t (&m)[16]) {
  uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
  // kFed: W[j] stands in for M[g(j)] + K[j]; otherwise M and K are added apart
  auto W = [&](int j) __attribute__((always_inline)) -> uint32_t { return m[md5_msg_idx(j)]; };
  auto step = [&](uint32_t& w, uint32_t x, uint32_t y, uint32_t z, int j, int s, int fn)
      __attribute__((always_inline)) {
    uint32_t t = vadd(w, W(j));
    if constexpr (!kFed) t = vaddk(t, kMd5K[j]);
    const uint32_t f = fn == 1 ? f1(x, y, z) : fn == 2 ? f2(x, y, z) : fn == 3 ? f3(x, y, z) : f4(x, y, z);
    t = vadd(t, f);
    w = x + rotl(t, s);     // not pinned: a pin before v_bitop3 costs an s_nop
  };
  constexpr int S[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};
#pragma unroll
  for (int j = 0; j < 64; j += 4) {
    const int r = j >> 4;
    step(a, b, c, d, j, S[r][0], r + 1);
    step(d, a, b, c, j + 1, S[r][1], r + 1);
    step(c, d, a, b, j + 2, S[r][2], r + 1);
    step(b, c, d, a, j + 3, S[r][3], r + 1);
  }
  st.a += a;
  st.b += b;
  st.c += c;
  st.d += d;
}
template <bool kFed>
__global__ void __launch_bounds__(64)
diag_chain_adds(uint32_t nblocks, uint4* __restrict__ out) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  uint32_t m0[16];
#pragma unroll
  for (int k = 0; k < 16; ++k) m0[k] = i * 2654435761u + 40503u * k;
  State st = initial_state();
  for (uint32_t b = 0; b < nblocks; ++b) {
    uint32_t m[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) m[k] = m0[k] ^ b;     // off the chain, as diag_chain
    compress_adds<kFed>(st, m);
  }
  out[i] = make_uint4(st.a, st.b, st.c, st.d);
}

// Two independent chains per lane in one instruction stream (kind 81): does
// a lone wave issue faster when it has a second chain to interleave?  Same
// message words as diag_chain (xor with the block index), kLat step.
__global__ void __launch_bounds__(64)
diag_chain2(uint32_t nblocks, uint4* __restrict__ out) {
  const uint32_t i = blockIdx.x * 64u + threadIdx.x;
  uint4 w0[4], w1[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    w0[k] = make_uint4(i * 2654435761u + 4 * k, i * 40503u + 4 * k + 1, i ^ (0x9E37u * k), i + 77u * k);
    w1[k] = make_uint4(i * 97u + 4 * k, i * 1013u + 3 * k + 1, i ^ (0x51EDu * k), i + 31u * k);
  }
  State s0 = initial_state(), s1 = initial_state();
  s1.a ^= i;
  for (uint32_t b = 0; b < nblocks; ++b) {
    uint4 x[4], y[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      x[k] = make_uint4(w0[k].x ^ b, w0[k].y ^ b, w0[k].z ^ b, w0[k].w ^ b);
      y[k] = make_uint4(w1[k].x ^ b, w1[k].y ^ b, w1[k].z ^ b, w1[k].w ^ b);
    }
    compress_regs<true>(s0, x);
    compress_regs<true>(s1, y);
  }
  out[i] = make_uint4(s0.a ^ s1.a, s0.b ^ s1.b, s0.c ^ s1.c, s0.d ^ s1.d);
}

// 64-B-stage candidates at 8 waves per SIMD (fixed_x64_body above).
template <int CP, bool kDma>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8)))
diag_x64(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
         uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 4096];
  fixed_x64_body<CP, kDma>(base, n, len, stride, out, img);
}

// xpose2 with paired (256-B per chunk) refill.
template <int CP>
__global__ void __launch_bounds__(256)
diag_xpose2_pair(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<2, Md5Hasher<false>, CP, true>(base, n, len, stride, out, img);
}

// In-kernel clock (MI355X_MICROARCH 'DVFS give-back' item 6): per wave,
// (s_memtime delta, s_memrealtime delta) around the product body (kind 48) or
// the compute-only body (kind 49), written after the n digests.
template <class H>
__global__ void __launch_bounds__(256)
diag_xpose1nt_clk(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                  uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  fixed_xpose_body<1, H, 2>(base, n, len, stride, out, img);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    uint64_t* clk = reinterpret_cast<uint64_t*>(out + n);
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    clk[2 * w] = t1 - t0;
    clk[2 * w + 1] = r1 - r0;
  }
}

// The product C2 kernel (md5_fixed_xdma1nt: same body, same occupancy) with
// per-wave (s_memtime delta, s_memrealtime delta, s_memrealtime at start, at
// end) written after the n digests -- the per-launch shader clock of the
// bench's first launches (scripts/startup_probe.py).
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
diag_xdma1nt_clk(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  fixed_xdma_body<Md5Hasher<false>, 2>(base, n, len, stride, out, img);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    uint64_t* clk = reinterpret_cast<uint64_t*>(out + n);
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    clk[4 * w] = t1 - t0;
    clk[4 * w + 1] = r1 - r0;
    clk[4 * w + 2] = r0;
    clk[4 * w + 3] = r1;
  }
}

// DRAM-locality probes of the product C2 body (md5_fixed_xdma1nt's loader and
// hash, same occupancy): which chunks a wave takes.  S = lane stride inside a
// block of 64*S consecutive chunks (S waves share it, wave k taking chunks
// k, k+S, ...), so one DMA instruction's 8 rows lie S*16 KiB apart instead of
// 16 KiB; kPerm: the wave -> group assignment permuted (odd multiplier mod the
// wave count, a power of two), so concurrently running waves read far-apart
// regions instead of neighbouring ones.  Digests land at their chunk's index
// (bit-exact with the product); per-wave clock stamps after the digests.
template <int S, bool kPerm>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
diag_xdma_map(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
              uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img_all[4 * 8192];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t nwaves = n / 64;                       // n: a multiple of 64 * S (host checks)
  uint64_t w = (uint64_t)blockIdx.x * 4u + wave;
  if (w < nwaves) {
    if (kPerm) w = (w * 0x9E3779B1ull) & (nwaves - 1);  // nwaves: a power of two
    const uint64_t blk = w / S, k = w % S;
    const uint64_t wave_first = blk * 64u * S + k;      // lane l: chunk wave_first + l*S
    uint8_t* img = img_all + wave * 8192u;
    const uint32_t lane = threadIdx.x & 63u;
    const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(base + wave_first * stride);
    uint32_t voff[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const uint32_t row = (uint32_t)r * 8u + (lane >> 3);
      const uint32_t part = (lane & 7u) ^ ((row >> 1) & 7u);
      voff[r] = row * (uint32_t)S * (uint32_t)stride + part * 16u;
    }
    const uint32_t g = (lane >> 1) & 7u;
    const uint32_t nfull = len >> 6, nstage = nfull >> 1;
    Md5Hasher<false> h;
    auto st = h.init();
    auto issue = [&](uint32_t stg) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, img + r * 1024, 16, voff[r], stg * 128u, 0, 2);
    };
    issue(0);
    for (uint32_t stg = 0; stg < nstage; ++stg) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint4 wv[2][4];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(img + lane * 128 + ((q ^ g) * 16));
        wv[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (stg + 1 < nstage) issue(stg + 1);
      __builtin_amdgcn_sched_barrier(0);
      h.block(st, wv[0]);
      h.block(st, wv[1]);
    }
    const uint64_t ci = wave_first + (uint64_t)lane * S;
    const uint8_t* chunk = base + ci * stride;
    if (nfull & 1u) {
      uint4 wb[4];
      load_block(wb, reinterpret_cast<const uint4*>(chunk + ((uint64_t)(nfull - 1) << 6)));
      h.block(st, wb);
    }
    h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
    h.store(out, ci, st);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    uint64_t* clk = reinterpret_cast<uint64_t*>(out + n);
    const uint64_t wi = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    clk[2 * wi] = t1 - t0;
    clk[2 * wi + 1] = r1 - r0;
  }
}

// CRC-32 product body (crc32_fixed_xpose) with clock stamps after n*16 bytes.
__global__ void __launch_bounds__(256)
diag_crc_clk(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
             uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  __shared__ __attribute__((aligned(16))) uint8_t tabs[Crc32Hasher::kLdsBytes];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  fixed_xpose_body<1, Crc32Hasher, 2>(base, n, len, stride, reinterpret_cast<uint32_t*>(out), img, tabs);
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    uint64_t* clk = reinterpret_cast<uint64_t*>(out + n);
    const uint64_t w = ((uint64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    clk[2 * w] = t1 - t0;
    clk[2 * w + 1] = r1 - r0;
  }
}

// Dynamic (work-counter) xpose1nt: persistent grid, waves take 64-chunk groups.
__global__ void __launch_bounds__(256)
diag_xpose1nt_dyn(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                  uint4* __restrict__ out, uint32_t* counter) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_dyn_body<1, Md5Hasher<false>, 2>(base, n, len, stride, out, img, counter);
}

// xpose1nt without the peeled last stage (its refill re-reads the last 128 B
// of every chunk): A/B for the peel.
__global__ void __launch_bounds__(256)
diag_xpose1nt_nopeel(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                     uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wave_first = ((uint64_t)blockIdx.x * blockDim.x) + wave * 64u;
  if (wave_first >= n) return;
  Md5Hasher<false> h;
  fixed_xpose_group<1, Md5Hasher<false>, 2, false, false>(h, base, n, len, stride, out,
                                                          img + wave * 8192u, wave_first);
}

// Plain round-3 form (md5_core.h kX3 = false, the product before the xad
// pairs): the product loader and the compute-only body, for A/B.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
diag_xpose1nt_plain3(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<1, Md5Hasher<false, false>, 2>(base, n, len, stride, out, img);
}

__global__ void __launch_bounds__(256)
diag_compute_plain3(uint64_t n, uint32_t nblocks, uint4* __restrict__ out) {
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
      const uint32_t q = ((uint32_t)k + b) & 3u;
      w[k] = *reinterpret_cast<const uint4*>(rows + threadIdx.x * 64 + q * 16);
    }
    compress_regs<false, false>(st, w);
  }
  compress_pad_only(st, nblocks * 512u, 0u);
  if (i < n) out[i] = make_uint4(st.a, st.b, st.c, st.d);
}

// xpose layout filled by LDS-DMA instead of through VGPRs: per 128-B stage,
// 8 buffer_load_dwordx4 ... lds (8 rows x 128 B each, lane-linear
// destination = the xpose image layout), one 8 KiB image per wave; the DMA of
// stage s+1 is issued once this lane's reads of stage s have returned and
// runs under stage s's compression.  Saves the 8 ds_write_b128 per stage and
// the VGPR round trip of the data.
template <int CP>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
diag_xdma(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
          uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * 8192];
  Md5Hasher<false> h;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + wave * 8192u;
  const uint64_t wave_first = ((uint64_t)blockIdx.x * blockDim.x) + wave * 64u;
  if (wave_first >= n) return;
  const uint64_t left = n - wave_first;
  const uint32_t rows = left < 64 ? (uint32_t)left : 64u;
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(base + wave_first * stride);
  uint32_t voff[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint32_t row = (uint32_t)r * 8u + (lane >> 3);
    const uint32_t rc = row < rows ? row : rows - 1u;
    const uint32_t part = (lane & 7u) ^ ((row >> 1) & 7u);
    voff[r] = rc * (uint32_t)stride + part * 16u;
  }
  const uint32_t g = (lane >> 1) & 7u;
  const uint32_t nfull = len >> 6;
  const uint32_t nstage = nfull >> 1;
  typename Md5Hasher<false>::State st = h.init();
  auto issue = [&](uint32_t stg) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, img + r * 1024, 16, voff[r], stg * 128u, 0, CP);
  };
  if (nstage) {
    issue(0);
    for (uint32_t stg = 0; stg < nstage; ++stg) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint4 w[2][4];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(img + lane * 128 + ((q ^ g) * 16));
        w[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (stg + 1 < nstage) issue(stg + 1);
      __builtin_amdgcn_sched_barrier(0);
      h.block(st, w[0]);
      h.block(st, w[1]);
    }
  }
  const uint64_t i = wave_first + lane;
  const uint64_t ci = lane < rows ? i : n - 1;
  const uint8_t* chunk = base + ci * stride;
  if (nfull & 1u) {
    uint4 w[4];
    load_block(w, reinterpret_cast<const uint4*>(chunk + ((uint64_t)(nfull - 1) << 6)));
    h.block(st, w);
  }
  h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
  if (lane < rows) h.store(out, i, st);
}

// Double-buffered xdma: two 8 KiB images per wave, the DMA of stage s+2 goes
// into stage s's image as soon as this wave has read it, so a whole stage of
// compression covers each DMA's latency (one more stage in flight per wave,
// half the waves per CU: WPB waves per workgroup, 16 KiB LDS each).
template <int WPB>
__global__ void __launch_bounds__(64 * WPB)
diag_xdma2(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
           uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[WPB * 16384];
  Md5Hasher<false> h;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + wave * 16384u;
  const uint64_t wave_first = ((uint64_t)blockIdx.x * blockDim.x) + wave * 64u;
  if (wave_first >= n) return;
  const uint64_t left = n - wave_first;
  const uint32_t rows = left < 64 ? (uint32_t)left : 64u;
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(base + wave_first * stride);
  uint32_t voff[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint32_t row = (uint32_t)r * 8u + (lane >> 3);
    const uint32_t rc = row < rows ? row : rows - 1u;
    const uint32_t part = (lane & 7u) ^ ((row >> 1) & 7u);
    voff[r] = rc * (uint32_t)stride + part * 16u;
  }
  const uint32_t g = (lane >> 1) & 7u;
  const uint32_t nfull = len >> 6;
  const uint32_t nstage = nfull >> 1;
  typename Md5Hasher<false>::State st = h.init();
  auto issue = [&](uint32_t stg) __attribute__((always_inline)) {
    uint8_t* im = img + (stg & 1u) * 8192u;
#pragma unroll
    for (int r = 0; r < 8; ++r)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, im + r * 1024, 16, voff[r], stg * 128u, 0, 2);
  };
  if (nstage) {
    issue(0);
    if (nstage > 1) issue(1);
    for (uint32_t stg = 0; stg < nstage; ++stg) {
      // loads complete in order: with stage s+1's 8 DMAs still in flight,
      // vmcnt(8) means stage s has landed
      if (stg + 1 < nstage) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const uint8_t* im = img + (stg & 1u) * 8192u;
      uint4 w[2][4];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(im + lane * 128 + ((q ^ g) * 16));
        w[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (stg + 2 < nstage) issue(stg + 2);
      __builtin_amdgcn_sched_barrier(0);
      h.block(st, w[0]);
      h.block(st, w[1]);
    }
  }
  const uint64_t i = wave_first + lane;
  const uint64_t ci = lane < rows ? i : n - 1;
  const uint8_t* chunk = base + ci * stride;
  if (nfull & 1u) {
    uint4 w[4];
    load_block(w, reinterpret_cast<const uint4*>(chunk + ((uint64_t)(nfull - 1) << 6)));
    h.block(st, w);
  }
  h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
  if (lane < rows) h.store(out, i, st);
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

// VALU issue-rate probes: 8 independent chains per lane of one instruction
// kind (asm so nothing folds).  `clk` receives per-wave (s_memtime delta,
// s_memrealtime delta) for the in-kernel clock (MI355X_MICROARCH DVFS item 6).
template <int KIND>
__global__ void __launch_bounds__(256)
diag_valu_rate(uint32_t iters, uint32_t* __restrict__ out, uint64_t* __restrict__ clk) {
  uint32_t a[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) a[k] = threadIdx.x * 7u + (uint32_t)k;
  float f[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = (float)a[k];
  const uint32_t sv = iters ^ blockIdx.x;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  const uint64_t r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      if constexpr (KIND == 0)
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(sv), "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 1)
        asm volatile("v_alignbit_b32 %0, %0, %1, 7" : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 2)
        asm volatile("v_add_u32_e32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 3)
        asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(f[k]) : "v"(f[(k + 1) & 7]), "v"(1.0f));
      else if constexpr (KIND == 4)   // VOP3 encoding of a VOP2 op
        asm volatile("v_add_u32_e64 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 5)   // VOP2 with 32-bit literal (8-byte encoding)
        asm volatile("v_add_u32_e32 %0, 0x12345678, %0" : "+v"(a[k]));
      else if constexpr (KIND == 6)
        asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0xca" : "+v"(a[k]) : "v"(a[(k + 1) & 7]), "v"(a[(k + 2) & 7]));
      else if constexpr (KIND == 7)   // add3 with two VGPR + SGPR
        asm volatile("v_add3_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(a[(k + 1) & 7]), "s"(sv));
      else if constexpr (KIND == 8)
        asm volatile("v_xor_b32_e32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 9)
        asm volatile("v_mov_b32_e32 %0, %1" : "=v"(a[k]) : "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 10)
        asm volatile("v_bfi_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(a[(k + 1) & 7]), "v"(a[(k + 2) & 7]));
      else if constexpr (KIND == 11)
        asm volatile("v_lshl_add_u32 %0, %0, 3, %1" : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 12)   // 64-bit shift-add (gfx940+)
        asm volatile("v_lshl_add_u64 %0, %0, 3, %1" : "+v"(*reinterpret_cast<uint64_t*>(&a[k & 6])) : "v"(*reinterpret_cast<uint64_t*>(&a[(k + 2) & 6])));
      else if constexpr (KIND == 13)   // alignbit with SGPR shift
        asm volatile("v_alignbit_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(a[(k + 1) & 7]), "s"(sv));
      else if constexpr (KIND == 14)   // xad
        asm volatile("v_xad_u32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(a[(k + 1) & 7]), "v"(a[(k + 2) & 7]));
      else if constexpr (KIND == 15)   // perm
        asm volatile("v_perm_b32 %0, %0, %1, %2" : "+v"(a[k]) : "v"(a[(k + 1) & 7]), "v"(sv));
      else if constexpr (KIND == 16)   // SDWA add (word select)
        asm volatile("v_add_u32_sdwa %0, %0, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 17)   // VOP2 and
        asm volatile("v_and_b32_e32 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
      else if constexpr (KIND == 18)   // VOP2 shift
        asm volatile("v_lshlrev_b32_e32 %0, 5, %0" : "+v"(a[k]));
      else if constexpr (KIND == 19)   // v_pk_add_u16
        asm volatile("v_pk_add_u16 %0, %0, %1" : "+v"(a[k]) : "v"(a[(k + 1) & 7]));
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  const uint64_t r1 = __builtin_amdgcn_s_memrealtime();
  uint32_t x = 0;
#pragma unroll
  for (int k = 0; k < 8; ++k) x ^= a[k] ^ __float_as_uint(f[k]);
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  out[gid] = x;
  if ((threadIdx.x & 63u) == 0) {
    const uint32_t w = gid >> 6;
    clk[2 * w] = t1 - t0;
    clk[2 * w + 1] = r1 - r0;
  }
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
      hipLaunchKernelGGL(diag_compute<false>, dim3(grid), dim3(256), 0, s, n, len >> 6, o);
      break;
    case 12:
      hipLaunchKernelGGL(diag_compute<true>, dim3(grid), dim3(256), 0, s, n, len >> 6, o);
      break;
    case 20: hipLaunchKernelGGL(diag_xpose1_cp<0>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 21: hipLaunchKernelGGL(diag_xpose1_cp<1>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 22: hipLaunchKernelGGL(diag_xpose1_cp<2>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 23: hipLaunchKernelGGL(diag_xpose1_cp<3>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 24: hipLaunchKernelGGL(diag_xpose1_cp<16>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 25: hipLaunchKernelGGL(diag_xpose1_cp<18>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 26: hipLaunchKernelGGL(diag_xpose1_cp<19>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 34: case 35: case 36: case 37: {
      // occupancy A/B of the product xpose1nt kernel: extra dynamic LDS per
      // workgroup caps workgroups per CU (static image 32 KiB of 160 KiB):
      // 34: +0 (5 WG = 20 waves), 35: +8 KiB (4 WG = 16 waves, 64 waves per
      // CU = 4 whole generations), 36: +22 KiB (3 WG = 12 waves), 37: +48 KiB (2 WG)
      const size_t extra = kind == 34 ? 0 : kind == 35 ? 8192 : kind == 36 ? 22528 : 49152;
      if (extra > 32768)
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(md5_fixed_xpose1nt),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)extra);
      hipLaunchKernelGGL(md5_fixed_xpose1nt, dim3(grid), dim3(256), extra, s, b, n, len, stride, o);
      break;
    }
    case 61: case 62: {
      // occupancy A/B of the product xdma1nt kernel (as 34-37): 61: +8 KiB
      // (4 WG = 16 waves per CU), 62: +22 KiB (3 WG = 12 waves)
      const size_t extra = kind == 61 ? 8192 : 22528;
      hipLaunchKernelGGL(md5_fixed_xdma1nt, dim3(grid), dim3(256), extra, s, b, n, len, stride, o);
      break;
    }
    case 38: hipLaunchKernelGGL((diag_x64<2, false>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 39: hipLaunchKernelGGL((diag_x64<0, false>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 44: hipLaunchKernelGGL((diag_x64<2, true>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 45: hipLaunchKernelGGL((diag_x64<0, true>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 46: hipLaunchKernelGGL(diag_xpose2_pair<2>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 47: hipLaunchKernelGGL(diag_xpose2_pair<0>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 52: case 53: {
      // dynamic xpose1nt: 52 = 5 workgroups per CU (its occupancy), 53 = 4
      static uint32_t* counter = nullptr;
      if (!counter && hipMalloc((void**)&counter, 4) != hipSuccess) return -ENOMEM;
      int dev = 0, cus = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      (void)hipMemsetAsync(counter, 0, 4, s);
      const uint32_t g = (uint32_t)cus * (kind == 52 ? 5u : 4u);
      hipLaunchKernelGGL(diag_xpose1nt_dyn, dim3(g), dim3(256), 0, s, b, n, len, stride, o, counter);
      break;
    }
    case 55: hipLaunchKernelGGL(diag_xpose1nt_plain3, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 56: hipLaunchKernelGGL(diag_compute_plain3, dim3(grid), dim3(256), 0, s, n, len >> 6, o); break;
    case 57: hipLaunchKernelGGL(diag_xdma<2>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 63: hipLaunchKernelGGL(diag_xdma<3>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 64: hipLaunchKernelGGL(diag_xdma<18>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 65: hipLaunchKernelGGL(diag_xdma<19>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 66: hipLaunchKernelGGL(diag_xdma<1>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 59: hipLaunchKernelGGL(diag_xdma2<2>, dim3((uint32_t)((n + 127) / 128)), dim3(128), 0, s, b, n, len, stride, o); break;
    case 60: hipLaunchKernelGGL(diag_xdma2<1>, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, s, b, n, len, stride, o); break;
    case 58: hipLaunchKernelGGL(diag_xdma<0>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 54: hipLaunchKernelGGL(diag_xpose1nt_nopeel, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 91: case 92: case 93: case 94: case 95: {
      // DRAM-locality probes (diag_xdma_map): 91 = groups permuted, 92/93/94 =
      // lane stride 4/16/64, 95 = stride 16 + permuted.  n: a power of two,
      // a multiple of 64 * 64; 64 * S * stride < 2^32
      if ((n & (n - 1)) || n % (64u * 64u) || 64ull * 64u * stride >= (1ull << 32)) return -EINVAL;
      if (kind == 91) hipLaunchKernelGGL((diag_xdma_map<1, true>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      if (kind == 92) hipLaunchKernelGGL((diag_xdma_map<4, false>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      if (kind == 93) hipLaunchKernelGGL((diag_xdma_map<16, false>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      if (kind == 94) hipLaunchKernelGGL((diag_xdma_map<64, false>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      if (kind == 95) hipLaunchKernelGGL((diag_xdma_map<16, true>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    }
    case 90: hipLaunchKernelGGL(diag_xdma1nt_clk, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 51: hipLaunchKernelGGL(diag_crc_clk, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 50: hipLaunchKernelGGL(diag_xpose1nt_clk<FoldHasher>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 48: hipLaunchKernelGGL(diag_xpose1nt_clk<Md5Hasher<false>>, dim3(grid), dim3(256), 0, s, b, n, len, stride, o); break;
    case 49: hipLaunchKernelGGL(diag_compute_clk, dim3(grid), dim3(256), 0, s, n, len >> 6, o); break;
    case 40: case 41: case 42: case 43: {
      // compute-only occupancy sweep: static 16 KiB per workgroup plus extra
      // dynamic LDS caps workgroups per CU at 8 / 6 / 5 / 4 (32/24/20/16 waves)
      const size_t extra = kind == 40 ? 0 : kind == 41 ? 10240 : kind == 42 ? 16384 : 24576;
      hipLaunchKernelGGL(diag_compute<false>, dim3(grid), dim3(256), extra, s, n, len >> 6, o);
      break;
    }
    case 28: case 29: case 30: case 31: case 32: case 33: {
      // n = workgroups (64 threads, one wave each); len = bytes per chain
      const dim3 g1((uint32_t)n);
      const uint32_t nb = len >> 6;
      if (kind == 28) hipLaunchKernelGGL((diag_chain<64, false>), g1, dim3(64), 0, s, nb, o);
      if (kind == 29) hipLaunchKernelGGL((diag_chain<32, false>), g1, dim3(64), 0, s, nb, o);
      if (kind == 30) hipLaunchKernelGGL((diag_chain<16, false>), g1, dim3(64), 0, s, nb, o);
      if (kind == 31) hipLaunchKernelGGL((diag_chain<1, false>), g1, dim3(64), 0, s, nb, o);
      if (kind == 32) hipLaunchKernelGGL((diag_chain<64, true>), g1, dim3(64), 0, s, nb, o);
      if (kind == 33) hipLaunchKernelGGL((diag_chain<32, true>), g1, dim3(64), 0, s, nb, o);
      break;
    }
    case 81:   // n = workgroups, len = bytes per chain: two chains per lane, interleaved
      hipLaunchKernelGGL(diag_chain2, dim3((uint32_t)n), dim3(64), 0, s, len >> 6, o);
      break;
    case 80:   // n = workgroups, len = bytes per chain: the fed chain
      hipLaunchKernelGGL(diag_chain_fed, dim3((uint32_t)n), dim3(64), 0, s, len >> 6, o);
      break;
    case 84:   // n = workgroups, len = bytes per chain: 6 single adds per step
      hipLaunchKernelGGL(diag_chain_adds<false>, dim3((uint32_t)n), dim3(64), 0, s, len >> 6, o);
      break;
    case 85:   // the fed step with single adds (5 per step)
      hipLaunchKernelGGL(diag_chain_adds<true>, dim3((uint32_t)n), dim3(64), 0, s, len >> 6, o);
      break;
    case 13: case 14: {
      // single-chain latency: n lanes (one wave per CU at n = 16384), each
      // hashing `len` bytes; 64-thread workgroups so every CU gets one wave
      const dim3 g1((uint32_t)((n + 63) / 64));
      if (kind == 13) hipLaunchKernelGGL(diag_compute<false>, g1, dim3(64), 0, s, n, len >> 6, o);
      else hipLaunchKernelGGL(diag_compute<true>, g1, dim3(64), 0, s, n, len >> 6, o);
      break;
    }
    case 1:
      hipLaunchKernelGGL((md5_fixed_direct<2, FoldHasher>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 2:
      hipLaunchKernelGGL((md5_fixed_direct<4, FoldHasher>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 8:
      hipLaunchKernelGGL((md5_fixed_direct<2, FoldHasher, true>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 9:
      hipLaunchKernelGGL((md5_fixed_direct<4, FoldHasher, true>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 10:
      hipLaunchKernelGGL((md5_fixed_direct<2, Md5Hasher<false>, true>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 11:
      hipLaunchKernelGGL((md5_fixed_direct<4, Md5Hasher<false>, true>), dim3(grid), dim3(256), 0, s, b, n, len, stride, o);
      break;
    case 27: {
      int dev = 0, cus = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
      const uint64_t need = (n + 1023) / 1024;
      const uint32_t g = (uint32_t)(need < (uint64_t)cus ? need : (uint64_t)cus);
      hipLaunchKernelGGL(diag_crc_lane32_unpaired, dim3(g), dim3(1024), 0, s, b, n, len, stride, (uint32_t*)out);
      break;
    }
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
    case 100 ... 119: {
      // n = waves to launch (multiple of 4), len = iterations; out needs
      // 64*n u32 + 2*n u64 (clock pairs after the u32 area)
      uint32_t* o32 = (uint32_t*)out;
      uint64_t* clk = (uint64_t*)(o32 + 64 * n);
      const dim3 g((uint32_t)(n / 4));
#define RATE(K) if (kind == 100 + K) hipLaunchKernelGGL(diag_valu_rate<K>, g, dim3(256), 0, s, len, o32, clk);
      RATE(0) RATE(1) RATE(2) RATE(3) RATE(4) RATE(5) RATE(6) RATE(7) RATE(8) RATE(9)
      RATE(10) RATE(11) RATE(12) RATE(13) RATE(14) RATE(15) RATE(16) RATE(17) RATE(18) RATE(19)
#undef RATE
      break;
    }
    default:
      return -EINVAL;
  }
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Descriptor-kernel A/B (C3): 0 = (no kLat, no prio, D=2: round-1 kernel),
// 1 = (kLat, prio, D=2), 2 = D=4, 3 = D=8, 4 = D=8 without prio, 5 = D=12,
// 6 = D=8 with paired (whole-line) refill, 7 = D=8 holding the whole register
// file (one wave per SIMD: long chains run alone);
// +16: the same with 64-thread workgroups.
extern "C" int md5diag_desc(int kind, const void* base, const uint64_t* offs, const uint32_t* lens,
                            const uint32_t* order, uint64_t n, void* out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const uint32_t tpb = (kind & 16) ? 64u : 256u;
  const dim3 g((uint32_t)((n + tpb - 1) / tpb));
  const uint8_t* b = (const uint8_t*)base;
  uint4* o = (uint4*)out;
#define L(...) hipLaunchKernelGGL((md5_desc<__VA_ARGS__>), g, dim3(tpb), 0, s, b, offs, lens, order, n, (uint64_t)0, 0u, o)
  switch (kind & 15) {
    case 0: L(false, false, false, 2); break;
    case 1: L(false, true, true, 2); break;
    case 2: L(false, true, true, 4); break;
    case 3: L(false, true, true, 8); break;
    case 4: L(false, true, false, 8); break;
    case 5: L(false, true, true, 12); break;
    case 6: L(false, true, true, 8, true); break;
    case 7: L(false, true, true, 8, false, true); break;
    default: return -EINVAL;
  }
#undef L
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Placement / timing trace of the descriptor kernel: per wave, HW_ID,
// XCC_ID, s_memrealtime (100 MHz) at start and end.  rec[4*wave + 0..3].
template <int TPB>
__global__ void __launch_bounds__(256)
diag_desc_trace(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
                uint4* __restrict__ out, uint64_t* __restrict__ rec) {
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  desc_body<false, Md5Hasher<true>, true, 8>(base, offs, lens, order, n, 0, 0u, out);   // product config
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint64_t w = ((uint64_t)blockIdx.x * TPB + threadIdx.x) >> 6;
    rec[4 * w + 0] = hw;
    rec[4 * w + 1] = xcc;
    rec[4 * w + 2] = t0;
    rec[4 * w + 3] = t1;
  }
}

extern "C" int md5diag_desc_trace(int tpb, const void* base, const uint64_t* offs,
                                  const uint32_t* lens, const uint32_t* order, uint64_t n,
                                  void* out, void* rec, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (tpb == 256)
    hipLaunchKernelGGL(diag_desc_trace<256>, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s,
                       (const uint8_t*)base, offs, lens, order, n, (uint4*)out, (uint64_t*)rec);
  else
    hipLaunchKernelGGL(diag_desc_trace<64>, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, s,
                       (const uint8_t*)base, offs, lens, order, n, (uint4*)out, (uint64_t*)rec);
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// The product descriptor kernel (md5_desc_xpose) with `extra` bytes of dynamic
// LDS per 64-thread workgroup, which caps how many of its waves a CU holds
// (160 KiB / (8 KiB + extra)): a throttled short-chunk launch beside long
// chains (scripts/c3_throttle.py).
extern "C" int md5diag_desc_xpose_lds(const void* base, const uint64_t* offs, const uint32_t* lens,
                                      const uint32_t* order, uint64_t n, void* out,
                                      uint32_t extra, void* stream) {
  if (extra > 32768)
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(md5_desc_xpose),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)extra);
  hipLaunchKernelGGL(md5_desc_xpose, dim3((uint32_t)((n + 63) / 64)), dim3(64), extra,
                     (hipStream_t)stream, (const uint8_t*)base, offs, lens, order, n, (uint4*)out);
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// ---------------------------------------------------------------------------
// The round-1 A/B variants that left libmd5hip.so (md5_kernels_ab.h), by their
// former enum values (md5hip.h ABI 1), for A/B benches and parity tests:
//   fixed  2 direct4, 3 lds64, 4 lds128, 5 xpose1, 6 xpose2, 7 xpose1nt,
//          8 xpose2nt, 9 lds128nt  (1 direct2 and 10 xdma1nt: also the product's)
//   desc   2 xpose
//   crc    1 shared8, 2 lane32, 3 lane16, 4 xlane16, 5 xperm16; descriptor
//          batches: 5 = crc32_desc_xperm16
// ---------------------------------------------------------------------------
namespace {
int diag_cus() {
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 256;
  return cus;
}
template <int BB, bool NT>
int diag_launch_lds(const uint8_t* base, uint64_t n, uint32_t len, uint64_t stride, uint4* out,
                    hipStream_t s) {
  const size_t lds = (size_t)4 * 2 * 64 * BB;
  auto fn = BB == 64 ? md5_fixed_lds64 : NT ? md5_fixed_lds128nt : md5_fixed_lds128;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(fn),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -ENODEV;
  hipLaunchKernelGGL(fn, dim3((uint32_t)((n + 255) / 256)), dim3(256), lds, s, base, n, len, stride, out);
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
}  // namespace

namespace md5hip {
template __global__ void md5_fixed_direct<4, Md5Hasher<false>>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void crc32_fast<true>(const uint8_t*, const uint64_t*, const uint32_t*,
                                          uint64_t, uint64_t, uint32_t, uint32_t, uint32_t*);
}

// the round-1 fastcrc kernel (lane-direct), fixed-length chunks
extern "C" int md5diag_crc_fast_lane(const void* d_base, uint64_t n, uint32_t len, uint64_t stride,
                                     uint32_t fastcrc, uint32_t* d_out, void* stream) {
  if (n == 0) return 0;
  hipLaunchKernelGGL(crc32_fast<true>, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     (const uint8_t*)d_base, (const uint64_t*)nullptr, (const uint32_t*)nullptr, n,
                     stride, len, fastcrc, d_out);
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// fastcrc F = 64 / 128 with D window groups in flight per wave; P = false
// loads a 128-B window as two runs of four 16-B loads (the order before
// round 3's paired halves, depth code 20)
namespace md5hip {
template <int D, int T, bool P = true>
__global__ void __launch_bounds__(T)
diag_crc_fast_pipe(const uint8_t* __restrict__ base, uint64_t n, uint64_t stride, uint32_t flen,
                   uint32_t F, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32PermHasher::kLdsBytes];
  fast_pipe_body<D, P>(base, nullptr, nullptr, n, stride, flen, F, out, lds);
}
}  // namespace md5hip

extern "C" int md5diag_crc_fast_pipe(int depth, const void* d_base, uint64_t n, uint32_t len,
                                     uint64_t stride, uint32_t fastcrc, uint32_t* d_out, void* stream) {
  if (n == 0) return 0;
  if (fastcrc != 64 && fastcrc != 128) return -EINVAL;
  const dim3 g((uint32_t)(diag_cus() < (int)((2 * n + 63) / 64) ? diag_cus() : (2 * n + 63) / 64));
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* p = (const uint8_t*)d_base;
  // waves per CU so that the D buffers fit the register file: 16 / 12 / 8
  if (depth == 2) hipLaunchKernelGGL((diag_crc_fast_pipe<2, 1024>), g, dim3(1024), 0, s, p, n, stride, len, fastcrc, d_out);
  else if (depth == 3) hipLaunchKernelGGL((diag_crc_fast_pipe<3, 768>), g, dim3(768), 0, s, p, n, stride, len, fastcrc, d_out);
  else if (depth == 4) hipLaunchKernelGGL((diag_crc_fast_pipe<4, 512>), g, dim3(512), 0, s, p, n, stride, len, fastcrc, d_out);
  else if (depth == 13) hipLaunchKernelGGL((diag_crc_fast_pipe<2, 768>), g, dim3(768), 0, s, p, n, stride, len, fastcrc, d_out);
  else if (depth == 20) hipLaunchKernelGGL((diag_crc_fast_pipe<2, 1024, false>), g, dim3(1024), 0, s, p, n, stride, len, fastcrc, d_out);
  else return -EINVAL;
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// C2 energy per byte: fewer LDS round trips per byte --
// W 128-B stages per DMA round (W x 8 KiB image per wave: one vmcnt wait,
// one lgkmcnt wait and one DMA issue per W stages) -- against xdma1nt (W = 1).
// kPad: W = 1 with the LDS of W = 2 (the occupancy control).
namespace md5hip {
template <int W, bool kPad = false>
__global__ void __launch_bounds__(256)
diag_fixed_xdma_wide(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                     uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[4 * (kPad ? 2 : W) * 8192];
  Md5Hasher<false> h;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wave_first = (uint64_t)blockIdx.x * blockDim.x + wave * 64u;
  if (wave_first >= n) return;
  uint8_t* img = lds + wave * (kPad ? 2 : W) * 8192u;
  const uint64_t left = n - wave_first;
  const uint32_t rows = left < 64 ? (uint32_t)left : 64u;
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(base + wave_first * stride);
  uint32_t voff[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint32_t row = (uint32_t)r * 8u + (lane >> 3);
    const uint32_t rc = row < rows ? row : rows - 1u;
    const uint32_t part = (lane & 7u) ^ ((row >> 1) & 7u);
    voff[r] = rc * (uint32_t)stride + part * 16u;
  }
  const uint32_t g = (lane >> 1) & 7u;
  const uint32_t nfull = len >> 6;
  const uint32_t nstage = nfull >> 1;
  const uint32_t nws = (nstage + W - 1) / W;
  typename Md5Hasher<false>::State st = h.init();
  auto issue = [&](uint32_t ws) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
#pragma unroll
      for (int j = 0; j < W; ++j) {
        const uint32_t stg = ws * W + j;
        if (W == 1 || stg < nstage)
          __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, img + j * 8192 + r * 1024, 16, voff[r],
                                                   stg * 128u, 0, 2);
      }
  };
  if (nstage) {
    issue(0);
    for (uint32_t ws = 0; ws < nws; ++ws) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint4 w[W][2][4];
#pragma unroll
      for (int j = 0; j < W; ++j)
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          const u32x4 v = *reinterpret_cast<const u32x4*>(img + j * 8192 + lane * 128 + ((q ^ g) * 16));
          w[j][q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
        }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      if (ws + 1 < nws) issue(ws + 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int j = 0; j < W; ++j)
        if (ws * W + j < nstage) {
          h.block(st, w[j][0]);
          h.block(st, w[j][1]);
        }
    }
  }
  const uint64_t i = wave_first + lane;
  const uint64_t ci = lane < rows ? i : n - 1;
  const uint8_t* chunk = base + ci * stride;
  if (nfull & 1u) {
    uint4 w[4];
    load_block(w, reinterpret_cast<const uint4*>(chunk + ((uint64_t)(nfull - 1) << 6)));
    h.block(st, w);
  }
  h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
  if (lane < rows) h.store(out, i, st);
}
}  // namespace md5hip

extern "C" int md5diag_variant_fixed(int v, const void* d_base, uint64_t n, uint32_t len,
                                     uint64_t stride, void* d_out, void* stream) {
  if (n == 0) return 0;
  if (!d_base || !d_out || len > stride || ((uintptr_t)d_base & 15u) || (stride & 15u)) return -EINVAL;
  if (stride >= (1ull << 31) / 64) return -EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)d_base;
  uint4* o = (uint4*)d_out;
  const dim3 grid((uint32_t)((n + 255) / 256)), blk(256);
  typedef void (*K)(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
  K k = nullptr;
  switch (v) {
    case 1: k = md5_fixed_direct<2, Md5Hasher<false>>; break;
    case 2: k = md5_fixed_direct<4, Md5Hasher<false>>; break;
    case 3: return diag_launch_lds<64, false>(b, n, len, stride, o, s);
    case 4: return diag_launch_lds<128, false>(b, n, len, stride, o, s);
    case 9: return diag_launch_lds<128, true>(b, n, len, stride, o, s);
    case 5: k = md5_fixed_xpose1; break;
    case 6: k = md5_fixed_xpose2; break;
    case 7: k = md5_fixed_xpose1nt; break;
    case 8: k = md5_fixed_xpose2nt; break;
    case 10: k = md5_fixed_xdma1nt; break;
    case 70: k = diag_fixed_xdma_wide<2>; break;
    case 71: k = diag_fixed_xdma_wide<1, true>; break;
    case 72: k = diag_fixed_xdma_wide<4>; break;
    case 73: k = diag_fixed_xdma_wide<1>; break;
    default: return -EINVAL;
  }
  hipLaunchKernelGGL(k, grid, blk, 0, s, b, n, len, stride, o);
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int md5diag_variant_desc(int v, const void* d_base, const uint64_t* offs,
                                    const uint32_t* lens, const uint32_t* order, uint64_t n,
                                    void* d_out, void* stream) {
  if (n == 0) return 0;
  if (v >= 4 && v <= 8) {   // HYBRID with fed chains (md5_kernels.h), one long group per CU:
    // 4 / 5 = two addend tables, ring of 4 / 8 blocks; 6 = two tables, feeder
    // off (barriers only; timing); 7 = one table, ring 4; 8 = one table, feeder off
    const uint32_t nlong = (uint32_t)diag_cus();
    auto k = v == 4 ? md5_desc_hybrid_fed<4, 2> : v == 5 ? md5_desc_hybrid_fed<8, 2>
           : v == 6 ? md5_desc_hybrid_fed<4, 2, true> : v == 7 ? md5_desc_hybrid_fed<4, 1>
           : md5_desc_hybrid_fed<4, 1, true>;
    hipLaunchKernelGGL(k, dim3((uint32_t)hybrid_fed_grid(n, nlong)), dim3(128), 0,
                       (hipStream_t)stream, (const uint8_t*)d_base, offs, lens, order, n,
                       (uint4*)d_out, nlong);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
  }
  if (v == 9) {   // every group of >= 2 blocks as a fed pair (small batches)
    hipLaunchKernelGGL((md5_desc_fed_pairs<4, 2, 2>), dim3((uint32_t)((n + 63) / 64)), dim3(128), 0,
                       (hipStream_t)stream, (const uint8_t*)d_base, offs, lens, order, n, (uint4*)d_out);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
  }
  if (v != 2) return -EINVAL;
  hipLaunchKernelGGL(md5_desc_xpose, dim3((uint32_t)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     (const uint8_t*)d_base, offs, lens, order, n, (uint4*)d_out);
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Fed chains as a split launch (kind 0) or the same split with plain HYBRID
// lane-direct long waves in the first part (kind 1, control): groups
// [0, L = min(CUs, groups)) as md5_desc_fed_pairs on a high-priority stream,
// groups [L, ...) as md5_desc_xdma on `stream`, joined by events.  Needs an
// order (the split is by position in it).
extern "C" int md5diag_fed_split(int kind, const void* d_base, const uint64_t* offs,
                                 const uint32_t* lens, const uint32_t* order, uint64_t n,
                                 void* d_out, void* stream) {
  if (n == 0) return 0;
  if (!order) return -EINVAL;
  static hipStream_t hs = nullptr;
  static hipEvent_t e0 = nullptr, e1 = nullptr;
  if (!hs) {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
        hipStreamCreateWithPriority(&hs, hipStreamNonBlocking, hi) != hipSuccess ||
        hipEventCreateWithFlags(&e0, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e1, hipEventDisableTiming) != hipSuccess)
      return -ENODEV;
  }
  hipStream_t s = (hipStream_t)stream;
  const uint64_t groups = (n + 63) / 64;
  const uint64_t L = groups < (uint64_t)diag_cus() ? groups : (uint64_t)diag_cus();
  const uint8_t* b = (const uint8_t*)d_base;
  if (hipEventRecord(e0, s) != hipSuccess || hipStreamWaitEvent(hs, e0, 0) != hipSuccess) return -EIO;
  const uint64_t nfirst = L * 64 < n ? L * 64 : n;
  if (kind == 0)
    hipLaunchKernelGGL((md5_desc_fed_pairs<4, 2>), dim3((uint32_t)L), dim3(128), 0, hs, b, offs, lens,
                       order, nfirst, (uint4*)d_out);
  else
    hipLaunchKernelGGL(md5_desc_hybrid, dim3((uint32_t)L), dim3(64), 0, hs, b, offs, lens, order, nfirst,
                       (uint4*)d_out, (uint32_t)L);
  if (hipGetLastError() != hipSuccess) return -EIO;
  if (n > nfirst)
    hipLaunchKernelGGL(md5_desc_xdma, dim3((uint32_t)(groups - L)), dim3(64), 0, s, b, offs, lens,
                       order + nfirst, n - nfirst, (uint4*)d_out);
  if (hipGetLastError() != hipSuccess) return -EIO;
  if (hipEventRecord(e1, hs) != hipSuccess || hipStreamWaitEvent(s, e1, 0) != hipSuccess) return -EIO;
  return 0;
}

// Exclusive chain CUs.  As md5diag_fed_split, but the first L groups' pair
// (kind 0: fed chain + feeder) or lone chain wave (kind 1: HYBRID's
// lane-direct long wave, the control) is launched with its LDS padded to the
// CU's whole 160 KiB, so no other workgroup -- in particular no XDMA wave of
// the rest, launched beside it on `stream` -- shares its CU.  L is the
// caller's (the longest groups, in order).  kind 2: every group a padded fed
// pair, no rest (small batches; L ignored).
namespace {
int excl_pad(const void* k, uint32_t* pad) {
  hipFuncAttributes at;
  if (hipFuncGetAttributes(&at, k) != hipSuccess) return -EIO;
  const uint32_t total = 160u * 1024u;
  *pad = total > (uint32_t)at.sharedSizeBytes ? total - (uint32_t)at.sharedSizeBytes : 0u;
  return hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)*pad) == hipSuccess
             ? 0 : -EIO;
}
}  // namespace

extern "C" int md5diag_fed_split_excl(int kind, uint64_t L, const void* d_base, const uint64_t* offs,
                                      const uint32_t* lens, const uint32_t* order, uint64_t n,
                                      void* d_out, void* stream) {
  if (n == 0) return 0;
  const uint8_t* b = (const uint8_t*)d_base;
  const uint64_t groups = (n + 63) / 64;
  if (kind == 2) {
    const void* k = reinterpret_cast<const void*>(md5_desc_fed_pairs<4, 2, 2>);
    uint32_t pad = 0;
    if (int e = excl_pad(k, &pad)) return e;
    hipLaunchKernelGGL((md5_desc_fed_pairs<4, 2, 2>), dim3((uint32_t)groups), dim3(128), pad,
                       (hipStream_t)stream, b, offs, lens, order, n, (uint4*)d_out);
    return hipGetLastError() == hipSuccess ? 0 : -EIO;
  }
  if (!order || L == 0) return -EINVAL;
  static hipStream_t hs = nullptr;
  static hipEvent_t e0 = nullptr, e1 = nullptr;
  if (!hs) {
    int lo = 0, hi = 0;
    if (hipDeviceGetStreamPriorityRange(&lo, &hi) != hipSuccess ||
        hipStreamCreateWithPriority(&hs, hipStreamNonBlocking, hi) != hipSuccess ||
        hipEventCreateWithFlags(&e0, hipEventDisableTiming) != hipSuccess ||
        hipEventCreateWithFlags(&e1, hipEventDisableTiming) != hipSuccess)
      return -ENODEV;
  }
  hipStream_t s = (hipStream_t)stream;
  if (L > groups) L = groups;
  const uint64_t nfirst = L * 64 < n ? L * 64 : n;
  const void* k = kind != 1 ? reinterpret_cast<const void*>(md5_desc_fed_pairs<4, 2>)
                            : reinterpret_cast<const void*>(md5_desc_hybrid);
  uint32_t pad = 0;
  if (int e = excl_pad(k, &pad)) return e;
  if (hipEventRecord(e0, s) != hipSuccess || hipStreamWaitEvent(hs, e0, 0) != hipSuccess) return -EIO;
  if (kind != 1)
    hipLaunchKernelGGL((md5_desc_fed_pairs<4, 2>), dim3((uint32_t)L), dim3(128), pad, hs, b, offs, lens,
                       order, nfirst, (uint4*)d_out);
  else
    hipLaunchKernelGGL(md5_desc_hybrid, dim3((uint32_t)L), dim3(64), pad, hs, b, offs, lens, order, nfirst,
                       (uint4*)d_out, (uint32_t)L);
  if (hipGetLastError() != hipSuccess) return -EIO;
  if (n > nfirst && kind == 3)     // the rest as HYBRID: its own longest groups lane-direct
    hipLaunchKernelGGL(md5_desc_hybrid, dim3((uint32_t)(groups - L)), dim3(64), 0, s, b, offs, lens,
                       order + nfirst, n - nfirst, (uint4*)d_out, (uint32_t)(diag_cus() - (int)L));
  else if (n > nfirst)
    hipLaunchKernelGGL(md5_desc_xdma, dim3((uint32_t)(groups - L)), dim3(64), 0, s, b, offs, lens,
                       order + nfirst, n - nfirst, (uint4*)d_out);
  if (hipGetLastError() != hipSuccess) return -EIO;
  if (hipEventRecord(e1, hs) != hipSuccess || hipStreamWaitEvent(s, e1, 0) != hipSuccess) return -EIO;
  return 0;
}

extern "C" int md5diag_variant_crc(int v, const void* d_base, uint64_t n, uint32_t len,
                                   uint64_t stride, uint32_t* d_out, void* stream) {
  if (n == 0) return 0;
  if (!d_base || !d_out || len > stride || ((uintptr_t)d_base & 15u) || (stride & 15u)) return -EINVAL;
  if (stride >= (1ull << 31) / 64) return -EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* b = (const uint8_t*)d_base;
  const uint64_t groups = (n + 63) / 64;
  const uint32_t percu = (uint32_t)(groups < (uint64_t)diag_cus() ? groups : (uint64_t)diag_cus());
  switch (v) {
    case 1:
      hipLaunchKernelGGL(crc32_fixed_xpose, dim3((uint32_t)((n + 255) / 256)), dim3(256), 0, s, b, n,
                         len, stride, d_out);
      break;
    case 2: case 3: {
      const uint64_t need = (n + 1023) / 1024, cap = (uint64_t)diag_cus() * (v == 2 ? 1 : 2);
      hipLaunchKernelGGL(v == 2 ? crc32_fixed_lane32 : crc32_fixed_lane16,
                         dim3((uint32_t)(need < cap ? need : cap)), dim3(1024), 0, s, b, n, len, stride, d_out);
      break;
    }
    case 4:
      hipLaunchKernelGGL(crc32_fixed_xlane16, dim3(percu), dim3(1024), 0, s, b, n, len, stride, d_out);
      break;
    case 5:
      hipLaunchKernelGGL(crc32_fixed_xperm16, dim3(percu), dim3(1024), 0, s, b, n, len, stride, d_out);
      break;
    default:
      return -EINVAL;
  }
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

extern "C" int md5diag_variant_crc_desc(int v, const void* d_base, const uint64_t* offs,
                                        const uint32_t* lens, const uint32_t* order, uint64_t n,
                                        uint32_t* d_out, void* stream) {
  if (n == 0) return 0;
  if (v != 5) return -EINVAL;
  const uint64_t groups = (n + 63) / 64;
  const uint32_t percu = (uint32_t)(groups < (uint64_t)diag_cus() ? groups : (uint64_t)diag_cus());
  hipLaunchKernelGGL(crc32_desc_xperm16, dim3(percu), dim3(1024), 0, (hipStream_t)stream,
                     (const uint8_t*)d_base, offs, lens, order, n, d_out);
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// ---------------------------------------------------------------------------
// The product descriptor kernels (XDMA / HYBRID) with a per-wave record:
// HW_ID, XCC_ID, s_memrealtime (100 MHz) at start and end -- where the waves
// of a coalesced mixed batch ran and for how long (scripts/c3_trace_x.py).
//   kind 0  md5_desc_xdma      kind 1  md5_desc_hybrid (whole-line refill, product)
//   kind 2  md5_desc_hybrid with the round-1 single-block refill (A/B)
// rec == nullptr: no record (timing-only A/B).
// ---------------------------------------------------------------------------
namespace md5hip {
// kVPad: the kernel claims VGPRs up to v[kVPad] (an empty asm clobber), so the
// register file, not LDS, caps its waves per SIMD (4 at v127, 3 at v167, 2 at
// v255) -- evenly over the four SIMDs, as HYBRID's 163 VGPRs do.
template <uint32_t kLong, bool kLongPair, int CP = 2, int kVPad = 0>
__global__ void __launch_bounds__(64)
diag_desc_x(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
            const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
            uint4* __restrict__ out, uint32_t nlong, uint64_t* __restrict__ rec) {
  __shared__ __attribute__((aligned(16))) uint8_t img[8192];
  if constexpr (kVPad == 127) asm volatile("" ::: "v127");
  else if constexpr (kVPad == 167) asm volatile("" ::: "v167");
  else if constexpr (kVPad == 255) asm volatile("" ::: "v255");
  else if constexpr (kVPad == 511) asm volatile("" ::: "v255", "a255");   // the whole file
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  Md5Hasher<true> h;
  const uint64_t first = (uint64_t)blockIdx.x * 64u;
  if (first < n)
    desc_xpose_group<CP, Md5Hasher<true>, kLong, 1, false, true, true, DescArrays, kLongPair>(
        h, base, DescArrays{offs, lens, order}, n, first, out, img, nlong);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if (rec && (threadIdx.x & 63u) == 0) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint64_t w = blockIdx.x;
    rec[4 * w + 0] = hw;
    rec[4 * w + 1] = xcc;
    rec[4 * w + 2] = t0;
    rec[4 * w + 3] = t1;
  }
}
}  // namespace md5hip

extern "C" int md5diag_desc_x(int kind, const void* base, const uint64_t* offs, const uint32_t* lens,
                              const uint32_t* order, uint64_t n, void* out, uint32_t nlong, void* rec,
                              void* stream) {
  if (n == 0) return 0;
  const dim3 g((uint32_t)((n + 63) / 64)), b(64);
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* bs = (const uint8_t*)base;
  uint64_t* r = (uint64_t*)rec;
  if (kind == 0)
    hipLaunchKernelGGL((diag_desc_x<0, true>), g, b, 0, s, bs, offs, lens, order, n, (uint4*)out, nlong, r);
  else if (kind == 1)
    hipLaunchKernelGGL((diag_desc_x<kHybridLongBlocks, true>), g, b, 0, s, bs, offs, lens, order, n,
                       (uint4*)out, nlong, r);
  else if (kind == 2)
    hipLaunchKernelGGL((diag_desc_x<kHybridLongBlocks, false>), g, b, 0, s, bs, offs, lens, order, n,
                       (uint4*)out, nlong, r);
  else if (kind == 3)        // XDMA, default cache policy
    hipLaunchKernelGGL((diag_desc_x<0, true, 0>), g, b, 0, s, bs, offs, lens, order, n, (uint4*)out,
                       nlong, r);
  else if (kind == 4)        // HYBRID, default cache policy
    hipLaunchKernelGGL((diag_desc_x<kHybridLongBlocks, true, 0>), g, b, 0, s, bs, offs, lens, order, n,
                       (uint4*)out, nlong, r);
  else if (kind == 8)        // XDMA, 4 / 3 / 2 waves per SIMD by VGPRs
    hipLaunchKernelGGL((diag_desc_x<0, true, 2, 127>), g, b, 0, s, bs, offs, lens, order, n,
                       (uint4*)out, nlong, r);
  else if (kind == 9)
    hipLaunchKernelGGL((diag_desc_x<0, true, 2, 167>), g, b, 0, s, bs, offs, lens, order, n,
                       (uint4*)out, nlong, r);
  else if (kind == 10)
    hipLaunchKernelGGL((diag_desc_x<0, true, 2, 255>), g, b, 0, s, bs, offs, lens, order, n,
                       (uint4*)out, nlong, r);
  else if (kind == 11)       // HYBRID at 2 / 1 waves per SIMD by registers (a chain's SIMD
    hipLaunchKernelGGL((diag_desc_x<kHybridLongBlocks, true, 2, 255>), g, b, 0, s, bs, offs, lens,
                       order, n, (uint4*)out, nlong, r);   // shared with one / no other wave)
  else if (kind == 12)
    hipLaunchKernelGGL((diag_desc_x<kHybridLongBlocks, true, 2, 511>), g, b, 0, s, bs, offs, lens,
                       order, n, (uint4*)out, nlong, r);
  else if (kind >= 5 && kind <= 7) {   // XDMA at 16 / 12 / 8 waves per CU (dynamic LDS pad)
    const uint32_t waves = kind == 5 ? 16u : kind == 6 ? 12u : 8u;
    const uint32_t pad = (160u * 1024u) / waves - 8192u + 64u;
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(diag_desc_x<0, true, 2>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, (int)pad);
    hipLaunchKernelGGL((diag_desc_x<0, true, 2>), g, b, pad, s, bs, offs, lens, order, n, (uint4*)out,
                       nlong, r);
  }
  else
    return -EINVAL;
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Descriptor XDMA with two LDS-DMA images per wave (stage s+2's DMA issued as
// stage s is read), default cache policy: for 16-B-packed ragged batches the
// line two stages share is then fetched twice within one stage instead of a
// compression apart.  16 KiB LDS per one-wave workgroup.
// md5diag_desc_x2: kind 0 = this, kind 1 = the same with one image (16 KiB
// allocated, so occupancy matches).
namespace md5hip {
template <int NB>
__global__ void __launch_bounds__(64)
diag_desc_x2(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
             const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
             uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[16384];
  asm volatile("" ::: "v127");
  Md5Hasher<true> h;
  const uint64_t first = (uint64_t)blockIdx.x * 64u;
  if (first < n)
    desc_xpose_group<0, Md5Hasher<true>, 0, 1, false, true, true, DescArrays, true, NB>(
        h, base, DescArrays{offs, lens, order}, n, first, out, img);
}
}  // namespace md5hip

extern "C" int md5diag_desc_x2(int kind, const void* base, const uint64_t* offs, const uint32_t* lens,
                               const uint32_t* order, uint64_t n, void* out, void* stream) {
  if (n == 0) return 0;
  const dim3 g((uint32_t)((n + 63) / 64)), b(64);
  hipStream_t s = (hipStream_t)stream;
  if (kind == 0)
    hipLaunchKernelGGL(md5hip::diag_desc_x2<2>, g, b, 0, s, (const uint8_t*)base, offs, lens, order, n,
                       (uint4*)out);
  else if (kind == 1)
    hipLaunchKernelGGL(md5hip::diag_desc_x2<1>, g, b, 0, s, (const uint8_t*)base, offs, lens, order, n,
                       (uint4*)out);
  else
    return -EINVAL;
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// md5_desc_balanced_t with the per-wave record of md5diag_desc_x (one record
// per persistent wave: its whole run over the groups it took, and how many)
// for WPB waves per workgroup, NB LDS-DMA images per wave, split queues (A/B).
namespace md5hip {
template <int WPB, int NB, bool kSplit, int W = 1, bool kHashOff = false, int CP = 2,
          uint32_t kLong = 0>
__global__ void __launch_bounds__(64 * WPB)
diag_desc_balanced(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                   const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
                   uint4* __restrict__ out, uint32_t* __restrict__ ctr, uint64_t* __restrict__ rec) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  const uint32_t taken =
      balanced_body<WPB, NB, kSplit, W, kHashOff, CP, kLong>(base, offs, lens, order, n, out, ctr,
                                                            lds_dyn);
  const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
  if ((threadIdx.x & 63u) == 0 && rec) {
    uint32_t hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    const uint64_t w = (uint64_t)blockIdx.x * WPB + (threadIdx.x >> 6);
    rec[5 * w + 0] = hw;
    rec[5 * w + 1] = xcc;
    rec[5 * w + 2] = t0;
    rec[5 * w + 3] = t1;
    rec[5 * w + 4] = taken;
  }
}
}  // namespace md5hip

namespace {
template <int WPB, int NB, bool kSplit, int W = 1, bool kHashOff = false, int CP = 2,
          uint32_t kLong = 0>
int diag_launch_balanced(const void* base, const uint64_t* offs, const uint32_t* lens,
                         const uint32_t* order, uint64_t n, void* out, uint32_t* ctr, void* rec,
                         hipStream_t s) {
  const uint32_t lds = BalancedCfg<WPB, NB, W>::kLds;
  auto kern = diag_desc_balanced<WPB, NB, kSplit, W, kHashOff, CP, kLong>;
  if (hipFuncSetAttribute(reinterpret_cast<const void*>(kern),
                          hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) != hipSuccess)
    return -ENODEV;
  hipLaunchKernelGGL(kern, dim3((uint32_t)diag_cus()), dim3(64 * WPB),
                     lds, s, (const uint8_t*)base, offs, lens, order, n, (uint4*)out, ctr,
                     (uint64_t*)rec);
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}
}  // namespace

// rec: 5 x uint64 per wave (WPB x CUs waves), or nullptr.  kind (waves per
// WG / buffers NB / 128-B stages per wide stage W): 0 = 4/1/1, 1 = 4/2/1, 2 = 8/1/1, 3 = 8/1/1 split queues, 4 = 8/2/1 split,
// 5 = 4/1/2, 6 = 4/1/4, 7 = 4/2/2, 14 = 4/1/5; loads
// only (no compression, digests meaningless): 8 = 4/1/1, 9 = 4/1/2,
// 10 = 4/1/4, 11 = 4/2/2, 12 = 4/2/1, 13 = 8/1/1, 15 = 4/1/5.  Default cache
// policy instead of nt (lines stay in L2: a 16-B-aligned chunk's visit
// boundaries share a 128-B line): 16 = 4/1/4, 17 = 4/1/4 loads only,
// 18 = 4/1/2, 19 = 4/1/1 (the product's shape), 20 = 4/2/1, 21 = 8/1/1, 22 = 4/1/1 loads only,
// 23 = 8/1/1 split queues; 24 / 25 = the product's shape with groups whose
// longest chunk is >= 256 KiB / 1 MiB run lane-direct (HYBRID's long path);
// 26 = the product's shape with three images, stages register-pipelined.
extern "C" int md5diag_desc_balanced(int kind, const void* base, const uint64_t* offs,
                                     const uint32_t* lens, const uint32_t* order, uint64_t n,
                                     void* out, void* rec, void* stream) {
  if (n == 0) return 0;
  static uint32_t* ctr = nullptr;
  if (!ctr && hipMalloc(&ctr, 16) != hipSuccess) return -ENOMEM;
  hipStream_t s = (hipStream_t)stream;
  if (hipMemsetAsync(ctr, 0, 16, s) != hipSuccess) return -EIO;
  switch (kind) {
    case 0: return diag_launch_balanced<4, 1, false>(base, offs, lens, order, n, out, ctr, rec, s);
    case 1: return diag_launch_balanced<4, 2, false>(base, offs, lens, order, n, out, ctr, rec, s);
    case 2: return diag_launch_balanced<8, 1, false>(base, offs, lens, order, n, out, ctr, rec, s);
    case 3: return diag_launch_balanced<8, 1, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 4: return diag_launch_balanced<8, 2, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 5: return diag_launch_balanced<4, 1, false, 2>(base, offs, lens, order, n, out, ctr, rec, s);
    case 6: return diag_launch_balanced<4, 1, false, 4>(base, offs, lens, order, n, out, ctr, rec, s);
    case 7: return diag_launch_balanced<4, 2, false, 2>(base, offs, lens, order, n, out, ctr, rec, s);
    case 8: return diag_launch_balanced<4, 1, false, 1, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 9: return diag_launch_balanced<4, 1, false, 2, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 10: return diag_launch_balanced<4, 1, false, 4, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 11: return diag_launch_balanced<4, 2, false, 2, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 12: return diag_launch_balanced<4, 2, false, 1, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 13: return diag_launch_balanced<8, 1, false, 1, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 14: return diag_launch_balanced<4, 1, false, 5>(base, offs, lens, order, n, out, ctr, rec, s);
    case 15: return diag_launch_balanced<4, 1, false, 5, true>(base, offs, lens, order, n, out, ctr, rec, s);
    case 16: return diag_launch_balanced<4, 1, false, 4, false, 0>(base, offs, lens, order, n, out, ctr, rec, s);
    case 17: return diag_launch_balanced<4, 1, false, 4, true, 0>(base, offs, lens, order, n, out, ctr, rec, s);
    case 18: return diag_launch_balanced<4, 1, false, 2, false, 0>(base, offs, lens, order, n, out, ctr, rec, s);
    case 19: return diag_launch_balanced<4, 1, false, 1, false, 0>(base, offs, lens, order, n, out, ctr, rec, s);
    case 20: return diag_launch_balanced<4, 2, false, 1, false, 0>(base, offs, lens, order, n, out, ctr, rec, s);
    case 21: return diag_launch_balanced<8, 1, false, 1, false, 0>(base, offs, lens, order, n, out, ctr, rec, s);
    case 22: return diag_launch_balanced<4, 1, false, 1, true, 0>(base, offs, lens, order, n, out, ctr, rec, s);
    case 23: return diag_launch_balanced<8, 1, true, 1, false, 0>(base, offs, lens, order, n, out, ctr, rec, s);
    case 24: return diag_launch_balanced<4, 1, false, 1, false, 2, kHybridLongBlocks>(base, offs, lens, order, n, out,
                                                                                     ctr, rec, s);
    case 25: return diag_launch_balanced<4, 1, false, 1, false, 2, 4 * kHybridLongBlocks>(base, offs, lens, order, n,
                                                                                         out, ctr, rec, s);
    case 26: return diag_launch_balanced<4, 3, false, 1, false, 2>(base, offs, lens, order, n, out, ctr, rec, s);
    default: return -EINVAL;
  }
}
