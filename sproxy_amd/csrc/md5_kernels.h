// md5_kernels.h -- batched per-chunk digests (MD5, CRC32) over independent
// chunks, hand-written for gfx950; the digest is a policy (hashers.h).
//
// One lane hashes one chunk (MD5 is a strict 64-step chain per block, so the
// only parallelism is across chunks).  A 64-lane wave owns 64 chunks.  What
// differs between the kernels is how message blocks travel HBM -> VGPRs:
//
//   md5_fixed_direct  each lane streams its own chunk with global_load_dwordx4
//                     (4 per 64-B block), a D-deep register ring in flight.
//   md5_fixed_lds     the wave fetches its 64 chunks' next block(s) with
//                     LDS-DMA (global_load_lds_dwordx4: 4 or 8 lanes per chunk,
//                     so each wave-instruction reads whole 64/128-B runs), then
//                     every lane pulls its own row out of LDS with ds_read_b128.
//                     Source-side XOR swizzle keeps the row reads conflict-free.
//   md5_desc          per-chunk (offset, length) descriptors, optional
//                     permutation (longest-first packing), any alignment.
//
// Reference semantics: md5.c:153-265 (Init/Update/Final) applied to each chunk
// independently; digests are bit-exact with md5.c (tests/test_gpu_parity.py).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "hashers.h"
#include "md5_core.h"

namespace md5hip {

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint4 ld16(const uint4* p) {
  const u32x4 v = *reinterpret_cast<const u32x4*>(p);
  return make_uint4(v.x, v.y, v.z, v.w);
}

__device__ __forceinline__ void load_block(uint4 (&r)[4], const uint4* p) {
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = ld16(p + k);
}

// A buffer descriptor the compiler can prove wave-uniform: both address
// halves go through readfirstlane.  Without that proof hipcc wraps every
// buffer_load in a waterfall loop (4 v_readfirstlane + 2 v_cmp + exec juggling
// per load; it did so in crc32_fixed_xpose, whose table setup precedes it).
__device__ __forceinline__ __amdgpu_buffer_rsrc_t uniform_rsrc(const uint8_t* p) {
  const uint64_t a = (uint64_t)(uintptr_t)p;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  void* u = (void*)(uintptr_t)(((uint64_t)hi << 32) | lo);
  return __builtin_amdgcn_make_buffer_rsrc(u, (short)0, 0x7FFFFFFF, 0x00020000);
}

// ---------------------------------------------------------------------------
// Fixed-length, lane-direct loads.  base/stride 16-B aligned, len <= stride.
// ---------------------------------------------------------------------------
// (hashers without LDS state only: Md5Hasher, FoldHasher)
// Ring refill.  kPair: slots are refilled two at a time (blocks 2k, 2k+1 --
// one whole 128-B line when the chunk is 128-B aligned), so a lane never
// leaves half a line in the cache for a later instruction: with ~16 waves x
// 64 lanes per CU the half-consumed lines of all lanes add up to the size of
// an XCD's L2, and unpaired refills re-fetch the evicted halves.
template <class H, int D, bool kPair>
__device__ __forceinline__ void ring_steps(H& h, typename H::State& st, uint4 (&R)[D][4],
                                           const uint4* p, uint32_t blk, uint32_t lastb) {
#pragma unroll
  for (int j = 0; j < D; ++j) {
    h.block(st, R[j]);
    if constexpr (kPair) {
      if (j & 1) {
        load_block(R[j - 1], p + 4 * min(blk + j - 1 + D, lastb));
        load_block(R[j], p + 4 * min(blk + j + D, lastb));
      }
    } else {
      load_block(R[j], p + 4 * min(blk + j + D, lastb));
    }
  }
}

template <int D, class H = Md5Hasher<false>, bool kPair = false>
__global__ void __launch_bounds__(256)
md5_fixed_direct(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 typename H::Out* __restrict__ out) {
  static_assert(!kPair || D % 2 == 0, "paired refill needs an even ring");
  H h;
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* chunk = base + i * stride;
  const uint4* p = reinterpret_cast<const uint4*>(chunk);
  const uint32_t nfull = len >> 6;
  typename H::State st = h.init();
  if (nfull) {
    // D-deep register ring.  Prefetch indices are clamped to the last block so
    // every load is unconditional (no phi copies); the <= D re-reads at the end
    // hit in L1/L2.
    const uint32_t lastb = nfull - 1;
    uint4 R[D][4];
#pragma unroll
    for (int j = 0; j < D; ++j) load_block(R[j], p + 4 * min((uint32_t)j, lastb));
    uint32_t blk = 0;
    for (; blk + D <= nfull; blk += D)     // steady state: no conditionals, so
      ring_steps<H, D, kPair>(h, st, R, p, blk, lastb);   // the waits stay counted
#pragma unroll
    for (int j = 0; j < D - 1; ++j)
      if (blk + j < nfull) h.block(st, R[j]);
  }
  h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
  h.store(out, i, st);
}

// ---------------------------------------------------------------------------
// Fixed-length, xpose image filled by LDS-DMA ("xdma"; the default).
// The same 8 chunks x 128 B wave-instructions and the same LDS image layout
// as the xpose kernels (lane-linear destination = row r*8 + lane/8, slot
// lane%8 holding part (lane%8) ^ ((row>>1)&7)), but issued as
// buffer_load_dwordx4 ... lds: the data skips the VGPRs and the 8
// ds_write_b128 per stage.  One 8 KiB image per wave: once this lane's
// ds_reads of stage s have returned, the DMA of stage s+1 is issued and runs
// under stage s's compression.  The kernel is power-bound, so
// the saved instructions and register traffic buy clock: 1.7 % faster.
// Requires 64 * stride < 2^31 (checked by the launcher).
// ---------------------------------------------------------------------------
// xdma_group: one wave hashes the 64-chunk group starting at wave_first (< n)
// through its 8 KiB image `img`; the hasher is set up by the caller.
template <class H, int CP = 2>
__device__ __forceinline__ void xdma_group(H& h, const uint8_t* __restrict__ base, uint64_t n,
                                           uint32_t len, uint64_t stride, uint64_t wave_first,
                                           typename H::Out* __restrict__ out, uint8_t* img) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t left = n - wave_first;
  const uint32_t rows = left < 64 ? (uint32_t)left : 64u;
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(base + wave_first * stride);
  uint32_t voff[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint32_t row = (uint32_t)r * 8u + (lane >> 3);
    const uint32_t rc = row < rows ? row : rows - 1u;            // ragged last wave
    const uint32_t part = (lane & 7u) ^ ((row >> 1) & 7u);       // source swizzle
    voff[r] = rc * (uint32_t)stride + part * 16u;
  }
  const uint32_t g = (lane >> 1) & 7u;
  const uint32_t nfull = len >> 6;
  const uint32_t nstage = nfull >> 1;
  typename H::State st = h.init();
  // CP applies to line-aligned chunks; with base or stride off the 128-B
  // line a stage shares a line with the next, which must stay in L2: default
  // policy (as desc_xpose_group)
  const bool lined = ((((uintptr_t)base + wave_first * stride) | stride) & 127u) == 0;
  auto run = [&](auto pol) __attribute__((always_inline)) {
    constexpr int P = decltype(pol)::value;
    auto issue = [&](uint32_t stg) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < 8; ++r)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rsrc, img + r * 1024, 16, voff[r], stg * 128u, 0, P);
    };
    issue(0);
    for (uint32_t stg = 0; stg < nstage; ++stg) {
      // hipcc does not order ds_read after an LDS-DMA into the same bytes, so
      // wait explicitly; exactly one stage is in flight here
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      uint4 w[2][4];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(img + lane * 128 + ((q ^ g) * 16));
        w[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the refill
      if (stg + 1 < nstage) issue(stg + 1);
      __builtin_amdgcn_sched_barrier(0);
      h.block(st, w[0]);
      h.block(st, w[1]);
    }
  };
  if (nstage) {
    if (CP == 0 || !lined) run(std::integral_constant<int, 0>{});
    else run(std::integral_constant<int, CP>{});
  }
  // leftover odd block, then the tail
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

template <class H = Md5Hasher<false>, int CP = 2>
__device__ __forceinline__ void fixed_xdma_body(const uint8_t* __restrict__ base, uint64_t n,
                                                uint32_t len, uint64_t stride,
                                                typename H::Out* __restrict__ out, uint8_t* lds) {
  H h;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wave_first = ((uint64_t)blockIdx.x * blockDim.x) + wave * 64u;
  if (wave_first >= n) return;
  xdma_group<H, CP>(h, base, n, len, stride, wave_first, out, lds + wave * 8192u);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
md5_fixed_xdma1nt(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                  uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xdma_body<Md5Hasher<false>, 2>(base, n, len, stride, out, img);
}

// ---------------------------------------------------------------------------
// Descriptor batch: chunk c = order ? order[i] : i at base + offs[c], lens[c].
// Per-lane trip counts differ, so the host packs lanes longest-first
// (md5hip_plan_order).  Lanes whose chunk start is 16-B aligned stream it
// with dwordx4 loads through a 2-block ring; unaligned chunks take aligned
// dword loads + v_alignbit_b32 (17 loads per block).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void load_block_unaligned(uint4 (&r)[4], const uint8_t* p) {
  const uintptr_t addr = (uintptr_t)p;
  const uint32_t* w = reinterpret_cast<const uint32_t*>(addr & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(addr & 3u) * 8u;
  uint32_t v[17];
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = w[j];
  // The 17th word starts at addr - sh/8 + 64 < addr + 64 <= chunk end only when
  // sh != 0; with sh == 0 it would lie past the block and is not needed.
  v[16] = sh ? w[16] : 0u;
  uint32_t o[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) o[j] = __builtin_amdgcn_alignbit(v[j + 1], v[j], sh);
#pragma unroll
  for (int k = 0; k < 4; ++k) r[k] = make_uint4(o[4 * k], o[4 * k + 1], o[4 * k + 2], o[4 * k + 3]);
}

// Wave-uniform max over the 64 lanes (butterfly), for the priority choice.
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return __builtin_amdgcn_readfirstlane(v);
}
__device__ __forceinline__ uint32_t wave_min(uint32_t v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = min(v, (uint32_t)__shfl_xor((int)v, o, 64));
  return __builtin_amdgcn_readfirstlane(v);
}

// One lane digests [chunk, chunk + len) into st (blocks + finish): aligned
// chunks through a D-deep dwordx4 register ring, unaligned ones through
// dword loads + v_alignbit_b32.
template <class H, int D, bool kPair = false>
__device__ __forceinline__ void lane_range(H& h, typename H::State& st, const uint8_t* chunk,
                                           uint32_t len) {
  const uint32_t nfull = len >> 6;
  if (((uintptr_t)chunk & 15u) == 0) {
    const uint4* p = reinterpret_cast<const uint4*>(chunk);
    if (nfull) {
      const uint32_t lastb = nfull - 1;
      uint4 R[D][4];
#pragma unroll
      for (int j = 0; j < D; ++j) load_block(R[j], p + 4 * min((uint32_t)j, lastb));
      uint32_t blk = 0;
      for (; blk + D <= nfull; blk += D)
        ring_steps<H, D, kPair>(h, st, R, p, blk, lastb);
#pragma unroll
      for (int j = 0; j < D - 1; ++j)
        if (blk + j < nfull) h.block(st, R[j]);
    }
  } else {
    for (uint32_t blk = 0; blk < nfull; ++blk) {
      uint4 w[4];
      load_block_unaligned(w, chunk + ((uint64_t)blk << 6));
      h.block(st, w);
    }
  }
  h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
}

// kImplicit: chunk i at base + i*stride with length `flen` (the fixed-length
// API's fallback for chunk starts that are not 16-B aligned).
// kLat: latency-form step (md5_core.h).  kPrio: waves holding long chunks
// raise their issue priority, so the longest serial chains -- which bound a
// mixed batch -- progress at their latency limit while short-chunk waves fill
// the remaining issue slots.
// D: depth of the per-lane register ring (blocks in flight per lane).  Mixed
// batches have few waves per SIMD (C3: ~1.2), so latency must be hidden by
// prefetch depth, not by occupancy.
template <bool kImplicit, class H = Md5Hasher<true>, bool kPrio = true, int D = 8,
          bool kPair = false, bool kHog = false>
__device__ __forceinline__ void desc_body(const uint8_t* __restrict__ base,
                                          const uint64_t* __restrict__ offs,
                                          const uint32_t* __restrict__ lens,
                                          const uint32_t* __restrict__ order, uint64_t n,
                                          uint64_t stride, uint32_t flen,
                                          typename H::Out* __restrict__ out,
                                          uint8_t* hlds = nullptr) {
  H h;
  h.setup(hlds);                     // before any early exit (may barrier)
  if constexpr (kHog)                // claim the whole register file: one wave per SIMD
    asm volatile("" ::: "v255", "a255");
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t c = (!kImplicit && order) ? (uint64_t)order[i] : i;
  const uint8_t* chunk = base + (kImplicit ? c * stride : offs[c]);
  const uint32_t len = kImplicit ? flen : lens[c];
  const uint32_t nfull = len >> 6;
  if constexpr (kPrio) {
    const uint32_t wmax = wave_max(nfull);
    if (wmax >= 4096u) __builtin_amdgcn_s_setprio(3);        // >= 256 KiB
    else if (wmax >= 1024u) __builtin_amdgcn_s_setprio(2);   // >= 64 KiB
    else if (wmax >= 256u) __builtin_amdgcn_s_setprio(1);    // >= 16 KiB
  }
  typename H::State st = h.init();
  lane_range<H, D, kPair>(h, st, chunk, len);
  h.store(out, c, st);
}

template <bool kImplicit, bool kLat = true, bool kPrio = true, int D = 8, bool kPair = false,
          bool kHog = false>
__global__ void __launch_bounds__(256)
md5_desc(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
         const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
         uint64_t stride, uint32_t flen, uint4* __restrict__ out) {
  desc_body<kImplicit, Md5Hasher<kLat>, kPrio, D, kPair, kHog>(base, offs, lens, order, n, stride,
                                                               flen, out);
}

// ---------------------------------------------------------------------------
// Descriptor batch with whole-line loads ("desc xpose").  A netcache batch is
// mostly full chunk_size blocks plus each object's shorter last block
// (blk_io.c:377); lanes are ordered longest-first (md5hip_plan_order), so a
// wave's 64 chunks have nearly equal lengths.  The wave then loads like the
// fixed xpose kernel -- each global_load_dwordx4 wave-instruction reads 8
// chunks x 128 B -- from per-row 64-bit addresses (chunks lie anywhere in the
// arena), a row's stage index clamped to its own last stage, and a lane
// compresses a stage only while it still has one.  Rows without any 128-B
// stage re-read the wave's longest chunk (always in bounds).  A wave with a
// chunk start that is not 16-B aligned takes the lane-direct path (desc_body).
// One wave per workgroup, as md5_desc: the dispatcher spreads long-chunk waves
// one per CU, and s_setprio favours them.
// ---------------------------------------------------------------------------
// kLong > 0: the first `nlong` waves (one per CU; with longest-first order
// these hold the batch's longest chunks) take the lane-direct path with an
// 8-block register ring when their longest chunk has >= kLong blocks.  The
// host planner (md5hip_plan_desc) picks this variant only for batches whose
// longest chunks stand out; a test inside the kernel cost the lane-direct
// ring its loads in flight (hipcc kept 7 instead of 28 outstanding).  Such a
// wave is a serial chain that runs nearly alone on its SIMD: the xpose
// stage's LDS round trip (8 ds_write_b128 + 8 ds_read_b128 + waits per
// 128 B) sits on its critical path, while one lane-direct wave per CU does
// not yet crowd the address unit (4 per CU did: DESIGN.md §5, C3).
// kHalf: 4 KiB half image (rows 0-31, then rows 32-63, as xpose_half_group) so
// a hasher with large LDS tables fits beside 16 waves' images; `first` is the
// wave's first position in `order` (< n), the hasher is set up by the caller.
// kDma (full image, D = 1): the 8 row loads of a stage are LDS-DMA
// (global_load_lds_dwordx4 from the same per-row addresses) straight into the
// image, as fixed_xdma_body: no VGPR staging, no ds_write; the DMA of stage
// s+1 is issued once this wave's row reads of stage s have returned.
// HYBRID's test that a wave's long chunks are the batch's critical path: in
// longest-first order, the chunk `depth` positions in (two waves per CU) is at
// most a quarter of this wave's longest.  A batch of equal-length blocks
// (a netcache chunk_size sweep) fails it and keeps the xpose/xdma loader for
// every wave; a mixed batch (C3) or a batch of fewer chunks than two waves
// per CU passes, and its first waves run their chains lane-direct.
__device__ __forceinline__ bool long_outlier(const uint32_t* __restrict__ lens,
                                             const uint32_t* __restrict__ order, uint64_t n,
                                             uint64_t depth, uint32_t bmax) {
  const uint64_t p = depth < n - 1 ? depth : n - 1;
  const uint32_t probe = lens[order ? order[p] : p] >> 6;
  return 4u * (uint64_t)probe <= bmax;
}

// HYBRID's lane-direct threshold: a wave whose longest chunk has this many
// 64-B blocks (256 KiB)
constexpr uint32_t kHybridLongBlocks = 4096;

// Where chunk i of a descriptor batch lies: (offset, length) arrays, packed
// onto lanes in `order` when given.
struct DescArrays {
  const uint64_t* __restrict__ offs;
  const uint32_t* __restrict__ lens;
  const uint32_t* __restrict__ order;
  static constexpr bool kPairXor = false;
  static constexpr bool kAbs = false;          // off() is relative to base
  __device__ __forceinline__ uint64_t index(uint64_t i) const { return order ? (uint64_t)order[i] : i; }
  __device__ __forceinline__ uint64_t off(uint64_t c) const { return offs[c]; }
  __device__ __forceinline__ uint32_t len(uint64_t c) const { return lens[c]; }
};

// blk_make_crc's fastcrc windows (blk_io.c:408-424) as a descriptor batch of
// 2n rows: row 2k = the first F bytes of chunk k, row 2k+1 = its last F
// bytes; a chunk of <= F bytes is row 2k alone (row 2k+1 empty: CRC 0, the
// XOR identity).  kPairXor: lanes 2k and 2k+1 combine, out[k] = crc ^ crc.
// Chunk k at offs[k] / lens[k], or (offs == nullptr) at k * stride, flen.
struct FastWindows {
  const uint64_t* __restrict__ offs;
  const uint32_t* __restrict__ lens;
  uint64_t stride;
  uint32_t flen, F;
  static constexpr bool kPairXor = true;
  static constexpr bool kAbs = false;
  __device__ __forceinline__ uint64_t index(uint64_t i) const { return i; }
  __device__ __forceinline__ uint32_t clen(uint64_t k) const { return offs ? lens[k] : flen; }
  __device__ __forceinline__ uint64_t off(uint64_t c) const {
    const uint64_t k = c >> 1;
    const uint64_t o = offs ? offs[k] : k * stride;
    const uint32_t L = clen(k);
    return ((c & 1u) && L > F) ? o + (L - F) : o;
  }
  __device__ __forceinline__ uint32_t len(uint64_t c) const {
    const uint32_t L = clen(c >> 1);
    return L <= F ? ((c & 1u) ? 0u : L) : F;
  }
};

// A finished lane's digest: stored at c, or (kPairXor) XORed with its pair
// lane and stored by the even lane at c / 2.  Pairs are live together.
template <class Src, class H>
__device__ __forceinline__ void emit(H& h, typename H::Out* __restrict__ out, uint64_t c,
                                     const typename H::State& st) {
  if constexpr (Src::kPairXor) {
    const uint32_t v = st.c ^ (uint32_t)__shfl_xor((int)st.c, 1, 64);
    if (!(c & 1u)) out[c >> 1] = v;
  } else {
    h.store(out, c, st);
  }
}

// kLongPair: HYBRID's lane-direct long waves refill their 8-block ring two
// blocks (one whole 128-B line) at a time, so no lane leaves half a line
// behind to be fetched again after eviction (ring_steps).
// NB (kDma): LDS-DMA images per wave, 1 or 2.  2 is BALANCED's lone wave per
// SIMD: the next stage's DMA goes into the other image under this stage's
// row reads (below).
// kShift (kDma, one image): a wave holding a chunk that does not start on a
// 128-B line loads whole LINES instead of chunk-relative 128-B stages, each
// line once; a lane rotates its line reads by its chunk's 16-B offset s and
// takes a window's last s pieces from the next line (one line of registers
// more, 32 v_cndmask per 128 B).  Chunk-relative stages of such a chunk
// straddle two lines and share one with the next stage, which L2 evicts
// between the two visits under 16 waves per CU (16-B-packed ragged blocks:
// 1.29x the payload read from HBM).
template <int CP, class H, uint32_t kLong = 0, int D = 1, bool kHalf = false, bool kPeel = true,
          bool kDma = false, class Src = DescArrays, bool kLongPair = true, int NB = 1,
          bool kShift = false>
__device__ __forceinline__ void desc_xpose_group(H& h, const uint8_t* __restrict__ base,
                                                 const Src& src, uint64_t n,
                                                 uint64_t first, typename H::Out* __restrict__ out,
                                                 uint8_t* img, uint32_t nlong = 0) {
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t i = first + lane;
  const bool live = i < n;
  const uint64_t c = src.index(live ? i : first);
  const uint64_t off = src.off(c);
  const uint8_t* chunk = Src::kAbs ? reinterpret_cast<const uint8_t*>((uintptr_t)off) : base + off;
  const uint32_t len = live ? src.len(c) : 0u;
  const uint32_t nfull = len >> 6;
  const uint32_t nst = nfull >> 1;                       // this lane's 128-B stages
  const uint32_t smax = wave_max(nst);
  const uint32_t bmax = wave_max(nfull);
  if (bmax >= 4096u) __builtin_amdgcn_s_setprio(3);      // as desc_body
  else if (bmax >= 1024u) __builtin_amdgcn_s_setprio(2);
  else if (bmax >= 256u) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);                    // (a persistent wave's previous group)
  typename H::State st = h.init();
  const bool unaligned = __ballot(live && (((uintptr_t)chunk & 15u) != 0)) != 0;
  if (kLong && bmax >= kLong && (first >> 6) < nlong) {
    if (live) {
      lane_range<H, 8, kLongPair>(h, st, chunk, len);
      emit<Src>(h, out, c, st);
    }
    return;
  }
  if (unaligned) {
    if (live) {                      // rare: a short ring keeps VGPRs for the main path
      lane_range<H, 2>(h, st, chunk, len);
      emit<Src>(h, out, c, st);
    }
    return;
  }
  if (smax) {
    // the row with the most stages stands in for rows without any
    const uint32_t mrow = __builtin_ctzll(__ballot(nst == smax));
    const uint8_t* rptr[8];            // base + offset: stays a global pointer (no flat loads)
    uint32_t rlast[8];
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      uint32_t row = (uint32_t)r * 8u + (lane >> 3);
      const uint32_t rn = (uint32_t)__shfl((int)nst, (int)row, 64);
      if (rn == 0) row = mrow;
      const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)off, (int)row, 64);
      const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(off >> 32), (int)row, 64);
      const uint32_t part = (lane & 7u) ^ ((row >> 1) & 7u);      // source swizzle (xpose)
      const uint64_t ra = (((uint64_t)hi << 32) | lo) + part * 16u;
      rptr[r] = Src::kAbs ? reinterpret_cast<const uint8_t*>((uintptr_t)ra) : base + ra;
      rlast[r] = (rn ? rn : smax) - 1u;
    }
    const uint32_t g = (lane >> 1) & 7u;
    auto load_stage = [&](u32x4 (&R)[8], uint32_t stg) __attribute__((always_inline)) {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const u32x4* a = reinterpret_cast<const u32x4*>(rptr[r] + (min(stg, rlast[r]) << 7));
        R[r] = CP ? __builtin_nontemporal_load(a) : *a;
      }
    };
    const uint8_t* myrow = img + (kHalf ? (lane & 31u) : lane) * 128u;
    auto read_row = [&](uint4 (&w)[2][4]) __attribute__((always_inline)) {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const u32x4 v = *reinterpret_cast<const u32x4*>(myrow + ((q ^ g) * 16));
        w[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
      }
    };
    auto consume = [&](u32x4 (&R)[8], uint32_t stg, uint32_t next, bool refill = true)
        __attribute__((always_inline)) {
      uint4 w[2][4];
      if constexpr (kHalf) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          *reinterpret_cast<u32x4*>(img + r * 1024 + lane * 16) = R[r];
        __builtin_amdgcn_wave_barrier();
        if (lane < 32u) read_row(w);
        __builtin_amdgcn_wave_barrier();
#pragma unroll
        for (int r = 4; r < 8; ++r)
          *reinterpret_cast<u32x4*>(img + (r - 4) * 1024 + lane * 16) = R[r];
        __builtin_amdgcn_wave_barrier();
        if (lane >= 32u) read_row(w);
      } else {
#pragma unroll
        for (int r = 0; r < 8; ++r)
          *reinterpret_cast<u32x4*>(img + r * 1024 + lane * 16) = R[r];
        __builtin_amdgcn_wave_barrier();
        read_row(w);
      }
      __builtin_amdgcn_wave_barrier();
      if (refill) load_stage(R, next);
      __builtin_amdgcn_sched_barrier(0);
      if (stg < nst) {
        h.block(st, w[0]);
        h.block(st, w[1]);
      }
    };
    static_assert(NB == 1 || (NB == 2 && kDma), "LDS-DMA images per wave: 1 or 2");
    if constexpr (kDma && NB == 2) {
      // Two 8 KiB images for a LONE wave on its SIMD (BALANCED): a lone
      // wave issues one instruction per slot, so everything it does besides
      // VALU comes straight off its chain.  Per 128-B stage: the next stage's
      // DMA goes into the other image BEFORE this stage's rows are read (so
      // the ds_read latency is spent issuing it, not waiting), block 0 starts
      // as soon as its four rows are in (lgkmcnt(4)), and the DMA's LDS base
      // is set twice per stage, not eight times: rows 0-3 / 4-7 take M0 =
      // image / image + 4 KiB and their 1 KiB row offset in the instruction
      // (which adds it to the global address too, so the row pointers are
      // pre-biased by it).  The DMA lead stays one stage, as with one image:
      // a third image for a two-stage lead (the 96 KiB a CU already reserves
      // for BALANCED) measured 1.0-1.4 % slower on 3 and 6 coalesced C3
      // batches (profiles/r04h/balanced3_ab.json).
      static_assert(D == 1 && !kHalf, "LDS-DMA images: full 8 KiB stages");
      const bool lined = __ballot(((uint32_t)(uintptr_t)chunk & 127u) != 0 && live && nst != 0) == 0;
      const uint32_t rmin = wave_min(nst ? nst : smax) - 1u;
      auto* limg = (__attribute__((address_space(3))) uint8_t*)img;
      const uint8_t* bptr[8];
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        bptr[r] = rptr[r] - (r & 3) * 1024;
        asm volatile("" : "+v"(bptr[r]));      // keep the bias in the pointer (not re-added per stage)
      }
      auto run2 = [&](auto pol) __attribute__((always_inline)) {
        constexpr int P = decltype(pol)::value;
        // row R's DMA (the offset must be an immediate: R is a template constant)
        auto dma = [&](auto R, const uint8_t* g, __attribute__((address_space(3))) uint8_t* im)
            __attribute__((always_inline)) {
          constexpr int r = decltype(R)::value;
          __builtin_amdgcn_global_load_lds(g, im + (r >> 2) * 4096, 16, (r & 3) * 1024, P);
        };
        // stage stg into image B (a template constant: the image bases fold
        // into M0 values and ds_read offsets, no address arithmetic per stage)
        auto issue = [&](uint32_t stg, auto B) __attribute__((always_inline)) {
          auto* im = limg + decltype(B)::value * 8192u;
          auto rows = [&](auto... R) __attribute__((always_inline)) {
            if (stg <= rmin) {                                 // wave-uniform, no row clamped
              const uint64_t so = (uint64_t)stg << 7;
              (dma(R, bptr[decltype(R)::value] + so, im), ...);
            } else {
              (dma(R, bptr[decltype(R)::value] + (min(stg, rlast[decltype(R)::value]) << 7), im), ...);
            }
          };
          rows(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{},
               std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{},
               std::integral_constant<int, 4>{}, std::integral_constant<int, 5>{},
               std::integral_constant<int, 6>{}, std::integral_constant<int, 7>{});
        };
        using I0 = std::integral_constant<int, 0>;
        using I1 = std::integral_constant<int, 1>;
        // this lane's 8 row-piece addresses in image 0, kept in VGPRs: image
        // 1's are the same + 8192, an immediate of the ds_read
        using lds_u4 = const __attribute__((address_space(3))) u32x4;
        uint32_t raddr[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) {
          raddr[q] = (uint32_t)(uintptr_t)(limg + (myrow - img) + ((q ^ g) * 16));
          asm volatile("" : "+v"(raddr[q]));
        }
        // one stage held in image B; the next goes into the other one
        auto stage = [&](uint32_t stg, auto B) __attribute__((always_inline)) {
          constexpr int b = decltype(B)::value;
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");      // stage stg landed (the only one out)
          uint4 w[2][4];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const u32x4 v = *reinterpret_cast<lds_u4*>(raddr[q] + b * 8192u);
            w[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
          }
          if (stg + 1 < smax) {                                  // issued under the reads' latency
            if constexpr (b == 0) issue(stg + 1, I1{});
            else issue(stg + 1, I0{});
          }
          asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");   // block 0's rows
          __builtin_amdgcn_sched_barrier(0);
          if (stg < nst) h.block(st, w[0]);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          if (stg < nst) h.block(st, w[1]);
        };
        // The stages every live lane holds whole, whose next DMAs
        // clamp no row: no per-lane guard, no clamp test (the common case:
        // LPT groups are near-uniform), four stages per loop test.  The row
        // pointers are formed once per four stages (pb = bptr + offset); the
        // stages' DMAs reach +128 .. +512 through the instruction offset,
        // which the LDS address takes too, so their M0 is the image base less
        // that much (the images sit kImgPad bytes into the workgroup's LDS,
        // balanced_body).
        auto dma_at = [&](auto R, auto OFF, const uint8_t* g, __attribute__((address_space(3))) uint8_t* im)
            __attribute__((always_inline)) {
          constexpr int r = decltype(R)::value;
          constexpr int o = decltype(OFF)::value;
          __builtin_amdgcn_global_load_lds(g, im + (r >> 2) * 4096 - o, 16, (r & 3) * 1024 + o, P);
        };
        auto stage_all = [&](const uint8_t* const (&pb)[8], auto J) __attribute__((always_inline)) {
          constexpr int j = decltype(J)::value;                 // stage j of the quad
          constexpr int b = j & 1;
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          uint4 w[2][4];
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const u32x4 v = *reinterpret_cast<lds_u4*>(raddr[q] + b * 8192u);
            w[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
          }
          {
            auto* im = limg + (b ^ 1) * 8192u;
            using O = std::integral_constant<int, 128 * (j + 1)>;   // the next stage: quad + j + 1
            auto rows = [&](auto... R) __attribute__((always_inline)) {
              (dma_at(R, O{}, pb[decltype(R)::value], im), ...);
            };
            rows(std::integral_constant<int, 0>{}, std::integral_constant<int, 1>{},
                 std::integral_constant<int, 2>{}, std::integral_constant<int, 3>{},
                 std::integral_constant<int, 4>{}, std::integral_constant<int, 5>{},
                 std::integral_constant<int, 6>{}, std::integral_constant<int, 7>{});
          }
          asm volatile("s_waitcnt lgkmcnt(4)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          h.block(st, w[0]);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_sched_barrier(0);
          h.block(st, w[1]);
        };
        const uint32_t fmin = wave_min(live ? nst : 0xFFFFFFFFu);   // stages every live lane holds
        const uint32_t lim = min(rmin, fmin - 1u);                 // fmin 0: wraps, guarded below
        issue(0, I0{});
        uint32_t stg = 0;
        if (fmin > 0)
          for (; stg + 4 <= lim; stg += 4) {
            const uint8_t* pb[8];
            const uint64_t so = (uint64_t)stg << 7;
#pragma unroll
            for (int r = 0; r < 8; ++r) pb[r] = bptr[r] + so;
            stage_all(pb, std::integral_constant<int, 0>{});
            stage_all(pb, std::integral_constant<int, 1>{});
            stage_all(pb, std::integral_constant<int, 2>{});
            stage_all(pb, std::integral_constant<int, 3>{});
          }
        for (; stg < smax; stg += 2) {
          stage(stg, I0{});
          if (stg + 1 < smax) stage(stg + 1, I1{});
        }
      };
      if (CP == 0 || !lined) run2(std::integral_constant<int, 0>{});
      else run2(std::integral_constant<int, CP>{});
    } else if constexpr (kDma) {
      static_assert(D == 1 && !kHalf, "LDS-DMA image: one full 8 KiB stage");
      // Cache policy per wave: CP (nt for the product kernels) when every
      // row starts on a 128-B line; otherwise each 128-B stage straddles two
      // lines and shares one with the row's next stage, and nt loads let that
      // line leave L2 before the next stage asks for it (16-B-packed ragged
      // blocks: 1.83x HBM bytes, 1.35x time), so such waves load with the
      // default policy (profiles/r02_desc_cache_policy_ab.json).
      const bool lined =
          __ballot(((uint32_t)(uintptr_t)chunk & 127u) != 0 && live && nst != 0) == 0;
      // Until the first row runs out (stage rmin), no row's stage index is
      // clamped and the stage offset is wave-uniform: one 64-bit add per row
      // with the offset in SGPRs instead of min + shift + add (16 VALU fewer
      // per 128-B stage, ~2.5 % of the stage's VALU).
      const uint32_t rmin = wave_min(nst ? nst : smax) - 1u;
      // the image as an LDS pointer once: a generic pointer per DMA costs a
      // null-check select (2 SALU) per row and stage
      auto* limg = (__attribute__((address_space(3))) uint8_t*)img;
      auto run = [&](auto pol) __attribute__((always_inline)) {
        constexpr int P = decltype(pol)::value;
        auto issue = [&](uint32_t stg) __attribute__((always_inline)) {
          if (stg <= rmin) {                                   // wave-uniform
            const uint64_t so = (uint64_t)stg << 7;
#pragma unroll
            for (int r = 0; r < 8; ++r)
              __builtin_amdgcn_global_load_lds(rptr[r] + so, limg + r * 1024, 16, 0, P);
          } else {
#pragma unroll
            for (int r = 0; r < 8; ++r)
              __builtin_amdgcn_global_load_lds(rptr[r] + (min(stg, rlast[r]) << 7), limg + r * 1024,
                                               16, 0, P);
          }
        };
        issue(0);
        for (uint32_t stg = 0; stg < smax; ++stg) {
          // hipcc does not order ds_read after an LDS-DMA into the same bytes
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          uint4 w[2][4];
          read_row(w);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the refill
          if (stg + 1 < smax) issue(stg + 1);
          __builtin_amdgcn_sched_barrier(0);
          if (stg < nst) {
            h.block(st, w[0]);
            h.block(st, w[1]);
          }
        }
      };
      // kShift: whole lines.  Row r's line L is the 128-B line L of its chunk's
      // line-aligned base; window k (chunk bytes [128k, 128k + 128)) is line k
      // from piece s on, then line k + 1's first s pieces.  A lane reads line
      // L rotated by s (piece q of the read = line piece (q + s) & 7), so
      // window k's piece q is line k's read for q + s < 8, line k+1's after.
      // Lines 0..smax (a row with s > 0 needs line nst; one with s = 0 is
      // clamped to its own last stage).
      auto run_lines = [&]() __attribute__((always_inline)) {
        // rptr / rlast re-pointed at lines (their stage values are dead here)
        const uint64_t ca = (uint64_t)(uintptr_t)chunk;
#pragma unroll
        for (int r = 0; r < 8; ++r) {
          uint32_t row = (uint32_t)r * 8u + (lane >> 3);
          const uint32_t rn = (uint32_t)__shfl((int)nst, (int)row, 64);
          if (rn == 0) row = mrow;
          const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)ca, (int)row, 64);
          const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(ca >> 32), (int)row, 64);
          const uint32_t part = (lane & 7u) ^ ((row >> 1) & 7u);      // source swizzle (xpose)
          rptr[r] = reinterpret_cast<const uint8_t*>(
              (uintptr_t)((((uint64_t)hi << 32) | (lo & ~127u)) + part * 16u));
          rlast[r] = (rn ? rn : smax) - 1u + ((lo & 127u) != 0u);
        }
        auto issue = [&](uint32_t L) __attribute__((always_inline)) {
          if (L <= rmin) {                                     // wave-uniform, no row clamped
            const uint64_t so = (uint64_t)L << 7;
#pragma unroll
            for (int r = 0; r < 8; ++r)
              __builtin_amdgcn_global_load_lds(rptr[r] + so, limg + r * 1024, 16, 0, 0);
          } else {
#pragma unroll
            for (int r = 0; r < 8; ++r)
              __builtin_amdgcn_global_load_lds(rptr[r] + (min(L, rlast[r]) << 7), limg + r * 1024, 16,
                                               0, 0);
          }
        };
        const uint32_t sh = ((uint32_t)ca >> 4) & 7u;
        auto read_rot = [&](uint4 (&R)[2][4]) __attribute__((always_inline)) {
#pragma unroll
          for (int q = 0; q < 8; ++q) {
            const u32x4 v = *reinterpret_cast<const u32x4*>(myrow + ((((q + sh) & 7u) ^ g) * 16));
            R[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
          }
        };
        uint4 ra[2][4], rb[2][4];
        issue(0);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        read_rot(ra);
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        issue(1);
        // window k: `cur` (line k) completed in place from `nxt` (line k + 1,
        // read here; the next window's `cur`)
        auto step = [&](uint32_t k, uint4 (&cur)[2][4], uint4 (&nxt)[2][4]) __attribute__((always_inline)) {
          asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
          read_rot(nxt);
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // reads done before the refill
          if (k + 2 <= smax) issue(k + 2);
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int q = 0; q < 8; ++q)
            if ((uint32_t)q + sh >= 8u) cur[q >> 2][q & 3] = nxt[q >> 2][q & 3];
          if (k < nst) {
            h.block(st, cur[0]);
            h.block(st, cur[1]);
          }
        };
        for (uint32_t k = 0; k < smax; k += 2) {
          step(k, ra, rb);
          if (k + 1 < smax) step(k + 1, rb, ra);
        }
      };
      if (kShift && !lined) run_lines();
      else if (CP == 0 || !lined) run(std::integral_constant<int, 0>{});
      else run(std::integral_constant<int, CP>{});
    } else {
    // D-stage register ring (2*D blocks of prefetch per lane)
    const uint32_t lasts = smax - 1;
    u32x4 R[D][8];
#pragma unroll
    for (int j = 0; j < D; ++j) load_stage(R[j], min((uint32_t)j, lasts));
    uint32_t stg = 0;
    if constexpr (D == 1 && kPeel) {
      for (; stg + 1 < smax; ++stg) consume(R[0], stg, stg + 1);   // last stage peeled:
      consume(R[0], stg, 0, false);                               // no re-read past the end
    } else {
      for (; stg + D <= smax; stg += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) consume(R[j], stg + j, min(stg + j + D, lasts));
      }
#pragma unroll
      for (int j = 0; j < D - 1; ++j)
        if (stg + j < smax) consume(R[j], stg + j, lasts);
    }
    }
  }
  if (live) {
    if (nfull & 1u) {
      uint4 w[4];
      load_block(w, reinterpret_cast<const uint4*>(chunk + ((uint64_t)(nfull - 1) << 6)));
      h.block(st, w);
    }
    h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
    emit<Src>(h, out, c, st);
  }
}

template <int CP, class H = Md5Hasher<true>, uint32_t kLong = 0, int D = 1, bool kDma = false,
          bool kShift = false>
__device__ __forceinline__ void desc_xpose_body(const uint8_t* __restrict__ base,
                                                const uint64_t* __restrict__ offs,
                                                const uint32_t* __restrict__ lens,
                                                const uint32_t* __restrict__ order, uint64_t n,
                                                typename H::Out* __restrict__ out, uint8_t* img,
                                                uint32_t nlong = 0) {
  H h;
  const uint64_t first = ((uint64_t)blockIdx.x * blockDim.x) + (threadIdx.x & ~63u);
  if (first >= n) return;
  desc_xpose_group<CP, H, kLong, D, false, true, kDma, DescArrays, true, 1, kShift>(
      h, base, DescArrays{offs, lens, order}, n, first, out, img, nlong);
}

// Occupancy: 81 VGPRs and the 8 KiB image would allow 5 one-wave workgroups
// per SIMD; claiming VGPRs up to v127 (an empty asm clobber) makes the
// register file cap it at 4 per SIMD, and the descriptor batches run 3-7 %
// faster (u16k 3.13 -> 2.89 ms, 16-B-packed ragged 3.14 -> 3.06,
// profiles/r02_desc_occupancy_ab.json; HYBRID's 163 VGPRs, 3 per SIMD, did
// the same).  Capping through LDS instead (16 or 12 waves per CU) was slower:
// with one-wave workgroups an LDS limit is per CU, not per SIMD.
__global__ void __launch_bounds__(64)
md5_desc_xdma(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
              const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
              uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[8192];
  asm volatile("" ::: "v127");
  desc_xpose_body<2, Md5Hasher<true>, 0, 1, true>(base, offs, lens, order, n, out, img);
}

// LINES: XDMA for batches whose chunks mostly do not start on a 128-B line
// (device-resident chunks packed at 16 B): waves holding such a chunk load
// whole lines, each once (kShift), instead of chunk-relative stages that
// straddle two lines (1.29x the payload from HBM under XDMA).  The second
// line of registers costs occupancy (3 waves per SIMD instead of 4), so
// line-aligned batches keep XDMA: md5hip_plan_desc_at chooses.
__global__ void __launch_bounds__(64)
md5_desc_lines(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
               const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
               uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[8192];
  desc_xpose_body<2, Md5Hasher<true>, 0, 1, true, true>(base, offs, lens, order, n, out, img);
}

__global__ void __launch_bounds__(64)
md5_desc_hybrid(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
                uint4* __restrict__ out, uint32_t nlong) {
  __shared__ __attribute__((aligned(16))) uint8_t img[8192];
  desc_xpose_body<2, Md5Hasher<true>, kHybridLongBlocks, 1, true>(base, offs, lens, order, n, out,
                                                                  img, nlong);   // else xdma
}

// ---------------------------------------------------------------------------
// Pre-summed schedule ("fed" chains).  The same 64 steps with the per-step
// addend W[j] = M[kMsgIdx[j]] + K[j] supplied by someone else (md5_w below,
// in another wave), so a step is 4 VALU -- v_bitop3, v_add3 (w + W + f),
// v_alignbit, v_add -- instead of 5: the lone wave that runs a long chunk's
// serial chain is issue-bound, and the fifth op moves to the feeding wave.
// ---------------------------------------------------------------------------
// message word of step j (md5.c:74-139: rounds 1-4 index schedules)
__host__ __device__ constexpr int md5_msg_idx(int j) {
  return j < 16 ? j : j < 32 ? (1 + 5 * j) & 15 : j < 48 ? (5 + 3 * j) & 15 : (7 * j) & 15;
}
// step j's T constant (the RFC 1321 table, as in compress above)
__device__ constexpr uint32_t kMd5K[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au, 0xa8304613u,
    0xfd469501u, 0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu, 0x6b901122u, 0xfd987193u,
    0xa679438eu, 0x49b40821u, 0xf61e2562u, 0xc040b340u, 0x265e5a51u, 0xe9b6c7aau, 0xd62f105du,
    0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u, 0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu,
    0xa9e3e905u, 0xfcefa3f8u, 0x676f02d9u, 0x8d2a4c8au, 0xfffa3942u, 0x8771f681u, 0x6d9d6122u,
    0xfde5380cu, 0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u, 0x289b7ec6u, 0xeaa127fau,
    0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u, 0xf4292244u,
    0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u, 0xffeff47du, 0x85845dd1u,
    0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u, 0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu,
    0xeb86d391u};

// The 64 addends of one block, 4 per uint4 in step order: q[j >> 2] lane j & 3.
__device__ __forceinline__ void md5_w(const uint4 (&m)[4], uint4 (&q)[16]) {
  auto M = [&](int i) __attribute__((always_inline)) -> uint32_t {
    const uint4& v = m[i >> 2];
    return (i & 3) == 0 ? v.x : (i & 3) == 1 ? v.y : (i & 3) == 2 ? v.z : v.w;
  };
#pragma unroll
  for (int t = 0; t < 16; ++t)
    q[t] = make_uint4(M(md5_msg_idx(4 * t)) + kMd5K[4 * t], M(md5_msg_idx(4 * t + 1)) + kMd5K[4 * t + 1],
                      M(md5_msg_idx(4 * t + 2)) + kMd5K[4 * t + 2],
                      M(md5_msg_idx(4 * t + 3)) + kMd5K[4 * t + 3]);
}

#define MD5HIP_FSTEP(F, w, x, y, z, W, s) w = x + rotl(w + (W) + F(x, y, z), s)

// Steps 4*T0 .. 4*T1-1 of one block from its pre-summed addends (md5_w).  A
// quad of steps leaves the roles (a, b, c, d) where it found them, so a block
// can be split at any quad (the fed chain wave passes a barrier mid-block).
template <int T0, int T1>
__device__ __forceinline__ void fed_steps(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d,
                                          const uint4 (&q)[16]) {
#pragma unroll
  for (int t = T0; t < T1; ++t) {
    const uint4 v = q[t];
    if (t < 4) {
      MD5HIP_FSTEP(f1, a, b, c, d, v.x, 7);
      MD5HIP_FSTEP(f1, d, a, b, c, v.y, 12);
      MD5HIP_FSTEP(f1, c, d, a, b, v.z, 17);
      MD5HIP_FSTEP(f1, b, c, d, a, v.w, 22);
    } else if (t < 8) {
      MD5HIP_FSTEP(f2, a, b, c, d, v.x, 5);
      MD5HIP_FSTEP(f2, d, a, b, c, v.y, 9);
      MD5HIP_FSTEP(f2, c, d, a, b, v.z, 14);
      MD5HIP_FSTEP(f2, b, c, d, a, v.w, 20);
    } else if (t < 12) {
      MD5HIP_FSTEP(f3, a, b, c, d, v.x, 4);
      MD5HIP_FSTEP(f3, d, a, b, c, v.y, 11);
      MD5HIP_FSTEP(f3, c, d, a, b, v.z, 16);
      MD5HIP_FSTEP(f3, b, c, d, a, v.w, 23);
    } else {
      MD5HIP_FSTEP(f4, a, b, c, d, v.x, 6);
      MD5HIP_FSTEP(f4, d, a, b, c, v.y, 10);
      MD5HIP_FSTEP(f4, c, d, a, b, v.z, 15);
      MD5HIP_FSTEP(f4, b, c, d, a, v.w, 21);
    }
  }
}
#undef MD5HIP_FSTEP

// One block from its 64 pre-summed addends: MD5Transform, md5.c:63-146.
__device__ __forceinline__ void compress_fed(State& st, const uint4 (&q)[16]) {
  uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
  fed_steps<0, 16>(a, b, c, d, q);
  st.a += a;  // feed-forward, md5.c:142-145
  st.b += b;
  st.c += c;
  st.d += d;
}

// ---------------------------------------------------------------------------
// Fed chains (HYBRID's long groups, two waves each).  A lone wave running 64
// long chunks' serial chains is bound by its own VALU issue: ~20 cycles per
// step for 5 VALU (the off-chain a + M + K included; profiles/
// r01_chain_probe.json).  Here a second wave of the workgroup -- the feeder,
// on another SIMD -- streams the same 64 chunks lane-direct, forms each
// block's 64 addends M[g(j)] + K[j] (md5_w) and hands them over through LDS
// tables of [16 quads][64 lanes] x 16 B (both sides conflict-free); the chain
// wave reads a block's addends with 16 ds_read_b128 and runs 4 VALU per step
// (compress_fed).
//
// NT = 2 tables, one s_barrier per block (both waves execute 1 + bmax):
//   chain : X_k | read W(k+1) from T[(k+1)&1] | block k from registers
//   feeder: X_k | write W(k+2) into T[k&1]
// At X_k the chain's reads of W(k) (from T[k&1], issued in iteration k-1)
// have returned and the feeder's W(k+1) is written, so each side has a whole
// block of slack.  NT = 1 table (16 KiB: a 2-wave workgroup then needs no more
// LDS than two XDMA waves), two s_barriers per block (2 + 2 * bmax):
//   chain : B_k | read W(k+1) | steps 0-15 of block k | A_k | steps 16-63
//   feeder: B_k | A_k | write W(k+2) (under the chain's steps 16-63)  The barrier is bare (s_waitcnt lgkmcnt(0); s_barrier): a
// workgroup fence would also drain the feeder's global-load ring.  Lanes past
// their own last block keep computing on whatever the feeder clamped to and
// discard the result, so no branch ever skips a barrier.
// kFeedOff (diagnostics): the feeder only keeps the barriers (digests wrong).
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lds_handoff() {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
}
// the same, pinning the chain state: steps cannot move across it
__device__ __forceinline__ void lds_handoff(uint32_t& a, uint32_t& b, uint32_t& c, uint32_t& d) {
  asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) :: "memory");
}

constexpr uint32_t kFedTable = 16 * 64 * 16;     // one block's addends, 16 KiB

// kDigest = false (MD5Update on contexts): the chain starts from st0 and the
// state after the lane's nfull blocks is returned, with no padding or store.
// kAbs: off is an absolute address (base unused; offsetting a null base would
// be undefined), taken as a global pointer so the feeder's loads stay global.
template <int D, int NT, bool kFeedOff = false, bool kDigest = true, bool kAbs = false>
__device__ __forceinline__ State fed_long_group(const uint8_t* __restrict__ base, uint4* __restrict__ out,
                                                uint8_t* lds, bool feeder, uint32_t nfull,
                                                uint32_t bmax, uint64_t off, uint32_t len,
                                                uint64_t c, bool live, State st0 = initial_state()) {
  static_assert(D % 2 == 0, "paired refill");
  auto at = [&](uint64_t o) __attribute__((always_inline)) -> const uint8_t* {
    if constexpr (kAbs)
      return (const uint8_t*)(const __attribute__((address_space(1))) uint8_t*)(uintptr_t)o;
    else
      return base + o;
  };
  const uint8_t* chunk = at(off);
  const uint32_t lane = threadIdx.x & 63u;
  auto tab = [&](uint32_t k) __attribute__((always_inline)) {
    return reinterpret_cast<uint4(*)[64]>(lds + (NT == 2 ? (k & 1u) * kFedTable : 0u));
  };
  __builtin_amdgcn_s_setprio(3);
  if (feeder) {
    // lanes without a whole block stream the wave's longest chunk (in bounds)
    // (base + offset keeps the loads global: a flat load would also count in
    // lgkmcnt, and every hand-over would drain the ring)
    const uint32_t mlane = __builtin_ctzll(__ballot(nfull == bmax));
    const uint32_t lo = (uint32_t)__shfl((int)(uint32_t)off, (int)mlane, 64);
    const uint32_t hi = (uint32_t)__shfl((int)(uint32_t)(off >> 32), (int)mlane, 64);
    const uint4* p = reinterpret_cast<const uint4*>(at(nfull ? off : ((uint64_t)hi << 32) | lo));
    const uint32_t lastb = (nfull ? nfull : bmax) - 1u;
    uint4 R[D][4];
    if constexpr (!kFeedOff) {
#pragma unroll
      for (int j = 0; j < D; ++j) load_block(R[j], p + 4 * min((uint32_t)j, lastb));
    }
    // W(k) into T[k&1] from ring slot k % D; odd slots refill their pair
    // (blocks k-1+D, k+D: one whole 128-B line when the chunk is line-aligned)
    auto put = [&](uint32_t k, int slot) __attribute__((always_inline)) {
      if constexpr (!kFeedOff) {
        uint4 q[16];
        md5_w(R[slot], q);
        uint4 (*t)[64] = tab(k);
#pragma unroll
        for (int i = 0; i < 16; ++i) t[i][lane] = q[i];
        if (slot & 1) {
          load_block(R[slot - 1], p + 4 * min(k - 1 + D, lastb));
          load_block(R[slot], p + 4 * min(k + D, lastb));
        }
      }
    };
    put(0, 0);
    if constexpr (NT == 1) {
      lds_handoff();                             // B_init: W(0) in
      lds_handoff();                             // A_init: W(0) read
    }
    put(1, 1);
    lds_handoff();                               // X_init / B_0: W(1) in
    for (uint32_t k0 = 0; k0 < bmax; k0 += D) {
#pragma unroll
      for (int j = 0; j < D; ++j) {
        const uint32_t k = k0 + j;
        if (k < bmax) {                          // wave-uniform
          if constexpr (NT == 1) lds_handoff();  // A_k
          else lds_handoff();                    // X_k
          if (k + 2 < bmax) put(k + 2, (j + 2) % D);
          if constexpr (NT == 1) {
            if (k + 1 < bmax) lds_handoff();     // B_{k+1}
          }
        }
      }
    }
    return st0;
  }
  State st = st0;
  uint4 q[2][16];                                // W(k) and W(k+1), alternating
  lds_handoff();                                 // X_init / B_init
#pragma unroll
  for (int i = 0; i < 16; ++i) q[0][i] = tab(0)[i][lane];
  if constexpr (NT == 1) lds_handoff();          // A_init
  auto blk = [&](uint32_t k, uint4 (&cur)[16], uint4 (&nxt)[16]) __attribute__((always_inline)) {
    uint32_t a = st.a, b = st.b, cc = st.c, d = st.d;
    lds_handoff(a, b, cc, d);                    // X_k / B_k
    uint4 (*t)[64] = tab(k + 1);
#pragma unroll
    for (int i = 0; i < 16; ++i) nxt[i] = t[i][lane];
    __builtin_amdgcn_sched_barrier(0);           // all 16 reads out before the steps
    if constexpr (NT == 1) {
      fed_steps<0, 4>(a, b, cc, d, cur);
      lds_handoff(a, b, cc, d);                  // A_k: the reads of W(k+1) are in
      fed_steps<4, 16>(a, b, cc, d, cur);
    } else {
      fed_steps<0, 16>(a, b, cc, d, cur);
    }
    const bool act = k < nfull;
    st.a = act ? st.a + a : st.a;
    st.b = act ? st.b + b : st.b;
    st.c = act ? st.c + cc : st.c;
    st.d = act ? st.d + d : st.d;
  };
  for (uint32_t k = 0; k < bmax; k += 2) {
    blk(k, q[0], q[1]);
    if (k + 1 < bmax) blk(k + 1, q[1], q[0]);    // wave-uniform
  }
  if constexpr (kDigest) {
    if (live) {
      Md5Hasher<true> h;
      h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
      h.store(out, c, st);
    }
  }
  return st;
}

// Small batches as fed pairs ("FED", round 3): one 2-wave workgroup per
// 64-chunk group.  A netcache vector (16-16,384 blocks) is at most one group
// per CU, each wave nearly alone on its SIMD, and the launch lasts one
// chunk's serial chain -- bound by the chain wave's own VALU issue, ~4.3
// cycles per instruction whatever the opcode (profiles/r03r/chain_mix.json).
// The feeder wave (another SIMD, idle otherwise) forms every step's
// M[g(j)] + K[j], so the chain runs 4 VALU per step instead of 5: 147 ->
// 138 us for 64-4,096 x 16 KiB, 41 -> 38.6 us at 4 KiB
// (profiles/r03q/small_fed_*.json).  A group holding a chunk start that is
// not 16-B aligned, or no chunk of two whole blocks, runs LANE's lane-direct
// body on wave 0 instead.
// kImplicit: chunk i at base + i * stride, `flen` bytes (the fixed-length
// API's small batches).
constexpr uint32_t kFedMinBlocks = 2;

template <bool kImplicit>
__global__ void __launch_bounds__(128)
md5_desc_fed(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
             const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
             uint64_t stride, uint32_t flen, uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kFedTable];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const DescArrays src{offs, lens, order};
  const uint64_t first = (uint64_t)blockIdx.x * 64u;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t i = first + lane;
  const bool live = i < n;
  const uint64_t c = kImplicit ? (live ? i : first) : src.index(live ? i : first);
  const uint64_t off = kImplicit ? c * stride : src.off(c);
  const uint32_t len = live ? (kImplicit ? flen : src.len(c)) : 0u;
  const uint32_t nfull = len >> 6;
  const uint32_t bmax = wave_max(nfull);
  const bool unaligned = __ballot(live && ((((uintptr_t)base + off) & 15u) != 0)) != 0;
  if (bmax >= kFedMinBlocks && !unaligned) {     // wave-uniform, the same in both waves
    fed_long_group<4, 2>(base, out, lds, wave == 1, nfull, bmax, off, len, c, live);
    return;
  }
  if (wave != 0 || !live) return;
  Md5Hasher<true> h;
  typename Md5Hasher<true>::State st = h.init();
  lane_range<Md5Hasher<true>, 8>(h, st, base + off, len);
  h.store(out, c, st);
}

// ---------------------------------------------------------------------------
// Descriptor batch, LPT-scheduled ("BALANCED"): a persistent grid of ONE wave
// per SIMD (4-wave workgroups holding more than half a CU's LDS, so each CU
// runs exactly one) pulls 64-chunk groups in longest-first order from a
// device counter: list scheduling of the longest-processing-time order on
// 4 x CUs machines.  For a mixed batch holding several waves of work per SIMD
// (coalesced C3 submissions), the hardware's placement -- all waves resident
// at once, ~5 per SIMD, a strided slice of the order on each -- leaves SIMDs
// loaded unevenly: 1 MiB chains ran 2x their solo time sharing a SIMD and
// SIMDs went idle from 54 % of the launch on (scripts/c3_trace_x.py, deleted in 4de68d0,
// profiles/r02_c3_trace.json).  Here every SIMD takes the next-longest group
// whenever its wave frees up.  ctr[0] hands out groups, ctr[1] counts waves
// done; the last wave out resets both, so a counter serves the next launch
// on its stream (md5_kernels.hip keeps one per device and stream).
// ---------------------------------------------------------------------------
// WPB waves per workgroup (one per SIMD at 4, two at 8), each with NB 8 KiB
// LDS-DMA images; the workgroup asks for more than half the CU's LDS, so a
// CU runs exactly one.
template <int WPB, int NB = 1>
struct BalancedCfg {
  static constexpr uint32_t kWave = NB * 8192u;
  // the images start kImgPad bytes in: a DMA whose instruction offset
  // carries the stage step (desc_xpose_group, NB = 2) takes M0 = image -
  // up to 512 B
  static constexpr uint32_t kImgPad = 512u;
  static constexpr uint32_t kLds = WPB * kWave + kImgPad > 81920u ? WPB * kWave + kImgPad : 81920u + 16384u;
  static_assert(WPB * kWave + kImgPad <= 160u * 1024u, "LDS per CU");
};

// The persistent body: each wave takes the next 64-chunk group (longest
// first) from ctr[0] until none is left; ctr[2] counts waves done, and the
// last one out resets the counters for the next launch on the stream.  (Two
// waves per SIMD, with or without split long / short queues at different
// s_setprio, measured slower: a 1 MiB chain sharing its SIMD runs at half
// speed, profiles/r02_c3_balanced_ab.json, r04v/balanced_2wps_ab.json.)
// Returns the number of groups this wave took.
template <int WPB, int NB, int CP = 2, uint32_t kLong = 0>
__device__ __forceinline__ uint32_t balanced_body(const uint8_t* __restrict__ base,
                                                  const uint64_t* __restrict__ offs,
                                                  const uint32_t* __restrict__ lens,
                                                  const uint32_t* __restrict__ order, uint64_t n,
                                                  uint4* __restrict__ out, uint32_t* __restrict__ ctr,
                                                  uint8_t* lds) {
  Md5Hasher<true> h;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + BalancedCfg<WPB, NB>::kImgPad + wave * BalancedCfg<WPB, NB>::kWave;
  const uint64_t ngroups = (n + 63) / 64;
  const DescArrays src{offs, lens, order};
  uint32_t taken = 0;
  for (;;) {
    uint32_t t = 0;
    if (lane == 0) t = atomicAdd(&ctr[0], 1u);
    t = __builtin_amdgcn_readfirstlane((uint32_t)__shfl((int)t, 0, 64));
    if ((uint64_t)t >= ngroups) break;
    ++taken;
    desc_xpose_group<CP, Md5Hasher<true>, kLong, 1, false, true, true, DescArrays, true, NB>(
        h, base, src, n, (uint64_t)t * 64u, out, img, 0xFFFFFFFFu);   // kLong: every long group lane-direct
  }
  if (lane == 0) {
    const uint32_t total = gridDim.x * (blockDim.x >> 6);
    if (atomicAdd(&ctr[2], 1u) == total - 1u) {     // every wave has made its last grab
      atomicExch(&ctr[0], 0u);
      atomicExch(&ctr[1], 0u);
      atomicExch(&ctr[2], 0u);
    }
  }
  return taken;
}

// the product's shape (profiles/r02_c3_balanced_ab.json,
// r02_c3_wide_ab.json, r02_c3_cache_policy_ab.json): one wave per SIMD, two
// 8 KiB images of 128-B stages (round 4, below), one queue, the DEFAULT cache policy for any
// group with a chunk off the 128-B line (nt only for line-aligned groups,
// as every LDS-DMA loader here).  A C3 chunk
// starts 16-B aligned, so each 128-B stage straddles two lines and shares one
// with the next stage; with `nt` loads (the C2 kernel's policy, where chunks
// are line-aligned) that line left L2 before the next stage came, and HBM
// bytes ran 1.21-1.7x the payload, capping the loads alone at 3.9 TB/s.  The
// default policy keeps it: 1.005x, the same kernel 22.1 -> 16.1-16.7 ms on
// five coalesced batches.  Wider stages (W x 128 B per visit), two buffers
// filled the round-2 way (DMA after the reads), 8 waves per CU and split
// long/short queues measured no better (their code is in git history,
// profiles/r02_c3_wide_ab.json, r02_c3_balanced_ab.json).
constexpr int kBalancedWaves = 4;
// two images: the lone wave's next DMA issued under its row reads, the LDS
// base set twice per stage (round 4: 0.8-1.7 % faster on 3 and 6 coalesced
// C3 batches, profiles/r04c/balanced_ab.json)
constexpr int kBalancedImages = 2;
constexpr int kBalancedPolicy = 2;   // nt for line-aligned groups only (desc_xpose_group)

template <int WPB, int NB, int CP>
__global__ void __launch_bounds__(64 * WPB) __attribute__((amdgpu_waves_per_eu(1, WPB / 4)))
md5_desc_balanced_t(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                    const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
                    uint4* __restrict__ out, uint32_t* __restrict__ ctr) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];   // BalancedCfg<WPB, NB>::kLds
  (void)balanced_body<WPB, NB, CP>(base, offs, lens, order, n, out, ctr, lds_dyn);
}

// ---------------------------------------------------------------------------
// CRC-32 batches (netcache blk_make_crc, blk_io.c:354-430), same loaders.
// ---------------------------------------------------------------------------
// XDMA16: the XPERM16 tables (64 KiB) beside twelve waves' full 8 KiB images
// filled by LDS-DMA (xdma_group, as the MD5 default): no VGPR staging, no
// ds_write, one image read per stage instead of two half-image rounds.  One
// 768-thread workgroup per CU (160 KiB LDS), grid-stride over 64-chunk groups,
// wave-major as crc32_xlane_body.
__global__ void __launch_bounds__(768)
crc32_fixed_xdma16(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                   uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32PermHasher::kLdsBytes + 12 * 8192];
  Crc32PermHasher h;
  h.setup(lds);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + Crc32PermHasher::kLdsBytes + wave * 8192u;
  const uint64_t ngroups = (n + 63) / 64;
  for (uint64_t gi = (uint64_t)wave * gridDim.x + blockIdx.x; gi < ngroups; gi += (uint64_t)gridDim.x * 12u)
    xdma_group<Crc32PermHasher, 2>(h, base, n, len, stride, gi * 64u, out, img);
}

// Descriptor batches with XDMA16's layout: the descriptor loader's per-row
// loads as LDS-DMA into twelve waves' full 8 KiB images beside the tables.
__global__ void __launch_bounds__(768)
crc32_desc_xdma16(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                  const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order,
                  uint64_t n, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32PermHasher::kLdsBytes + 12 * 8192];
  Crc32PermHasher h;
  h.setup(lds);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + Crc32PermHasher::kLdsBytes + wave * 8192u;
  const uint64_t ngroups = (n + 63) / 64;
  for (uint64_t gi = (uint64_t)wave * gridDim.x + blockIdx.x; gi < ngroups; gi += (uint64_t)gridDim.x * 12u)
    desc_xpose_group<2, Crc32PermHasher, 0, 1, false, true, true>(
        h, base, DescArrays{offs, lens, order}, n, gi * 64u, out, img);
}

// fastcrc (blk_io.c:408-424) through the same LDS-DMA loader: each 64-row
// wave group is 32 chunks' head and tail windows (FastWindows), F bytes each,
// so a wave-instruction still reads whole 128-B runs of 8 windows; lane pairs
// XOR their CRCs.  offs == nullptr: fixed-length chunks (k * stride, flen).
__global__ void __launch_bounds__(768)
crc32_fast_xdma16(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                  const uint32_t* __restrict__ lens, uint64_t n, uint64_t stride, uint32_t flen,
                  uint32_t F, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32PermHasher::kLdsBytes + 12 * 8192];
  Crc32PermHasher h;
  h.setup(lds);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + Crc32PermHasher::kLdsBytes + wave * 8192u;
  const FastWindows src{offs, lens, stride, flen, F};
  const uint64_t rows = 2 * n;
  const uint64_t ngroups = (rows + 63) / 64;
  for (uint64_t gi = (uint64_t)wave * gridDim.x + blockIdx.x; gi < ngroups; gi += (uint64_t)gridDim.x * 12u)
    desc_xpose_group<2, Crc32PermHasher, 0, 1, false, true, true, FastWindows>(h, base, src, rows,
                                                                               gi * 64u, out, img);
}

// fastcrc with F = 64 or 128 (the netcache harness runs 128): every window
// is one or two whole 64-B blocks, so a group of 64 windows is one short
// load round trip plus a few hundred VALU -- latency, not bandwidth, bound
// it in crc32_fast_xdma16 (one group in flight per wave).  Here each lane
// loads its own window straight into VGPRs (no LDS image: the 64 KiB of
// tables leave room for 16 waves per CU) and the NEXT group's windows are
// loaded before the current group is hashed, so a load round trip always
// runs under a group's compression.  A group with a window that is not
// exactly F bytes at a 16-B-aligned address (a chunk of <= F bytes, a
// ragged tail window) is hashed lane-direct (lane_range) with nothing in
// flight beside it.  Persistent: one 1024-thread workgroup per CU, groups
// wave-major, grid-stride.
// D: window groups in flight per wave (D-1 loaded ahead of the one hashed).
// kPairHalves: a 128-B window's two 64-B halves are requested in alternating
// instructions (bytes 0, 64, 16, 80, ...), so the second half of a line
// reaches L2 while the first half's fill is still pending there; loaded as
// two runs of four (0..48, then 64..112), 15 % of second halves found their
// line already evicted and fetched it again.
template <int D, bool kPairHalves = true>
__device__ __forceinline__ void fast_pipe_body(const uint8_t* __restrict__ base,
                                               const uint64_t* __restrict__ offs,
                                               const uint32_t* __restrict__ lens, uint64_t n,
                                               uint64_t stride, uint32_t flen, uint32_t F,
                                               uint32_t* __restrict__ out, uint8_t* lds) {
  Crc32PermHasher h;
  h.setup(lds);
  const FastWindows src{offs, lens, stride, flen, F};
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t rows = 2 * n;
  const uint64_t ngroups = (rows + 63) / 64;
  const uint64_t step = (uint64_t)gridDim.x * (blockDim.x >> 6);
  const uint32_t nb = F >> 6;                             // 1 or 2 blocks per window
  struct Win {
    const uint8_t* p;
    uint32_t len;
    bool live;
    bool pipe;                                            // wave-uniform
  };
  auto locate = [&](uint64_t gi) __attribute__((always_inline)) {
    Win w;
    const uint64_t c = gi * 64u + lane;
    w.live = c < rows;
    w.len = w.live ? src.len(c) : 0u;
    w.p = base + src.off(w.live ? c : gi * 64u);         // dead lanes read a live row
    const bool simple = !w.live || (w.len == F && ((uintptr_t)w.p & 15u) == 0);
    w.pipe = __ballot(!simple) == 0;
    return w;
  };
  auto fetch = [&](const Win& w, uint4 (&W)[2][4]) __attribute__((always_inline)) {
    const uint4* q = reinterpret_cast<const uint4*>(w.p);
    if (kPairHalves && nb == 2) {
#pragma unroll
      for (int k = 0; k < 4; ++k) {      // the barriers keep hipcc from sorting by offset
        W[0][k] = ld16(q + k);
        __builtin_amdgcn_sched_barrier(0);
        W[1][k] = ld16(q + 4 + k);
        __builtin_amdgcn_sched_barrier(0);
      }
    } else {
      load_block(W[0], q);
      if (nb == 2) load_block(W[1], q + 4);
    }
  };
  auto hash = [&](const Win& w, uint64_t gi, uint4 (&W)[2][4]) __attribute__((always_inline)) {
    typename Crc32PermHasher::State st = h.init();
    if (w.pipe) {
      h.block(st, W[0]);
      if (nb == 2) h.block(st, W[1]);
      h.finish(st, w.p, 0u, F);
    } else if (w.live) {
      lane_range<Crc32PermHasher, 2>(h, st, w.p, w.len);
    }
    if (w.live) emit<FastWindows>(h, out, gi * 64u + lane, st);
  };
  uint64_t g0 = (uint64_t)wave * gridDim.x + blockIdx.x;
  if (g0 >= ngroups) return;
  // a ring of D window buffers, indices fixed at compile time (unrolled)
  uint4 buf[D][2][4];
  Win win[D];
#pragma unroll
  for (int j = 0; j < D - 1; ++j) {
    const uint64_t g = g0 + (uint64_t)j * step;
    win[j] = Win{};
    if (g < ngroups) {
      win[j] = locate(g);
      if (win[j].pipe) fetch(win[j], buf[j]);
    }
  }
  for (;;) {
#pragma unroll
    for (int j = 0; j < D; ++j) {
      constexpr int kD = D;
      const int pj = (j + kD - 1) % kD;                 // the slot freed one group ago
      const uint64_t gp = g0 + (uint64_t)(j + kD - 1) * step;
      win[pj] = Win{};
      if (gp < ngroups) {
        win[pj] = locate(gp);
        if (win[pj].pipe) fetch(win[pj], buf[pj]);
      }
      const uint64_t g = g0 + (uint64_t)j * step;
      if (g < ngroups) hash(win[j], g, buf[j]);
    }
    g0 += (uint64_t)D * step;
    if (g0 >= ngroups) break;
  }
}

__global__ void __launch_bounds__(1024)
crc32_fast_pipe(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                const uint32_t* __restrict__ lens, uint64_t n, uint64_t stride, uint32_t flen,
                uint32_t F, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32PermHasher::kLdsBytes];
  fast_pipe_body<2>(base, offs, lens, n, stride, flen, F, out, lds);
}

// ---------------------------------------------------------------------------
// CRC-32 of small batches, one wave per chunk ("split", round 3).  Unlike
// MD5, CRC-32 is linear, so one chunk need not be one serial chain: the
// chunk is cut into 256-B segments, segment s on lane (s mod 64) of pass
// s / 64, each lane runs its own register over its segment (the first
// segment from ~0, the others from 0), and the registers are combined with
// crc32_combine's zero-byte operators (hashers.h CrcShift): a 6-level tree
// over the wave's lanes, each level advancing the left half through the
// right half's bytes (256 * 2^l), then pass after pass through 16 KiB.  The
// segments are counted from the END of the chunk, so every segment but the
// first is exactly 256 B (the first holds the L mod 256 leftover bytes, or a
// whole 256) and every shift is one of seven constants.  A lane's chain is 64
// dependent table steps instead of the chunk's 4,096 -- the netcache call
// site's vector of 16-1,024 blocks (blk_make_crc, blk_io.c:354-430) is a few
// microseconds of work instead of one 16 KiB chain.  256-thread workgroups
// (4 chunks) share one copy of the 64 KiB perm tables.
// ---------------------------------------------------------------------------
// The CRC-32 (crc32.c: ~0 in, ~ out) of [m, m + L) by the whole wave; the
// result is valid in lane 63.
__device__ __forceinline__ uint32_t split_crc_msg(Crc32PermHasher& h, const uint8_t* m, uint32_t L,
                                                  uint32_t lane) {
  const uint32_t nseg = (uint32_t)(((uint64_t)L + 255u) >> 8);
  const uint32_t r0 = nseg ? L - ((nseg - 1u) << 8) : 0u;          // first segment: 1..256 B
  const uint32_t npass = (nseg + 63u) >> 6;
  uint32_t acc = 0;
  for (uint32_t p = 0; p < npass; ++p) {
    // passes right-aligned: the first pass's low lanes hold no segment
    const int64_t s = (int64_t)nseg - 64 * (int64_t)(npass - p) + (int64_t)lane;
    uint32_t reg = 0;
    if (s >= 0) {
      const uint64_t start = s == 0 ? 0u : (uint64_t)r0 + ((uint64_t)(s - 1) << 8);
      typename Crc32PermHasher::State st{s == 0 ? 0xFFFFFFFFu : 0u};
      lane_range<Crc32PermHasher, 2>(h, st, m + start, s == 0 ? r0 : 256u);
      reg = ~st.c;                               // the raw register (finish complements)
    }
    // lane j ends holding segments [j - 2^(l+1) + 1, j] when j = 2^(l+1) - 1 mod 2^(l+1)
    auto level = [&](auto lv) __attribute__((always_inline)) {
      constexpr int l = decltype(lv)::value;
      const uint32_t left = (uint32_t)__shfl_up((int)reg, 1u << l, 64);
      const uint32_t sh = crc_shift<l>(left);
      if ((lane & ((2u << l) - 1u)) == (2u << l) - 1u) reg ^= sh;
    };
    level(std::integral_constant<int, 0>{});
    level(std::integral_constant<int, 1>{});
    level(std::integral_constant<int, 2>{});
    level(std::integral_constant<int, 3>{});
    level(std::integral_constant<int, 4>{});
    level(std::integral_constant<int, 5>{});
    acc = crc_shift<6>(acc) ^ reg;               // lane 63: all passes so far
  }
  return L ? ~acc : 0u;                          // empty: crc32.c returns ~~0 = 0
}

// F > 0: blk_make_crc's fastcrc mode, CRC(first F bytes) ^ CRC(last F bytes)
// for chunks longer than F (blk_io.c:408-424), each window split as above.
template <bool kImplicit>
__global__ void __launch_bounds__(256)
crc32_split(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
            const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
            uint64_t stride, uint32_t flen, uint32_t F, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32PermHasher::kLdsBytes];
  Crc32PermHasher h;
  h.setup(lds);                                  // all threads, before any exit
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint32_t wpb = blockDim.x >> 6;
  for (uint64_t q = (uint64_t)blockIdx.x * wpb + wave; q < n; q += (uint64_t)gridDim.x * wpb) {
    const uint64_t c = (!kImplicit && order) ? (uint64_t)order[q] : q;
    const uint8_t* m = base + (kImplicit ? c * stride : offs[c]);
    const uint32_t L = kImplicit ? flen : lens[c];
    uint32_t crc;
    if (F && L > F)
      crc = split_crc_msg(h, m, F, lane) ^ split_crc_msg(h, m + (L - F), F, lane);
    else
      crc = split_crc_msg(h, m, L, lane);
    if (lane == 63u) out[c] = crc;
  }
}

template <bool kImplicit>
__global__ void __launch_bounds__(256)
crc32_desc(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
           const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
           uint64_t stride, uint32_t flen, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t tabs[Crc32Hasher::kLdsBytes];
  desc_body<kImplicit, Crc32Hasher, true, 4>(base, offs, lens, order, n, stride, flen, out, tabs);
}

// ---------------------------------------------------------------------------
// MD5Update / MD5Final on caller-owned contexts (md5.c:169-265), one lane per
// context: the reference's streaming state machine, batched.  The context is
// md5.h:33-38's 88-byte struct MD5Context { u32 buf[4]; u32 bits[2]; u8 in[64]; }
// in device memory, updated byte for byte as md5.c leaves it:
//   bits  += len << 3 with the carry into bits[1] (md5.c:177-182);
//   t = pending bytes; if t and len < 64 - t: in[t .. t+len) = data, done
//   (md5.c:186-193); else the pending block is completed and compressed, then
//   every whole 64-B block of data (md5.c:204-210); in[] is left holding the
//   tail in its first bytes and, past them, the last block compressed (the
//   memcpy at md5.c:214 writes only the tail), or its old bytes if none was.
//   Final: 0x80, zeros, bit count, one or two compressions, digest = buf, the
//   whole context zeroed (md5.c:221-265).
// Data may sit at any byte alignment (the reference takes any void*).
// ---------------------------------------------------------------------------
struct CtxWords {
  uint32_t w[22];     // buf[0..3], bits[0..1], in[] as 16 little-endian words
};

__device__ __forceinline__ void ctx_load(CtxWords& c, const uint32_t* p) {
#pragma unroll
  for (int k = 0; k < 22; ++k) c.w[k] = p[k];
}
__device__ __forceinline__ void ctx_store(uint32_t* p, const CtxWords& c) {
#pragma unroll
  for (int k = 0; k < 22; ++k) p[k] = c.w[k];
}
// The whole 64-B blocks of an update go through the descriptor loader
// (desc_xpose_group: LDS-DMA 128-B stages of 8 contexts' data per
// wave-instruction, per-lane trip counts), each lane starting from its own
// context's state instead of MD5Init's, and nothing appended after them:
// CtxHasher's finish is empty and its store hands the state back.  LaneSpan
// is the lane's own (absolute address, length) -- the bulk of its update.
struct CtxHasher : Md5Hasher<true> {
  State s0, res;
  __device__ __forceinline__ State init() { return s0; }
  __device__ __forceinline__ void finish(State&, const uint8_t*, uint32_t, uint64_t) {}
  __device__ __forceinline__ void store(Out*, uint64_t, const State& st) { res = st; }
};
struct LaneSpan {
  uint64_t addr;
  uint32_t n;
  static constexpr bool kPairXor = false;
  static constexpr bool kAbs = true;
  __device__ __forceinline__ uint64_t index(uint64_t i) const { return i; }
  __device__ __forceinline__ uint64_t off(uint64_t) const { return addr; }
  __device__ __forceinline__ uint32_t len(uint64_t) const { return n; }
};

// One wave per 64 contexts (one-wave workgroups, the loader's 8 KiB image);
// 125 VGPRs hold it at 4 waves per SIMD, as md5_desc_xdma's clobber does.
// The body, per wave.  kFed: the whole blocks run as the
// chain wave of a fed pair (md5_update_ctx_fed, bmax = the group's most
// blocks); otherwise through the descriptor loader into `img` (8 KiB).
template <bool kFed>
__device__ __forceinline__ void update_ctx_body(uint32_t* __restrict__ ctxs,
                                                const uint64_t* __restrict__ ptrs,
                                                const uint32_t* __restrict__ lens, uint64_t n,
                                                uint8_t* img, uint32_t bmax) {
  const uint64_t first = (uint64_t)blockIdx.x * 64u;
  const uint64_t i = first + (threadIdx.x & 63u);
  const bool live = i < n;
  uint32_t* cp = ctxs + 22 * (live ? i : first);
  CtxWords c;
  ctx_load(c, cp);
  const uint32_t len = live ? lens[i] : 0u;
  const uint8_t* data = reinterpret_cast<const uint8_t*>(live ? ptrs[i] : 0ull);
  const uint32_t t0 = c.w[4];
  const uint32_t lo = t0 + (len << 3);                 // md5.c:179-182
  c.w[5] += (lo < t0 ? 1u : 0u) + (len >> 29);
  c.w[4] = lo;
  const uint32_t t = (t0 >> 3) & 63u;
  uint32_t in[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) in[j] = c.w[6 + j];
  const bool append_only = t && len < 64u - t;         // md5.c:189-192: no block completes
  State st{c.w[0], c.w[1], c.w[2], c.w[3]};
  uint32_t pos = 0;                                    // bytes of data consumed
  uint32_t last[16];                                   // the last block compressed
  bool any = false;
  if (append_only) {
    for (uint32_t k = 0; k < len; ++k) {
      const uint32_t p2 = t + k;
      const uint32_t b = data[k];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if ((uint32_t)j == (p2 >> 2)) {
          const uint32_t sh = 8u * (p2 & 3u);
          in[j] = (in[j] & ~(0xFFu << sh)) | (b << sh);
        }
    }
  } else if (t) {                                      // md5.c:194-199: complete the pending block
    const uint32_t need = 64u - t;
#pragma unroll
    for (int j = 0; j < 16; ++j) last[j] = in[j];
    for (uint32_t k = 0; k < need; ++k) {
      const uint32_t p2 = t + k;
      const uint32_t b = data[k];
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if ((uint32_t)j == (p2 >> 2)) {
          const uint32_t sh = 8u * (p2 & 3u);
          last[j] = (last[j] & ~(0xFFu << sh)) | (b << sh);
        }
    }
    compress(st, [&](int q) __attribute__((always_inline)) { return last[q]; });
    pos = need;
    any = true;
  }
  const uint32_t nblk = append_only ? 0u : (len - pos) >> 6;   // md5.c:204-210
  if constexpr (kFed) {
    st = fed_long_group<4, 2, false, false, true>(nullptr, nullptr, img, false, nblk, bmax,
                                            (uint64_t)(uintptr_t)(data + pos), nblk << 6, 0, live, st);
  } else {
    CtxHasher h;
    h.s0 = st;
    h.res = st;
    desc_xpose_group<2, CtxHasher, 0, 1, false, true, true, LaneSpan>(
        h, nullptr, LaneSpan{(uint64_t)(uintptr_t)(data + pos), nblk << 6}, n, first, nullptr, img);
    st = h.res;
  }
  if (!live) return;
  if (append_only) {
#pragma unroll
    for (int j = 0; j < 16; ++j) c.w[6 + j] = in[j];
    ctx_store(cp, c);
    return;
  }
  if (nblk) {                                          // the bytes md5.c leaves in in[] past the tail
    const uint8_t* lb = data + pos + ((uint64_t)(nblk - 1) << 6);
    uint4 w[4];
    if (((uintptr_t)lb & 15u) == 0) load_block(w, reinterpret_cast<const uint4*>(lb));
    else load_block_unaligned(w, lb);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      last[4 * k] = w[k].x; last[4 * k + 1] = w[k].y;
      last[4 * k + 2] = w[k].z; last[4 * k + 3] = w[k].w;
    }
    pos += nblk << 6;
    any = true;
  }
  const uint32_t r = len - pos;                        // md5.c:214: memcpy(in, buf, r)
  uint32_t tw[16];
  load_tail(data + pos, r, tw);
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const uint32_t keep = any ? last[j] : in[j];
    const int nb = (int)r - 4 * j;                     // tail bytes in word j
    const uint32_t m = nb >= 4 ? 0xFFFFFFFFu : nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u);
    c.w[6 + j] = (tw[j] & m) | (keep & ~m);
  }
  c.w[0] = st.a; c.w[1] = st.b; c.w[2] = st.c; c.w[3] = st.d;
  ctx_store(cp, c);
}

__global__ void __launch_bounds__(64)
md5_update_ctx(uint32_t* __restrict__ ctxs, const uint64_t* __restrict__ ptrs,
               const uint32_t* __restrict__ lens, uint64_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t img[8192];
  update_ctx_body<false>(ctxs, ptrs, lens, n, img, 0u);
}

// Few contexts (at most one 64-context group per CU): the launch is one
// update's serial chain, so the whole blocks run as fed pairs (a feeder wave
// forms M + K, as md5_desc_fed).  Both waves work out each lane's span of
// whole blocks from its context and length alone; a group with a span that
// is not 16-B aligned, or without two blocks, runs the loader body on wave 0.
__global__ void __launch_bounds__(128)
md5_update_ctx_fed(uint32_t* __restrict__ ctxs, const uint64_t* __restrict__ ptrs,
                   const uint32_t* __restrict__ lens, uint64_t n) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[2 * kFedTable];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t first = (uint64_t)blockIdx.x * 64u;
  const uint64_t i = first + (threadIdx.x & 63u);
  const bool live = i < n;
  const uint32_t len = live ? lens[i] : 0u;
  const uint8_t* data = reinterpret_cast<const uint8_t*>(live ? ptrs[i] : 0ull);
  const uint32_t t = (ctxs[22 * (live ? i : first) + 4] >> 3) & 63u;   // pending bytes
  const bool append_only = t && len < 64u - t;
  const uint32_t pos = append_only ? 0u : (t ? 64u - t : 0u);
  const uint32_t nblk = append_only ? 0u : (len - pos) >> 6;
  const uint32_t bmax = wave_max(nblk);
  const bool unaligned = __ballot(nblk && ((((uintptr_t)data + pos) & 15u) != 0)) != 0;
  if (bmax < kFedMinBlocks || unaligned) {     // wave-uniform, the same in both waves
    if (wave == 0) update_ctx_body<false>(ctxs, ptrs, lens, n, lds, 0u);
    return;
  }
  if (wave == 1) {
    fed_long_group<4, 2, false, false, true>(nullptr, nullptr, lds, true, nblk, bmax,
                                       (uint64_t)(uintptr_t)(data + pos), nblk << 6, 0, live);
    return;
  }
  update_ctx_body<true>(ctxs, ptrs, lens, n, lds, bmax);
}

__global__ void __launch_bounds__(256)
md5_final_ctx(uint32_t* __restrict__ ctxs, uint64_t n, uint4* __restrict__ digests) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t* cp = ctxs + 22 * i;
  CtxWords c;
  ctx_load(c, cp);
  const uint32_t count = (c.w[4] >> 3) & 63u;          // md5.c:229
  uint32_t w[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {                       // in[0..count), 0x80, zeros (md5.c:233-254)
    const int nb = (int)count - 4 * j;
    const uint32_t m = nb >= 4 ? 0xFFFFFFFFu : nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u);
    w[j] = c.w[6 + j] & m;
    if ((uint32_t)j == (count >> 2)) w[j] |= 0x80u << (8u * (count & 3u));
  }
  State st{c.w[0], c.w[1], c.w[2], c.w[3]};
  if (count >= 56u) {                                  // md5.c:240-249: two blocks
    compress(st, [&](int q) __attribute__((always_inline)) { return w[q]; });
#pragma unroll
    for (int j = 0; j < 14; ++j) w[j] = 0u;
  }
  w[14] = c.w[4];                                      // md5.c:257-259
  w[15] = c.w[5];
  compress(st, [&](int q) __attribute__((always_inline)) { return w[q]; });
  digests[i] = make_uint4(st.a, st.b, st.c, st.d);     // md5.c:262-263
#pragma unroll
  for (int k = 0; k < 22; ++k) c.w[k] = 0u;            // md5.c:264
  ctx_store(cp, c);
}

__global__ void __launch_bounds__(256)
md5_init_ctx(uint32_t* __restrict__ ctxs, uint64_t n) {  // md5.c:153-163 (in[] untouched)
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  uint32_t* cp = ctxs + 22 * i;
  const State s0 = initial_state();
  cp[0] = s0.a; cp[1] = s0.b; cp[2] = s0.c; cp[3] = s0.d;
  cp[4] = 0u; cp[5] = 0u;
}

// ---------------------------------------------------------------------------
// The longest-first order of a descriptor batch on the device (the batcher's
// planner, md5_submit.c): a counting sort whose bucket starts the host took
// from the histogram it keeps while chunks are reserved.  One atomic per
// distinct key per wave (the lanes of one key take consecutive positions),
// and all of a wave's atomics in ONE instruction: the key loop only finds
// each lane's leader and rank (scalar reads and ballots), then the leaders
// add at once and every lane reads its leader's base.  Waiting out one
// returning atomic per distinct key instead took 138 us for a 472 K-chunk
// burst of random lengths (~64 round trips per wave, profiles/r04b/
// c3q_breakdown.json).
// ---------------------------------------------------------------------------
__global__ void __launch_bounds__(256)
order_scatter(const uint32_t* __restrict__ lens, uint64_t n, uint32_t kmax,
              uint32_t* __restrict__ next, uint32_t* __restrict__ order) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t k0 = i < n ? (lens[i] >> 6) + 1u : 0u;
  // a key past kmax (lengths the caller's histogram does not cover) would
  // index before next[0]: such a chunk is left out of the order instead
  const bool live = i < n && k0 <= kmax;
  const uint32_t key = live ? k0 : 0u;
  const uint64_t below = (1ull << lane) - 1ull;
  uint32_t leader = 0, rank = 0, count = 0;
  uint64_t todo = __ballot(live);
  while (todo) {                                       // wave-uniform
    const uint32_t ld = (uint32_t)__builtin_ctzll(todo);
    const uint32_t lk = (uint32_t)__builtin_amdgcn_readlane((int)key, (int)ld);
    const uint64_t same = __ballot(live && key == lk);
    if (live && key == lk) {
      leader = ld;
      rank = (uint32_t)__popcll(same & below);
      if (lane == ld) count = (uint32_t)__popcll(same);
    }
    todo &= ~same;
  }
  uint32_t base = 0;
  if (count) base = atomicAdd(&next[kmax - key], count);   // leaders only
  base = (uint32_t)__shfl((int)base, (int)leader, 64);
  if (live) {
    const uint32_t pos = base + rank;
    if (pos < n) order[pos] = (uint32_t)i;             // bound: a torn bucket table stays in range
  }
}

// ---------------------------------------------------------------------------
// Device-side gather for the batcher's zero-copy path: segment k of a slice
// is read from registered (pinned, device-mapped) host memory over PCIe and
// written to its packed place in the slice's HBM buffer.  One workgroup per
// segment (grid-stride); 16-B accesses when both ends are 16-B aligned
// (cache pages are 4 KiB aligned, md5_submit.c packs chunks 128-B aligned),
// bytes otherwise.
// ---------------------------------------------------------------------------
struct GatherSeg {
  uint64_t src, dst;
  uint32_t len, pad;
};

// U: 16-B loads in flight per thread before the stores (PCIe latency).
template <int U>
__global__ void __launch_bounds__(256)
gather_segments(const GatherSeg* __restrict__ segs, uint64_t nseg, uint8_t* __restrict__ dst) {
  for (uint64_t k = blockIdx.x; k < nseg; k += gridDim.x) {
    const GatherSeg g = segs[k];
    const uint8_t* src = reinterpret_cast<const uint8_t*>(g.src);
    uint8_t* d = dst + g.dst;
    uint32_t head = 0;
    if (((g.src | (uintptr_t)d) & 15u) == 0) {
      const uint32_t n16 = g.len >> 4;
      const uint4* s16 = reinterpret_cast<const uint4*>(src);
      uint4* d16 = reinterpret_cast<uint4*>(d);
      uint32_t j = threadIdx.x;
      for (; j + (U - 1) * blockDim.x < n16; j += U * blockDim.x) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = s16[j + u * blockDim.x];
#pragma unroll
        for (int u = 0; u < U; ++u) d16[j + u * blockDim.x] = v[u];
      }
      for (; j < n16; j += blockDim.x) d16[j] = s16[j];
      head = n16 << 4;
    }
    for (uint32_t j = head + threadIdx.x; j < g.len; j += blockDim.x) d[j] = src[j];
  }
}

// ---------------------------------------------------------------------------
// Synthetic data: 32-bit word i of the buffer = mix32(seed, i) (a splitmix64
// finaliser).  tests/gen.py has the numpy mirror.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mix32(uint64_t seed, uint64_t i) {
  uint64_t z = seed + (i + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return (uint32_t)(z ^ (z >> 31));
}

__global__ void __launch_bounds__(256)
fill_synthetic(uint4* __restrict__ dst, uint64_t n16, uint64_t seed) {
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n16; i += stride) {
    const uint64_t w = 4 * i;
    dst[i] = make_uint4(mix32(seed, w), mix32(seed, w + 1), mix32(seed, w + 2), mix32(seed, w + 3));
  }
}

}  // namespace md5hip

