// md5_kernels_ab.h -- kernel variants measured in round 1 and NOT shipped
// (DESIGN.md §4-§5 hold the A/B numbers).  Included only by md5_diag.hip, so
// libmd5hip.so carries none of them; md5diag_variant_* (md5_diag.hip) launch
// them for A/B benches and their parity tests.
//
//   md5_fixed_lds64/128(nt)   LDS-DMA staging, 64/128 B per chunk per stage
//   md5_fixed_xpose1/2(nt)    register-staged transpose (xpose1nt: round-1 default)
//   md5_desc_xpose            descriptor batch, register-staged transpose
//   crc32_fixed_xpose         CRC-32 slicing-by-8 over one shared LDS table set
//   crc32_fixed_lane32/16     CRC-32 lane-private table copies, lane-direct loads
//   crc32_fixed_xlane16/xperm16, crc32_desc_xperm16   16 table copies, half images
//   md5_desc_hybrid_fed       round 2: HYBRID with "fed" chains (a feeder wave
//                             hands each block's M + K addends to the chain wave)
#pragma once
#include "md5_kernels.h"

namespace md5hip {

// ---------------------------------------------------------------------------
// Fixed-length, wave-cooperative LDS-DMA staging (two stage buffers per wave).
//   BB  bytes per chunk per stage (64 = one block, 128 = two blocks = one
//       128-B line per chunk per stage)
// LDS image of one stage: row L (= lane L's chunk) of BB bytes; 16-B slot q of
// row L holds part q ^ g(L), g(L) = (L >> 2) & 3 for BB=64, (L >> 1) & 7 for
// BB=128 -- distinct over every ds_read_b128 lane group (MI355X_MICROARCH §LDS),
// so the row reads are conflict-free.  The swizzle is applied on the SOURCE
// address because the DMA destination is lane-linear.
// Order per stage: wait stage s -> ds_read it into VGPRs -> issue DMA of stage
// s+1 into the other buffer -> compress.  Exactly one stage is in flight when
// the explicit vmcnt(0) guards the next ds_read.
// ---------------------------------------------------------------------------
template <int BB>
__device__ __forceinline__ uint32_t swz(uint32_t row) {
  return BB == 64 ? ((row >> 2) & 3u) : ((row >> 1) & 7u);
}

template <int BB, class H = Md5Hasher<false>, int CP = 0>
__device__ __forceinline__ void fixed_lds_body(const uint8_t* __restrict__ base, uint64_t n,
                                               uint32_t len, uint64_t stride,
                                               typename H::Out* __restrict__ out, uint8_t* lds) {
  H h;
  constexpr int LPC = BB / 16;         // lanes per chunk in one DMA instruction
  constexpr int CPI = 64 / LPC;        // chunks per DMA instruction
  constexpr int NI = 64 / CPI;         // DMA instructions per stage
  constexpr int BPS = BB / 64;         // blocks per stage
  constexpr int STAGE = 64 * BB;       // bytes per stage per wave

  const uint32_t lane = threadIdx.x & 63u;
  const uint32_t wave = threadIdx.x >> 6;
  uint8_t* ring = lds + (size_t)wave * 2 * STAGE;
  const uint64_t wave_first = ((uint64_t)blockIdx.x * blockDim.x) + wave * 64u;
  if (wave_first >= n) return;         // whole wave out of range (wave-uniform)
  const uint64_t last = n - 1;

  const uint8_t* src[NI];
#pragma unroll
  for (int r = 0; r < NI; ++r) {
    const uint32_t row = (uint32_t)r * CPI + lane / LPC;
    const uint32_t q = lane % LPC;
    const uint32_t part = q ^ (swz<BB>(row) & (LPC - 1));
    uint64_t c = wave_first + row;
    c = c > last ? last : c;           // tail lanes re-read the last chunk
    src[r] = base + c * stride + part * 16u;
  }
  const uint32_t nfull = len >> 6;
  const uint32_t nstage = nfull / BPS;   // whole stages; leftovers go direct

  auto issue = [&](uint32_t stg) __attribute__((always_inline)) {
    uint8_t* dst = ring + (stg & 1u) * STAGE;
#pragma unroll
    for (int r = 0; r < NI; ++r)
      __builtin_amdgcn_global_load_lds(src[r] + (size_t)stg * BB, dst + r * 1024, 16, 0, CP);
  };

  typename H::State st = h.init();
  if (nstage) issue(0);
  const uint32_t g = swz<BB>(lane) & (LPC - 1);
  for (uint32_t stg = 0; stg < nstage; ++stg) {
    const uint8_t* row = ring + (stg & 1u) * STAGE + lane * BB;
    // The compiler does not reliably order ds_read after an LDS-DMA into the
    // same bytes (it emitted no wait at all for BB=64), so wait explicitly:
    // exactly one stage is in flight here, so vmcnt(0) costs no overlap.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint4 w[BPS][4];
#pragma unroll
    for (int b = 0; b < BPS; ++b)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const uint32_t q = ((uint32_t)(b * 4 + k)) ^ g;
        w[b][k] = *reinterpret_cast<const uint4*>(row + q * 16u);
      }
    if (stg + 1 < nstage) issue(stg + 1);
#pragma unroll
    for (int b = 0; b < BPS; ++b) h.block(st, w[b]);
  }
  // leftover whole blocks (nfull % BPS), then the tail
  const uint64_t i = wave_first + lane;
  const uint64_t ci = i > last ? last : i;
  const uint8_t* chunk = base + ci * stride;
  for (uint32_t blk = nstage * BPS; blk < nfull; ++blk) {
    uint4 w[4];
    load_block(w, reinterpret_cast<const uint4*>(chunk + ((uint64_t)blk << 6)));
    h.block(st, w);
  }
  h.finish(st, chunk + ((uint64_t)nfull << 6), len & 63u, len);
  if (i <= last) h.store(out, i, st);
}

// ---------------------------------------------------------------------------
// Fixed-length, register-staged transpose ("xpose").
// Each wave-instruction loads 8 chunks x 128 B (8 lanes per 128-B line) with
// buffer_load_dwordx4 -- one wave-uniform buffer descriptor per 64-chunk group,
// a per-(lane, instruction) 32-bit voffset fixed for the whole kernel, and the
// stage offset in the scalar soffset, so the steady state spends no VALU on
// addressing.  Loads run D stages (D x 128 B per chunk) ahead in VGPRs; per
// stage the wave writes its 8 KiB image to LDS (ds_write_b128, conflict-free:
// 8 lanes cover one 128-B row) and each lane reads back its own row
// (ds_read_b128, source-swizzled as in md5_fixed_lds so the 16-lane groups hit
// distinct 16-B slots).  LDS is only a per-wave transpose buffer (8 KiB), so
// occupancy is set by VGPRs, not LDS, and all waits are compiler-counted.
// Requires 64 * stride < 2^31 (checked by the launcher).
// ---------------------------------------------------------------------------
// kPair (D even): the ring is refilled two slots at a time, so a chunk's two
// adjacent 128-B lines are requested back to back (one DRAM row visit for
// 256 B instead of two visits a stage apart).
template <int D, class H = Md5Hasher<false>, int CP = 0, bool kPair = false, bool kPeel = true>
__device__ __forceinline__ void fixed_xpose_group(H& h, const uint8_t* __restrict__ base,
                                                  uint64_t n, uint32_t len, uint64_t stride,
                                                  typename H::Out* __restrict__ out, uint8_t* img,
                                                  uint64_t wave_first) {
  static_assert(!kPair || D % 2 == 0, "paired refill needs an even ring");
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t left = n - wave_first;
  const uint32_t rows = left < 64 ? (uint32_t)left : 64u;
  const __amdgpu_buffer_rsrc_t rsrc = uniform_rsrc(base + wave_first * stride);
  uint32_t voff[8];
#pragma unroll
  for (int r = 0; r < 8; ++r) {
    const uint32_t row = (uint32_t)r * 8u + (lane >> 3);
    const uint32_t rc = row < rows ? row : rows - 1u;          // ragged last wave
    const uint32_t part = (lane & 7u) ^ ((row >> 1) & 7u);       // source swizzle
    voff[r] = rc * (uint32_t)stride + part * 16u;
  }
  const uint32_t g = (lane >> 1) & 7u;
  const uint32_t nfull = len >> 6;
  const uint32_t nstage = nfull >> 1;                 // 128-B stages
  typename H::State st = h.init();

  auto load_stage = [&](u32x4 (&R)[8], uint32_t stg) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
      R[r] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)voff[r], (int)(stg * 128u), CP);
  };
  // refill: 0 = none, 1 = this slot with stage `next`, 2 = this slot and the
  // previous one with stages next and next - 1 (kPair)
  auto consume = [&](u32x4 (&R)[8], uint32_t next, int refill, u32x4 (*Rprev)[8] = nullptr)
      __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
      *reinterpret_cast<u32x4*>(img + r * 1024 + lane * 16) = R[r];
    __builtin_amdgcn_wave_barrier();
    uint4 w[2][4];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(img + lane * 128 + ((q ^ g) * 16));
      w[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
    }
    __builtin_amdgcn_wave_barrier();
    if (refill == 2) load_stage(*Rprev, next - 1);
    if (refill >= 1) load_stage(R, next);             // refill this ring slot
    __builtin_amdgcn_sched_barrier(0);                // keep the refill ahead of the
    h.block(st, w[0]);                                // compression (hipcc sinks it)
    h.block(st, w[1]);
  };

  if (nstage) {
    const uint32_t lasts = nstage - 1;
    u32x4 R[D][8];
#pragma unroll
    for (int j = 0; j < D; ++j) load_stage(R[j], min((uint32_t)j, lasts));
    uint32_t stg = 0;
    if constexpr (D == 1 && kPeel) {
      // the last stage is peeled: no refill past the end (a clamped refill
      // would re-read the last 128 B of every chunk, +0.7 % HBM bytes)
      for (; stg + 1 < nstage; ++stg) consume(R[0], stg + 1, 1);
      consume(R[0], 0, 0);
    } else {                         // (D == 1 without kPeel: the clamped re-read)
      for (; stg + D <= nstage; stg += D) {
#pragma unroll
        for (int j = 0; j < D; ++j) {
          if constexpr (kPair) {
            if (j & 1) consume(R[j], min(stg + j + D, lasts), 2, &R[j - 1]);
            else consume(R[j], 0, 0);
          } else {
            consume(R[j], min(stg + j + D, lasts), 1);
          }
        }
      }
#pragma unroll
      for (int j = 0; j < D - 1; ++j)
        if (stg + j < nstage) consume(R[j], lasts, 0);
    }
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

template <int D, class H = Md5Hasher<false>, int CP = 0, bool kPair = false>
__device__ __forceinline__ void fixed_xpose_body(const uint8_t* __restrict__ base, uint64_t n,
                                                 uint32_t len, uint64_t stride,
                                                 typename H::Out* __restrict__ out, uint8_t* lds,
                                                 uint8_t* hlds = nullptr) {
  H h;
  h.setup(hlds);                     // before any early exit (may barrier)
  // readfirstlane: the wave index must be provably wave-uniform, or hipcc
  // wraps every buffer load in a waterfall loop (cdna_hip_programming.md T20)
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t wave_first = ((uint64_t)blockIdx.x * blockDim.x) + wave * 64u;
  if (wave_first >= n) return;
  fixed_xpose_group<D, H, CP, kPair>(h, base, n, len, stride, out, lds + (size_t)wave * 8192,
                                     wave_first);
}



// Non-template entry points (hipcc mis-handles explicitly instantiated
// __global__ templates that declare extern __shared__).
__global__ void __launch_bounds__(256)
md5_fixed_lds64(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                uint4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  fixed_lds_body<64>(base, n, len, stride, out, lds_dyn);
}

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
md5_fixed_xpose1(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<1>(base, n, len, stride, out, img);
}

__global__ void __launch_bounds__(256)
md5_fixed_xpose2(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<2>(base, n, len, stride, out, img);
}

// Non-temporal ("nt", aux = 2) load policy: every byte is read exactly once,
// so do not let the stream allocate in L2 / Infinity Cache.
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(5)))
md5_fixed_xpose1nt(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                   uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<1, Md5Hasher<false>, 2>(base, n, len, stride, out, img);
}


__global__ void __launch_bounds__(256)
md5_fixed_xpose2nt(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                   uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  fixed_xpose_body<2, Md5Hasher<false>, 2>(base, n, len, stride, out, img);
}

__global__ void __launch_bounds__(256)
md5_fixed_lds128nt(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                   uint4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  fixed_lds_body<128, Md5Hasher<false>, 2>(base, n, len, stride, out, lds_dyn);
}

__global__ void __launch_bounds__(256)
md5_fixed_lds128(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                 uint4* __restrict__ out) {
  extern __shared__ __attribute__((aligned(16))) uint8_t lds_dyn[];
  fixed_lds_body<128>(base, n, len, stride, out, lds_dyn);
}


__global__ void __launch_bounds__(64)
md5_desc_xpose(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
               const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
               uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[8192];
  desc_xpose_body<2>(base, offs, lens, order, n, out, img);
}


__global__ void __launch_bounds__(256)
crc32_fixed_xpose(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                  uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t img[4 * 8192];
  __shared__ __attribute__((aligned(16))) uint8_t tabs[Crc32Hasher::kLdsBytes];
  fixed_xpose_body<1, Crc32Hasher, 2>(base, n, len, stride, out, img, tabs);
}

// Lane-private tables (Crc32LaneHasher): one workgroup of kLaneBlock threads
// per CU (the tables fill most of the LDS), lane-direct dwordx4 loads with a
// D-deep ring, grid-stride over chunk groups so each workgroup fills its
// tables once.
template <int K, int D, bool kPair = true>
__device__ __forceinline__ void crc32_fixed_lane_body(const uint8_t* __restrict__ base, uint64_t n,
                                                      uint32_t len, uint64_t stride,
                                                      uint32_t* __restrict__ out, uint8_t* tabs) {
  Crc32LaneHasher<K> h;
  h.setup(tabs);
  const uint64_t step = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += step) {
    Crc32State st = h.init();
    lane_range<Crc32LaneHasher<K>, D, kPair>(h, st, base + i * stride, len);
    out[i] = st.c;
  }
}

__global__ void __launch_bounds__(1024)
crc32_fixed_lane32(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                   uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t tabs[Crc32LaneHasher<32>::kLdsBytes];
  crc32_fixed_lane_body<32, 4>(base, n, len, stride, out, tabs);
}

__global__ void __launch_bounds__(1024)
crc32_fixed_lane16(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                   uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t tabs[Crc32LaneHasher<16>::kLdsBytes];
  crc32_fixed_lane_body<16, 4>(base, n, len, stride, out, tabs);
}

// ---------------------------------------------------------------------------
// CRC-32 with conflict-reduced lane tables AND whole-line loads ("xlane16").
// ds_read_b32 banks on (addr/4) mod 32 in two 32-lane groups
// (MI355X_MICROARCH §LDS), so random lookups into one shared table set run
// ~3.5-way conflicted: crc32_fixed_xpose holds the top clock (2.38 GHz,
// profiles/r01_clock_probe_crc.json) and is LDS-cycle-bound.  Here
// Crc32LaneHasher<16> (16 interleaved copies, 64 KiB) leaves two lanes of a
// group per bank pair (1.5-way), and the xpose loader keeps whole-line loads
// with a HALF image -- 4 KiB per wave: rows 0-31 are written and read back by
// lanes 0-31, then rows 32-63 by lanes 32-63 -- so 16 waves' images fit beside
// the tables (64 + 64 KiB).  One 1024-thread workgroup per CU, grid-stride
// over 64-chunk groups, so each CU builds its tables once.
// ---------------------------------------------------------------------------
template <class H, int CP>
__device__ __forceinline__ void xpose_half_group(H& h, const uint8_t* __restrict__ base,
                                                 uint64_t n, uint32_t len, uint64_t stride,
                                                 uint64_t wave_first,
                                                 typename H::Out* __restrict__ out, uint8_t* img) {
  const uint32_t lane = threadIdx.x & 63u;
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
  const bool lo = lane < 32u;
  const uint8_t* myrow = img + (lane & 31u) * 128u;
  const uint32_t nfull = len >> 6;
  const uint32_t nstage = nfull >> 1;
  typename H::State st = h.init();

  auto load_stage = [&](u32x4 (&R)[8], uint32_t stg) __attribute__((always_inline)) {
#pragma unroll
    for (int r = 0; r < 8; ++r)
      R[r] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, (int)voff[r], (int)(stg * 128u), CP);
  };
  auto read_row = [&](uint4 (&w)[2][4]) __attribute__((always_inline)) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const u32x4 v = *reinterpret_cast<const u32x4*>(myrow + ((q ^ g) * 16));
      w[q >> 2][q & 3] = make_uint4(v.x, v.y, v.z, v.w);
    }
  };
  auto consume = [&](u32x4 (&R)[8], uint32_t next, bool refill) __attribute__((always_inline)) {
    uint4 w[2][4];
#pragma unroll
    for (int r = 0; r < 4; ++r)
      *reinterpret_cast<u32x4*>(img + r * 1024 + lane * 16) = R[r];
    __builtin_amdgcn_wave_barrier();
    if (lo) read_row(w);
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int r = 4; r < 8; ++r)
      *reinterpret_cast<u32x4*>(img + (r - 4) * 1024 + lane * 16) = R[r];
    __builtin_amdgcn_wave_barrier();
    if (!lo) read_row(w);
    __builtin_amdgcn_wave_barrier();
    if (refill) load_stage(R, next);
    __builtin_amdgcn_sched_barrier(0);
    h.block(st, w[0]);
    h.block(st, w[1]);
  };

  if (nstage) {
    const uint32_t lasts = nstage - 1;
    u32x4 R[8];
    load_stage(R, 0);
    for (uint32_t stg = 0; stg < nstage; ++stg) consume(R, min(stg + 1, lasts), stg < lasts);
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

template <class H>
__device__ __forceinline__ void crc32_xlane_body(const uint8_t* __restrict__ base, uint64_t n,
                                                 uint32_t len, uint64_t stride,
                                                 uint32_t* __restrict__ out, uint8_t* tabs,
                                                 uint8_t* img) {
  H h;
  h.setup(tabs);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t ngroups = (n + 63) / 64;
  // wave-major over the grid: group g goes to workgroup g % grid, so a batch
  // of fewer than 16 groups per CU still spreads over every CU
  for (uint64_t gi = (uint64_t)wave * gridDim.x + blockIdx.x; gi < ngroups; gi += (uint64_t)gridDim.x * 16u)
    xpose_half_group<H, 2>(h, base, n, len, stride, gi * 64u, out, img + wave * 4096u);
}

__global__ void __launch_bounds__(1024)
crc32_fixed_xlane16(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                    uint32_t* __restrict__ out) {
  // one array, tables first: they sit at LDS address 0, so a table's base
  // folds into the 16-bit ds_read offset instead of costing a v_or per lookup
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32LaneHasher<16>::kLdsBytes + 16 * 4096];
  crc32_xlane_body<Crc32LaneHasher<16>>(base, n, len, stride, out, lds,
                                        lds + Crc32LaneHasher<16>::kLdsBytes);
}

__global__ void __launch_bounds__(1024)
crc32_fixed_xperm16(const uint8_t* __restrict__ base, uint64_t n, uint32_t len, uint64_t stride,
                    uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32PermHasher::kLdsBytes + 16 * 4096];
  crc32_xlane_body<Crc32PermHasher>(base, n, len, stride, out, lds, lds + Crc32PermHasher::kLdsBytes);
}


// Descriptor batches (ragged netcache blocks) with the XPERM16 tables: the
// descriptor xpose loader (desc_xpose_group) with half images, one 1024-thread
// workgroup per CU, grid-stride over 64-chunk groups of `order`.
__global__ void __launch_bounds__(1024)
crc32_desc_xperm16(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                   const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order,
                   uint64_t n, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[Crc32PermHasher::kLdsBytes + 16 * 4096];
  Crc32PermHasher h;
  h.setup(lds);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  uint8_t* img = lds + Crc32PermHasher::kLdsBytes + wave * 4096u;
  const uint64_t ngroups = (n + 63) / 64;
  for (uint64_t gi = (uint64_t)wave * gridDim.x + blockIdx.x; gi < ngroups; gi += (uint64_t)gridDim.x * 16u)
    desc_xpose_group<2, Crc32PermHasher, 0, 1, true, false>(h, base, DescArrays{offs, lens, order}, n,
                                                            gi * 64u, out, img);   // (wave-major, as above)
}


// round-1 fastcrc kernel: lane-direct loads over shared slicing-by-8 tables
// fastcrc (blk_io.c:408-424): len <= f -> crc(all), else crc(first f bytes)
// ^ crc(last f bytes).  kImplicit: chunk i at base + i*stride, length flen.
template <bool kImplicit>
__global__ void __launch_bounds__(256)
crc32_fast(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
           const uint32_t* __restrict__ lens, uint64_t n, uint64_t stride, uint32_t flen,
           uint32_t fast, uint32_t* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t tabs[Crc32Hasher::kLdsBytes];
  Crc32Hasher h;
  h.setup(tabs);
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* chunk = base + (kImplicit ? i * stride : offs[i]);
  const uint32_t len = kImplicit ? flen : lens[i];
  Crc32State a = h.init();
  if (len <= fast) {
    lane_range<Crc32Hasher, 2>(h, a, chunk, len);
  } else {
    lane_range<Crc32Hasher, 2>(h, a, chunk, fast);
    Crc32State b = h.init();
    lane_range<Crc32Hasher, 2>(h, b, chunk + (len - fast), fast);
    a.c ^= b.c;
  }
  out[i] = a.c;
}


// The fed-chain machinery (md5_w, fed_steps, compress_fed, fed_long_group)
// moved to md5_kernels.h in round 3, where md5_desc_fed runs small batches.

// HYBRID with fed chains: 2-wave workgroups.  Workgroup b < L = min(nlong,
// groups) owns group b: a long aligned group (longest chunk >= kHybridLongBlocks
// blocks, every start 16-B aligned) runs as a fed pair, any other one on wave 0
// through the XDMA loader.  Workgroup b >= L runs groups L + 2(b - L) + wave,
// XDMA.  NT x 16 KiB of LDS: the addend tables, or two XDMA images.  (The
// workgroup cannot hold more waves: s_barrier counts every live wave of it,
// so XDMA waves beside a pair would hold up its hand-overs.)
template <int D = 4, int NT = 2, bool kFeedOff = false>
__global__ void __launch_bounds__(128)
md5_desc_hybrid_fed(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                    const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
                    uint4* __restrict__ out, uint32_t nlong) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[NT * kFedTable];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const uint64_t groups = (n + 63) / 64;
  const uint64_t L = nlong < groups ? nlong : groups;
  const uint64_t b = blockIdx.x;
  const DescArrays src{offs, lens, order};
  Md5Hasher<true> h;
  if (b < L) {
    const uint64_t first = b * 64u;
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t i = first + lane;
    const bool live = i < n;
    const uint64_t c = src.index(live ? i : first);
    const uint64_t off = src.off(c);
    const uint32_t len = live ? src.len(c) : 0u;
    const uint32_t nfull = len >> 6;
    const uint32_t bmax = wave_max(nfull);
    const bool unaligned = __ballot(live && ((((uintptr_t)base + off) & 15u) != 0)) != 0;
    if (bmax >= kHybridLongBlocks && !unaligned) {
      fed_long_group<D, NT, kFeedOff>(base, out, lds, wave == 1, nfull, bmax, off, len, c, live);
      return;
    }
    if (wave == 0)
      desc_xpose_group<2, Md5Hasher<true>, 0, 1, false, true, true>(h, base, src, n, first, out, lds);
    return;
  }
  const uint64_t grp = L + 2 * (b - L) + wave;
  if (grp >= groups) return;
  desc_xpose_group<2, Md5Hasher<true>, 0, 1, false, true, true>(h, base, src, n, grp * 64u, out,
                                                                lds + wave * 8192u);
}

// Only the first min(L, groups) groups of md5_desc_hybrid_fed (the pair
// workgroups), for a split launch: the rest goes to md5_desc_xdma on the
// caller's stream while this kernel runs on a high-priority stream, so the
// XDMA waves get the ordinary one-wave workgroups and 8 KiB images and the
// pairs their 32 KiB (md5diag_fed_split).  kMinBlocks = 2: every aligned
// group of at least two blocks runs as a pair (small batches, where each
// wave is nearly alone on its SIMD; md5diag_variant_desc 9).
template <int D = 4, int NT = 2, uint32_t kMinBlocks = kHybridLongBlocks>
__global__ void __launch_bounds__(128)
md5_desc_fed_pairs(const uint8_t* __restrict__ base, const uint64_t* __restrict__ offs,
                   const uint32_t* __restrict__ lens, const uint32_t* __restrict__ order, uint64_t n,
                   uint4* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[NT * kFedTable];
  const uint32_t wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const DescArrays src{offs, lens, order};
  Md5Hasher<true> h;
  const uint64_t first = (uint64_t)blockIdx.x * 64u;
  const uint32_t lane = threadIdx.x & 63u;
  const uint64_t i = first + lane;
  const bool live = i < n;
  const uint64_t c = src.index(live ? i : first);
  const uint64_t off = src.off(c);
  const uint32_t len = live ? src.len(c) : 0u;
  const uint32_t nfull = len >> 6;
  const uint32_t bmax = wave_max(nfull);
  const bool unaligned = __ballot(live && ((((uintptr_t)base + off) & 15u) != 0)) != 0;
  if (bmax >= kMinBlocks && !unaligned) {
    fed_long_group<D, NT>(base, out, lds, wave == 1, nfull, bmax, off, len, c, live);
    return;
  }
  if (wave == 0)
    desc_xpose_group<2, Md5Hasher<true>, 0, 1, false, true, true>(h, base, src, n, first, out, lds);
}

// grid of md5_desc_hybrid_fed
__host__ __device__ inline uint64_t hybrid_fed_grid(uint64_t n, uint32_t nlong) {
  const uint64_t groups = (n + 63) / 64;
  const uint64_t L = nlong < groups ? nlong : groups;
  return L + (groups - L + 1) / 2;
}

}  // namespace md5hip
