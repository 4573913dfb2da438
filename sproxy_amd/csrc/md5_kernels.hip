// md5_kernels.hip -- instantiates the batched-MD5 kernels (md5_kernels.h)
// and exports the C ABI of include/md5hip.h.
#include "md5_kernels.h"

namespace md5hip {
// Explicit instantiations: kernels referenced only from host templates are
// otherwise not emitted by hipcc (host stub and device code both missing).
template __global__ void md5_fixed_direct<2, Md5Hasher<false>>(const uint8_t*, uint64_t, uint32_t, uint64_t, uint4*);
template __global__ void md5_desc<false>(const uint8_t*, const uint64_t*, const uint32_t*,
                                         const uint32_t*, uint64_t, uint64_t, uint32_t, uint4*);
template __global__ void md5_desc<true>(const uint8_t*, const uint64_t*, const uint32_t*,
                                        const uint32_t*, uint64_t, uint64_t, uint32_t, uint4*);
template __global__ void crc32_desc<true>(const uint8_t*, const uint64_t*, const uint32_t*,
                                          const uint32_t*, uint64_t, uint64_t, uint32_t,
                                          uint32_t*);

}  // namespace md5hip

// ===========================================================================
// C ABI (include/md5hip.h)
// ===========================================================================
#include <errno.h>
#include <stdlib.h>
#include <string.h>
#include <atomic>
#include <map>
#include <tuple>
#include <mutex>
#include <thread>
#include <vector>

#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/counting_iterator.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include "../../include/md5hip.h"
#include "md5_internal.h"

using namespace md5hip;

namespace {

constexpr int kBlock = 256;
constexpr int kDescBlock = 64;

int device_ok() {
  int dev = -1;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return -ENODEV;
  return 0;
}

int launched() {
  return hipGetLastError() == hipSuccess ? 0 : -EIO;
}

// Compute units of the current device (grid sizing of one-workgroup-per-CU
// kernels and HYBRID's long-wave count).
// Cached per device: a small launch asks several times (planner, grid, the
// CRC choice), and the attribute query is a runtime call each time.
int cu_count() {
  static std::atomic<int> cached[64];
  int dev = 0, cus = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256;
  if (dev >= 0 && dev < 64 && (cus = cached[dev].load(std::memory_order_relaxed)) > 0) return cus;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
    return 256;
  if (dev >= 0 && dev < 64) cached[dev].store(cus, std::memory_order_relaxed);
  return cus;
}

// BALANCED's self-resetting group counters: one pair per (device, stream),
// allocated and zeroed on first use (launches on one stream are ordered, so
// a counter reset by the last wave of launch k is zero for launch k+1).
// hipStreamPerThread is one handle that names a different stream in every
// thread, so it is keyed by a per-thread id as well (ids are never reused,
// so a finished thread's launch still in flight keeps its own counter).
std::mutex g_ctr_mu;
std::map<std::tuple<int, hipStream_t, uint64_t>, uint32_t*> g_ctr;
std::atomic<uint64_t> g_thread_ids{0};

uint64_t this_thread_id() {
  thread_local const uint64_t id = ++g_thread_ids;
  return id;
}

uint32_t* balanced_counter(hipStream_t s) {
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return nullptr;
  const auto key = std::make_tuple(dev, s, s == hipStreamPerThread ? this_thread_id() : 0ull);
  std::lock_guard<std::mutex> lk(g_ctr_mu);
  auto it = g_ctr.find(key);
  if (it != g_ctr.end()) return it->second;
  uint32_t* c = nullptr;
  if (hipMalloc(&c, 4 * sizeof(uint32_t)) != hipSuccess) return nullptr;
  if (hipMemset(c, 0, 4 * sizeof(uint32_t)) != hipSuccess) { (void)hipFree(c); return nullptr; }
  g_ctr[key] = c;
  return c;
}

// A kernel's dynamic-LDS limit raised once per device (the attribute is set
// on the current device; a pool drives several from one process).
bool dyn_lds_ready(const void* kern, uint32_t lds) {
  static std::mutex mu;
  static std::map<std::pair<int, const void*>, bool> done;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return false;
  std::lock_guard<std::mutex> lk(mu);
  auto it = done.find({dev, kern});
  if (it != done.end()) return it->second;
  const bool ok = hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds) ==
                  hipSuccess;
  done[{dev, kern}] = ok;
  return ok;
}

// md5hip_plan_desc's decision from four order statistics of the batch: the
// longest chunk's blocks, the median group's first key, the summed first
// keys of all groups (work), and the blocks of the chunk two waves per CU deep.
int plan_choice(uint32_t bmax, uint64_t median, uint64_t total, uint32_t probe_blocks) {
  if (8u * median <= (uint64_t)bmax + 1) {
    const uint64_t simds = 4ull * (uint64_t)cu_count();
    if (10u * total >= 4u * simds * ((uint64_t)bmax + 1)) return MD5HIP_DESC_BALANCED;
  }
  return 4ull * probe_blocks <= bmax ? MD5HIP_DESC_HYBRID : MD5HIP_DESC_XDMA;
}

// One workgroup of `threads` per CU, grid-stride over 64-chunk groups.
uint32_t per_cu_grid(uint64_t n) {
  const uint64_t need = (n + 63) / 64;
  const uint64_t cap = (uint64_t)cu_count();
  return (uint32_t)(need < cap ? need : cap);
}

// MD5 batches of at most this many 64-chunk groups per CU run as fed pairs
// (md5_desc_fed; planners below, and the fixed-length AUTO launch).
constexpr uint64_t kFedGroupsPerCu = 1;

// CRC-32 of a full-CRC batch, split across a wave per chunk (crc32_split)
// or streamed one lane per chunk.  The streaming launch lasts one chunk's
// serial chain, ~13 ns per byte (220 us at 16 KiB, 12.9 ms at 1 MiB) with an
// ~18 us floor; the split one moves ~2.8 TB/s with ~3 ns per chunk of fixed
// work.  Measured crossovers (profiles/r03aa/, profiles/r03u/): ~36 K chunks
// at 16 KiB, ~38 K at 64 KiB, none up to 4 K at 1 MiB, ~3.5 K at 1 KiB.  So
// with the chunk length known, split up to 128 chunks per CU when chunks are
// >= 2 KiB and up to 12 per CU below; with it unknown (device-side lengths),
// up to kCrcSplitPerCu.
constexpr uint64_t kCrcSplitPerCu = 16;
constexpr uint32_t kCrcSplitMinWindow = 2048;    // fastcrc windows split from this size
bool crc_split_fits(uint64_t n, uint64_t len) {
  const uint64_t cus = (uint64_t)cu_count();
  if (len == 0) return n <= kCrcSplitPerCu * cus;
  return len >= 2048 ? n <= 128 * cus : n <= 12 * cus;
}
bool crc_split_pick(uint64_t n, int variant, uint64_t len = 0) {
  if (variant == CRC32HIP_SPLIT) return true;
  return variant == CRC32HIP_AUTO && crc_split_fits(n, len);
}
// 4 chunks (waves) per 256-thread workgroup; grid-stride past 8 per CU
uint32_t crc_split_grid(uint64_t n) {
  const uint64_t need = (n + 3) / 4;
  const uint64_t cap = 2ull * (uint64_t)cu_count();
  return (uint32_t)(need < cap ? need : cap);
}

}  // namespace

extern "C" {

int md5hip_abi_version(void) { return MD5HIP_ABI_VERSION; }

// md5_internal.h: the CRC variant for a descriptor batch whose mean chunk
// length the caller knows (the batcher does).  Not split = XDMA16 named
// explicitly: AUTO would decide again with the length unknown
// (kCrcSplitPerCu per CU) and split short-chunk batches past the crossover.
__attribute__((visibility("hidden"))) int md5hip_crc_desc_choice(uint64_t n, uint64_t mean_len) {
  return crc_split_fits(n, mean_len ? mean_len : 1) ? CRC32HIP_SPLIT : CRC32HIP_XDMA16;
}
// (with fastcrc the batcher passes 2n windows of fastcrc bytes; windows under
// kCrcSplitMinWindow keep the window kernels whatever the variant says)

// The shipped kernels are fixed: the round-1 A/B variants live in the
// diagnostic library (removed in round 4; git history at 993ee7d), and no environment
// variable re-routes a product launch.
int md5hip_resolve_variant(int v) { return v == MD5HIP_AUTO ? MD5HIP_XDMA1NT : v; }
int crc32hip_resolve_variant(int v) { return v == CRC32HIP_AUTO ? CRC32HIP_XDMA16 : v; }

const char* md5hip_variant_name(int v) {
  switch (v) {
    case MD5HIP_AUTO: return "auto";
    case MD5HIP_DIRECT2: return "direct2";
    case MD5HIP_XDMA1NT: return "xdma1nt";
    default: return "?";
  }
}

int md5hip_digest_desc(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                       const uint32_t* d_order, uint64_t n, unsigned char* d_digests,
                       void* stream) {
  return md5hip_digest_desc_variant(d_base, d_offsets, d_lens, d_order, n, d_digests, stream,
                                    MD5HIP_DESC_AUTO);
}

int md5hip_digest_desc_variant(const void* d_base, const uint64_t* d_offsets,
                               const uint32_t* d_lens, const uint32_t* d_order, uint64_t n,
                               unsigned char* d_digests, void* stream, int variant) {
  if (n == 0) return 0;
  if (!d_base || !d_offsets || !d_lens || !d_digests) return -EINVAL;
  if (((uintptr_t)d_digests & 15u) != 0) return -EINVAL;
  if (variant != MD5HIP_DESC_AUTO && variant != MD5HIP_DESC_LANE && variant != MD5HIP_DESC_HYBRID &&
      variant != MD5HIP_DESC_XDMA && variant != MD5HIP_DESC_BALANCED && variant != MD5HIP_DESC_FED &&
      variant != MD5HIP_DESC_LINES)
    return -EINVAL;
  if (int e = device_ok()) return e;
  const uint64_t g = (n + 63) / 64;
  if (g > 0x7fffffffull) return -EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* base = (const uint8_t*)d_base;
  if (variant == MD5HIP_DESC_HYBRID) {
    // the first waves (one per CU: the longest chunks in longest-first order)
    // run their chains lane-direct (md5hip_plan_desc picks HYBRID)
    hipLaunchKernelGGL(md5_desc_hybrid, dim3((uint32_t)g), dim3(64), 0, s, base, d_offsets, d_lens,
                       d_order, n, (uint4*)d_digests, (uint32_t)cu_count());
    return launched();
  }
  if (variant == MD5HIP_DESC_BALANCED) {
    uint32_t* ctr = balanced_counter(s);
    if (!ctr) return -ENOMEM;
    constexpr int WPB = kBalancedWaves;
    constexpr uint32_t lds = BalancedCfg<WPB, kBalancedImages>::kLds;
    auto kern = md5_desc_balanced_t<WPB, kBalancedImages, kBalancedPolicy>;
    if (!dyn_lds_ready(reinterpret_cast<const void*>(kern), lds)) return -ENODEV;
    // the kernel resets its counter on exit; zero it on the stream anyway, so
    // a launch that never finished (a fault) cannot poison the next one
    if (hipMemsetAsync(ctr, 0, 4 * sizeof(uint32_t), s) != hipSuccess) return -EIO;
    hipLaunchKernelGGL(kern, dim3((uint32_t)cu_count()), dim3(64 * WPB), lds, s,
                       base, d_offsets, d_lens, d_order, n, (uint4*)d_digests, ctr);
    return launched();
  }
  if (variant == MD5HIP_DESC_FED) {
    // chain + feeder wave per 64-chunk group (md5_kernels.h md5_desc_fed)
    hipLaunchKernelGGL(md5_desc_fed<false>, dim3((uint32_t)g), dim3(128), 0, s, base, d_offsets,
                       d_lens, d_order, n, (uint64_t)0, 0u, (uint4*)d_digests);
    return launched();
  }
  if (variant == MD5HIP_DESC_LINES) {
    hipLaunchKernelGGL(md5_desc_lines, dim3((uint32_t)g), dim3(64), 0, s, base, d_offsets, d_lens,
                       d_order, n, (uint4*)d_digests);
    return launched();
  }
  if (variant == MD5HIP_DESC_AUTO || variant == MD5HIP_DESC_XDMA) {
    hipLaunchKernelGGL(md5_desc_xdma, dim3((uint32_t)g), dim3(64), 0, s, base, d_offsets, d_lens,
                       d_order, n, (uint4*)d_digests);
    return launched();
  }
  // LANE.  One wave per workgroup: a mixed batch has few waves, and the
  // dispatcher then spreads them one per CU instead of packing 4 onto one CU
  // where the long chunks' lane-direct loads contend for the CU's address unit
  // (scripts/c3_trace.py, deleted in 4de68d0: 28.7 -> 13.2 ms on the C3 batch).
  hipLaunchKernelGGL(md5_desc<false>, dim3((uint32_t)g), dim3(kDescBlock), 0, s, base, d_offsets,
                     d_lens, d_order, n, (uint64_t)0, 0u, (uint4*)d_digests);
  return launched();
}

int md5hip_digest_fixed_variant(const void* d_base, uint64_t n, uint32_t len, uint64_t stride,
                                unsigned char* d_digests, void* stream, int variant) {
  if (n == 0) return 0;
  if (!d_base || !d_digests || len > stride) return -EINVAL;
  if (((uintptr_t)d_digests & 15u) != 0) return -EINVAL;
  if (variant != MD5HIP_AUTO && variant != MD5HIP_DIRECT2 && variant != MD5HIP_XDMA1NT)
    return -EINVAL;
  if (int e = device_ok()) return e;
  const uint64_t grid = (n + kBlock - 1) / kBlock;
  if (grid > 0x7fffffffull) return -EINVAL;
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* base = (const uint8_t*)d_base;
  uint4* out = (uint4*)d_digests;
  if (((uintptr_t)base & 15u) != 0 || (stride & 15u) != 0) {
    // chunk starts not 16-B aligned: descriptor kernel with implicit offsets
    hipLaunchKernelGGL(md5_desc<true>, dim3((uint32_t)((n + kDescBlock - 1) / kDescBlock)),
                       dim3(kDescBlock), 0, s, base,
                       (const uint64_t*)nullptr, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr, n, stride, len, out);
    return launched();
  }
  // xdma1nt addresses a 64-chunk group with 32-bit buffer offsets
  if (variant == MD5HIP_DIRECT2 || stride >= (1ull << 31) / 64) {
    hipLaunchKernelGGL((md5_fixed_direct<2, Md5Hasher<false>>), dim3((uint32_t)grid), dim3(kBlock),
                       0, s, base, n, len, stride, out);
    return launched();
  }
  if (variant == MD5HIP_AUTO && (n + 63) / 64 <= kFedGroupsPerCu * (uint64_t)cu_count() &&
      (len >> 6) >= kFedMinBlocks) {
    // a small batch: its launch is one chunk's chain, which fed pairs shorten
    hipLaunchKernelGGL(md5_desc_fed<true>, dim3((uint32_t)((n + 63) / 64)), dim3(128), 0, s, base,
                       (const uint64_t*)nullptr, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr, n, stride, len, out);
    return launched();
  }
  hipLaunchKernelGGL(md5_fixed_xdma1nt, dim3((uint32_t)grid), dim3(kBlock), 0, s, base, n, len,
                     stride, out);
  return launched();
}

int md5hip_digest_fixed(const void* d_base, uint64_t n, uint32_t len, uint64_t stride,
                        unsigned char* d_digests, void* stream) {
  return md5hip_digest_fixed_variant(d_base, n, len, stride, d_digests, stream, MD5HIP_AUTO);
}

int crc32hip_fixed_variant(const void* d_base, uint64_t n, uint32_t len, uint64_t stride,
                           uint32_t fastcrc, uint32_t* d_crcs, void* stream, int variant) {
  if (n == 0) return 0;
  if (!d_base || !d_crcs || len > stride || (fastcrc & 3u)) return -EINVAL;
  if (((uintptr_t)d_crcs & 3u) != 0) return -EINVAL;
  if (variant != CRC32HIP_AUTO && variant != CRC32HIP_XDMA16 && variant != CRC32HIP_SPLIT)
    return -EINVAL;
  if (int e = device_ok()) return e;
  hipStream_t s = (hipStream_t)stream;
  const uint8_t* base = (const uint8_t*)d_base;
  const uint64_t g = (n + kDescBlock - 1) / kDescBlock;
  if (g > 0x7fffffffull) return -EINVAL;
  // the split kernel: full-CRC batches, and windowed ones (two messages of
  // fastcrc bytes per chunk) with windows of >= 2 KiB; shorter windows are
  // chains short enough for the window kernels (F = 1000: split 28-48 us
  // against 30-32 us, F = 4096: 15-31 against 57-60; profiles/r03af/)
  const bool windows = fastcrc && len > fastcrc;
  if ((!windows || fastcrc >= kCrcSplitMinWindow) &&
      crc_split_pick(windows ? 2 * n : n, variant, windows ? fastcrc : (len ? len : 1))) {
    hipLaunchKernelGGL(crc32_split<true>, dim3(crc_split_grid(n)), dim3(256), 0, s, base,
                       (const uint64_t*)nullptr, (const uint32_t*)nullptr,
                       (const uint32_t*)nullptr, n, stride, len, fastcrc, d_crcs);
    return launched();
  }
  if (fastcrc && len > fastcrc) {
    if (fastcrc == 64 || fastcrc == 128) {
      // one- or two-block windows: lane loads, next group in flight
      hipLaunchKernelGGL(crc32_fast_pipe, dim3(per_cu_grid(2 * n)), dim3(1024), 0, s, base,
                         (const uint64_t*)nullptr, (const uint32_t*)nullptr, n, stride, len, fastcrc,
                         d_crcs);
      return launched();
    }
    // head and tail windows as 2n rows through the LDS-DMA loader
    hipLaunchKernelGGL(crc32_fast_xdma16, dim3(per_cu_grid(2 * n)), dim3(768), 0, s, base,
                       (const uint64_t*)nullptr, (const uint32_t*)nullptr, n, stride, len, fastcrc,
                       d_crcs);
    return launched();
  }
  const bool aligned = ((uintptr_t)base & 15u) == 0 && (stride & 15u) == 0;
  if (aligned && stride < (1ull << 31) / 64) {
    // one 768-thread workgroup per CU (160 KiB LDS), grid-stride, wave-major
    hipLaunchKernelGGL(crc32_fixed_xdma16, dim3(per_cu_grid(n)), dim3(768), 0, s, base, n, len,
                       stride, d_crcs);
    return launched();
  }
  hipLaunchKernelGGL(crc32_desc<true>, dim3((uint32_t)g), dim3(kDescBlock), 0, s, base,
                     (const uint64_t*)nullptr, (const uint32_t*)nullptr,
                     (const uint32_t*)nullptr, n, stride, len, d_crcs);
  return launched();
}

int crc32hip_fixed(const void* d_base, uint64_t n, uint32_t len, uint64_t stride,
                   uint32_t fastcrc, uint32_t* d_crcs, void* stream) {
  return crc32hip_fixed_variant(d_base, n, len, stride, fastcrc, d_crcs, stream, CRC32HIP_AUTO);
}

int crc32hip_desc(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                  const uint32_t* d_order, uint64_t n, uint32_t fastcrc, uint32_t* d_crcs,
                  void* stream) {
  return crc32hip_desc_variant(d_base, d_offsets, d_lens, d_order, n, fastcrc, d_crcs, stream,
                               CRC32HIP_AUTO);
}

int crc32hip_desc_variant(const void* d_base, const uint64_t* d_offsets, const uint32_t* d_lens,
                          const uint32_t* d_order, uint64_t n, uint32_t fastcrc, uint32_t* d_crcs,
                          void* stream, int variant) {
  if (n == 0) return 0;
  if (!d_base || !d_offsets || !d_lens || !d_crcs || (fastcrc & 3u)) return -EINVAL;
  if (((uintptr_t)d_crcs & 3u) != 0) return -EINVAL;
  if (variant != CRC32HIP_AUTO && variant != CRC32HIP_XDMA16 && variant != CRC32HIP_SPLIT)
    return -EINVAL;
  if (int e = device_ok()) return e;
  hipStream_t s = (hipStream_t)stream;
  const uint64_t g = (n + kDescBlock - 1) / kDescBlock;
  if (g > 0x7fffffffull) return -EINVAL;
  if ((fastcrc == 0 || fastcrc >= kCrcSplitMinWindow) && crc_split_pick(fastcrc ? 2 * n : n, variant)) {
    hipLaunchKernelGGL(crc32_split<false>, dim3(crc_split_grid(n)), dim3(256), 0, s,
                       (const uint8_t*)d_base, d_offsets, d_lens, d_order, n, (uint64_t)0, 0u,
                       fastcrc, d_crcs);
    return launched();
  }
  if (fastcrc == 64 || fastcrc == 128) {
    hipLaunchKernelGGL(crc32_fast_pipe, dim3(per_cu_grid(2 * n)), dim3(1024), 0, s,
                       (const uint8_t*)d_base, d_offsets, d_lens, n, (uint64_t)0, 0u, fastcrc,
                       d_crcs);
    return launched();
  }
  if (fastcrc) {
    hipLaunchKernelGGL(crc32_fast_xdma16, dim3(per_cu_grid(2 * n)), dim3(768), 0, s,
                       (const uint8_t*)d_base, d_offsets, d_lens, n, (uint64_t)0, 0u, fastcrc,
                       d_crcs);
    return launched();
  }
  // XDMA16: one 768-thread workgroup per CU, LDS-DMA images
  hipLaunchKernelGGL(crc32_desc_xdma16, dim3(per_cu_grid(n)), dim3(768), 0, s,
                     (const uint8_t*)d_base, d_offsets, d_lens, d_order, n, d_crcs);
  return launched();
}

// Batched MD5Init / MD5Update / MD5Final on caller-owned contexts.
int md5hip_init_ctx(struct MD5Context* d_ctxs, uint64_t n, void* stream) {
  if (n == 0) return 0;
  if (!d_ctxs || ((uintptr_t)d_ctxs & 3u)) return -EINVAL;
  if (int e = device_ok()) return e;
  const uint64_t g = (n + kBlock - 1) / kBlock;
  if (g > 0x7fffffffull) return -EINVAL;
  hipLaunchKernelGGL(md5_init_ctx, dim3((uint32_t)g), dim3(kBlock), 0, (hipStream_t)stream,
                     reinterpret_cast<uint32_t*>(d_ctxs), n);
  return launched();
}

int md5hip_update_ctx(struct MD5Context* d_ctxs, const void* const* d_ptrs, const uint32_t* d_lens,
                      uint64_t n, void* stream) {
  if (n == 0) return 0;
  if (!d_ctxs || !d_ptrs || !d_lens || ((uintptr_t)d_ctxs & 3u)) return -EINVAL;
  if (int e = device_ok()) return e;
  const uint64_t g = (n + 63) / 64;                   // one wave per 64 contexts
  if (g > 0x7fffffffull) return -EINVAL;
  if (g <= kFedGroupsPerCu * (uint64_t)cu_count()) {
    // few contexts: one update's chain bounds the launch; fed pairs shorten it
    hipLaunchKernelGGL(md5_update_ctx_fed, dim3((uint32_t)g), dim3(128), 0, (hipStream_t)stream,
                       reinterpret_cast<uint32_t*>(d_ctxs), reinterpret_cast<const uint64_t*>(d_ptrs),
                       d_lens, n);
    return launched();
  }
  hipLaunchKernelGGL(md5_update_ctx, dim3((uint32_t)g), dim3(64), 0, (hipStream_t)stream,
                     reinterpret_cast<uint32_t*>(d_ctxs), reinterpret_cast<const uint64_t*>(d_ptrs),
                     d_lens, n);
  return launched();
}

int md5hip_final_ctx(struct MD5Context* d_ctxs, uint64_t n, unsigned char* d_digests, void* stream) {
  if (n == 0) return 0;
  if (!d_ctxs || !d_digests || ((uintptr_t)d_ctxs & 3u) || ((uintptr_t)d_digests & 15u))
    return -EINVAL;
  if (int e = device_ok()) return e;
  const uint64_t g = (n + kBlock - 1) / kBlock;
  if (g > 0x7fffffffull) return -EINVAL;
  hipLaunchKernelGGL(md5_final_ctx, dim3((uint32_t)g), dim3(kBlock), 0, (hipStream_t)stream,
                     reinterpret_cast<uint32_t*>(d_ctxs), n, reinterpret_cast<uint4*>(d_digests));
  return launched();
}

int md5hip_gather_launch(const struct md5hip_seg* d_segs, uint64_t nseg, unsigned char* d_dst,
                         void* stream) {
  static_assert(sizeof(md5hip_seg) == sizeof(GatherSeg), "segment layout");
  if (nseg == 0) return 0;
  const uint64_t g = nseg < 65536 ? nseg : 65536;
  hipLaunchKernelGGL(gather_segments<4>, dim3((uint32_t)g), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<const GatherSeg*>(d_segs), nseg, d_dst);
  return launched();
}

int md5hip_fill_synthetic(void* d_dst, uint64_t nbytes, uint64_t seed, void* stream) {
  if (nbytes == 0) return 0;
  if (!d_dst || (nbytes & 15u) != 0 || ((uintptr_t)d_dst & 15u) != 0) return -EINVAL;
  if (int e = device_ok()) return e;
  const uint64_t n16 = nbytes / 16;
  uint64_t grid = (n16 + kBlock - 1) / kBlock;
  if (grid > 8192) grid = 8192;
  hipLaunchKernelGGL(fill_synthetic, dim3((uint32_t)grid), dim3(kBlock), 0, (hipStream_t)stream,
                     (uint4*)d_dst, n16, seed);
  return launched();
}

int md5hip_plan_order(const uint32_t* lens, uint64_t n, uint32_t* order) {
  if (n == 0) return 0;
  if (!lens || !order || n > 0xffffffffull) return -EINVAL;
  // counting sort on block count, descending; block counts are < 2^26
  // (len < 2^32), bucket by the bit length of nblocks then by value within
  // small buckets -- a two-level key keeps the histogram tiny.
  uint32_t maxb = 0;
  for (uint64_t i = 0; i < n; ++i) {
    const uint32_t b = (lens[i] >> 6) + 1;
    if (b > maxb) maxb = b;
  }
  if (maxb <= (1u << 20)) {
    // T contiguous index ranges, one histogram each; range t's chunks of key
    // k go after every earlier range's chunks of key k: stable, and the
    // batcher's large coalesced slots (~1 M chunks) plan on several cores.
    const uint64_t per = 1u << 17;
    const uint32_t T = n >= 2 * per ? (uint32_t)(n / per < 8 ? n / per : 8) : 1u;
    const size_t nb = (size_t)maxb + 1;
    uint32_t* cnt = (uint32_t*)calloc(nb * T, sizeof(uint32_t));
    if (!cnt) return -ENOMEM;
    auto range = [&](uint32_t t, uint64_t& lo, uint64_t& hi) {
      lo = n * t / T;
      hi = n * (t + 1) / T;
    };
    auto hist = [&](uint32_t t) {
      uint64_t lo, hi;
      range(t, lo, hi);
      uint32_t* c = cnt + nb * t;
      for (uint64_t i = lo; i < hi; ++i) c[maxb - ((lens[i] >> 6) + 1)]++;
    };
    auto scatter = [&](uint32_t t) {
      uint64_t lo, hi;
      range(t, lo, hi);
      uint32_t* c = cnt + nb * t;
      for (uint64_t i = lo; i < hi; ++i) order[c[maxb - ((lens[i] >> 6) + 1)]++] = (uint32_t)i;
    };
    // ranges 1..T-1 on helper threads; a range whose thread cannot be
    // started runs here (no exception leaves this extern "C" entry)
    auto fan_out = [&](auto&& fn) {
      std::vector<std::thread> th;
      std::vector<uint32_t> mine{0u};
      for (uint32_t t = 1; t < T; ++t) {
        try {
          th.emplace_back(fn, t);
        } catch (...) {
          mine.push_back(t);
        }
      }
      for (uint32_t t : mine) fn(t);
      for (auto& x : th) x.join();
    };
    fan_out(hist);
    uint32_t run = 0;
    for (size_t k = 0; k < nb; ++k)
      for (uint32_t t = 0; t < T; ++t) {
        const uint32_t c = cnt[nb * t + k];
        cnt[nb * t + k] = run;
        run += c;
      }
    fan_out(scatter);
    free(cnt);
    return 0;
  }
  // very long chunks: fall back to a comparison sort
  for (uint64_t i = 0; i < n; ++i) order[i] = (uint32_t)i;
  struct Cmp {
    static int f(const void* a, const void* b, void* ctx) {
      const uint32_t* L = (const uint32_t*)ctx;
      const uint32_t x = L[*(const uint32_t*)a] >> 6, y = L[*(const uint32_t*)b] >> 6;
      if (x != y) return x > y ? -1 : 1;
      return *(const uint32_t*)a < *(const uint32_t*)b ? -1 : 1;
    }
  };
  qsort_r(order, (size_t)n, sizeof(uint32_t), Cmp::f, (void*)lens);
  return 0;
}

// ---------------------------------------------------------------------------
// Batch arenas: device memory whose virtual range is reserved with 1 GiB
// alignment (hipMemAddressReserve + hipMemCreate + hipMemMap), so the page
// tables can use large fragments throughout.  A lane-direct chain walks its
// own chunk, so a wave touches 64 distinct pages per load; HYBRID's long
// chains on C3 ran 9.7 ms in a 16 MiB-aligned buffer and 10.4-11.5 ms in a
// 2 MiB-aligned one (scripts/alloc_probe.py, deleted in 4de68d0).  The whole-line
// loaders are indifferent.
// ---------------------------------------------------------------------------
namespace {
struct Arena {
  void* ptr;       // mapped, kArenaAlign-aligned
  size_t size;
  void* base;      // the reservation (the runtime ignores a reservation's
  size_t rsize;    // alignment argument, so it is over-reserved by kArenaAlign)
  hipMemGenericAllocationHandle_t h;
  int device;
};
std::mutex g_arena_mu;
std::vector<Arena> g_arenas;
constexpr size_t kArenaAlign = size_t(1) << 30;
}  // namespace

int md5hip_arena_alloc(int device, uint64_t bytes, void** out) {
  if (!out || bytes == 0) return -EINVAL;
  *out = nullptr;
  hipMemAllocationProp prop = {};
  prop.type = hipMemAllocationTypePinned;
  prop.location.type = hipMemLocationTypeDevice;
  prop.location.id = device;
  size_t gran = 0;
  if (hipMemGetAllocationGranularity(&gran, &prop, hipMemAllocationGranularityRecommended) !=
          hipSuccess || gran == 0)
    return -ENODEV;
  if (gran < (size_t(2) << 20)) gran = size_t(2) << 20;
  const size_t size = (size_t)((bytes + gran - 1) / gran * gran);
  void* base = nullptr;
  const size_t rsize = size + kArenaAlign;
  hipMemGenericAllocationHandle_t h{};
  if (hipMemAddressReserve(&base, rsize, kArenaAlign, nullptr, 0) != hipSuccess) return -ENOMEM;
  void* ptr = (void*)(((uintptr_t)base + kArenaAlign - 1) & ~(uintptr_t)(kArenaAlign - 1));
  if (hipMemCreate(&h, size, &prop, 0) != hipSuccess) {
    (void)hipMemAddressFree(base, rsize);
    return -ENOMEM;
  }
  hipMemAccessDesc acc = {};
  acc.location = prop.location;
  acc.flags = hipMemAccessFlagsProtReadWrite;
  if (hipMemMap(ptr, size, 0, h, 0) != hipSuccess) {
    (void)hipMemRelease(h);
    (void)hipMemAddressFree(base, rsize);
    return -ENOMEM;
  }
  if (hipMemSetAccess(ptr, size, &acc, 1) != hipSuccess) {
    (void)hipMemUnmap(ptr, size);
    (void)hipMemRelease(h);
    (void)hipMemAddressFree(base, rsize);
    return -EIO;
  }
  {
    std::lock_guard<std::mutex> lk(g_arena_mu);
    g_arenas.push_back(Arena{ptr, size, base, rsize, h, device});
  }
  *out = ptr;
  return 0;
}

int md5hip_arena_free(void* ptr) {
  if (!ptr) return -EINVAL;
  Arena a{};
  {
    std::lock_guard<std::mutex> lk(g_arena_mu);
    size_t k = 0;
    while (k < g_arenas.size() && g_arenas[k].ptr != ptr) ++k;
    if (k == g_arenas.size()) return -ENOENT;
    a = g_arenas[k];
    g_arenas.erase(g_arenas.begin() + (long)k);
  }
  // Not stream-ordered like torch's allocator: a kernel still queued on any
  // stream of the device may read the arena, so drain the device before the
  // pages go (md5hip.h: freeing an arena synchronizes its device).
  int rc = 0, prev = -1;
  const bool had = hipGetDevice(&prev) == hipSuccess;
  if (hipSetDevice(a.device) != hipSuccess || hipDeviceSynchronize() != hipSuccess) rc = -EIO;
  if (hipMemUnmap(a.ptr, a.size) != hipSuccess) rc = -EIO;
  if (hipMemRelease(a.h) != hipSuccess) rc = -EIO;
  if (hipMemAddressFree(a.base, a.rsize) != hipSuccess) rc = -EIO;
  if (had) (void)hipSetDevice(prev);
  return rc;
}

// Small batches (at most two 64-chunk groups per CU: the netcache call
// site's vectors of 16-1,024 blocks) run lane-direct.  There each wave is
// nearly alone on its SIMD and the launch lasts one chunk's serial chain; the
// 8-block register ring keeps HBM latency off that chain, where XDMA's
// per-stage DMA wait and LDS round trip stay on it: 147 vs 163 us for
// 64-4,096 x 16 KiB, 162 vs 171 us at 32,768; past two groups per CU the
// lane-direct loads crowd the address units (65,536 x 16 KiB: 228 vs
// 206 us; profiles/r03/small_batch_kernels_*.json).
constexpr uint64_t kLaneGroupsPerCu = 2;

// Of those, batches of at most one group per CU (kFedGroupsPerCu) run as fed
// pairs (FED: the chain wave's 5th VALU per step moves to a feeder wave on
// another SIMD; 147 -> 138 us at 64-4,096 x 16 KiB, 150.6 -> 141 at 16,384;
// profiles/r03q/small_fed_16k.json) when some chunk has two whole blocks.
static int small_choice(uint64_t ngroups, uint32_t bmax) {
  if (ngroups <= kFedGroupsPerCu * (uint64_t)cu_count() && bmax >= kFedMinBlocks)
    return MD5HIP_DESC_FED;
  return MD5HIP_DESC_LANE;
}

// Planner for descriptor batches (md5hip.h): the longest-first order, and
//  - FED / LANE for small batches (above);
//  - BALANCED for a mixed batch (longest chunk >= 256 KiB, median 64-chunk
//    group <= 1/8 of it) holding >= 0.4 x (SIMDs x longest chain) of work:
//    several waves per SIMD, where LPT placement beats the hardware's
//    (coalesced C3 submissions, profiles/r02_c3_trace.json);
//  - HYBRID when the longest chunks stand out -- the chunk two waves per CU
//    deep in the order is at most a quarter as long -- so their serial chains
//    bound the launch (one C3 batch; fewer long chunks than two waves per CU);
//  - XDMA otherwise (equal-length netcache blocks).  DESIGN.md §5.
int md5hip_plan_desc(const uint32_t* lens, uint64_t n, uint32_t* order) {
  if (int e = md5hip_plan_order(lens, n, order)) return e;
  if (n == 0) return MD5HIP_DESC_XDMA;
  const uint64_t ngroups = (n + 63) / 64;
  const uint32_t bmax = lens[order[0]] >> 6;
  if (ngroups <= kLaneGroupsPerCu * (uint64_t)cu_count()) return small_choice(ngroups, bmax);
  if (bmax < kHybridLongBlocks) return MD5HIP_DESC_XDMA;
  const uint64_t median = (uint64_t)(lens[order[(ngroups / 2) * 64]] >> 6) + 1;
  uint64_t total = 0;           // work in block-steps: a group runs as long as its first lane
  for (uint64_t g = 0; g < ngroups; ++g) total += (uint64_t)(lens[order[g * 64]] >> 6) + 1;
  const uint64_t depth = (uint64_t)cu_count() * 128u;
  const uint64_t p = depth < n - 1 ? depth : n - 1;
  return plan_choice(bmax, median, total, lens[order[p]] >> 6);
}

// md5_internal.h: XDMA becomes LINES when more than half the batch's bytes
// lie in chunks that start 16-B but not 128-B aligned (their stages would
// straddle lines).  Line-aligned and uniform batches keep XDMA, whose four
// waves per SIMD LINES' extra line of registers does not allow.
__attribute__((visibility("hidden"))) int md5hip_lines_choice(int variant, uint64_t unlined_bytes,
                                                              uint64_t bytes) {
  return variant == MD5HIP_DESC_XDMA && 2 * unlined_bytes > bytes ? MD5HIP_DESC_LINES : variant;
}

int md5hip_plan_desc_at(const uint32_t* lens, const uint64_t* addrs, uint64_t n, uint32_t* order) {
  if (!addrs && n) return -EINVAL;
  const int v = md5hip_plan_desc(lens, n, order);
  if (v != MD5HIP_DESC_XDMA) return v;
  uint64_t bytes = 0, unlined = 0;
  for (uint64_t i = 0; i < n; ++i) {
    bytes += lens[i];
    if ((addrs[i] & 127u) != 0 && (addrs[i] & 15u) == 0) unlined += lens[i];
  }
  return md5hip_lines_choice(v, unlined, bytes);
}

int md5hip_plan_hist(const uint32_t* hist, uint32_t kmax, uint64_t n, uint32_t* bucket_start) {
  if (!hist || kmax > MD5HIP_HIST_KMAX) return -EINVAL;
  // walk the keys longest-first; rank r of the sorted order holds key k for
  // r in [start(k), start(k) + hist[k])
  const uint64_t ngroups = (n + 63) / 64;
  const uint64_t rmed = (ngroups / 2) * 64;
  const uint64_t depth = (uint64_t)cu_count() * 128u;
  const uint64_t rprobe = n ? (depth < n - 1 ? depth : n - 1) : 0;
  uint64_t r = 0, total = 0, median = 0, probe = 0;
  uint32_t top = 0;
  for (uint32_t k = kmax; k >= 1; --k) {
    const uint64_t c = hist[k];
    if (bucket_start) bucket_start[kmax - k] = (uint32_t)r;
    if (!c) continue;
    if (!top) top = k;
    // group firsts 64 g in [r, r + c)
    const uint64_t g0 = (r + 63) / 64, g1 = (r + c - 1) / 64;
    if (g1 >= g0) total += (g1 - g0 + 1) * (uint64_t)k;
    if (rmed >= r && rmed < r + c) median = k;
    if (rprobe >= r && rprobe < r + c) probe = k;
    r += c;
  }
  if (bucket_start) bucket_start[kmax] = (uint32_t)r;   // key 0 (never used): the end
  if (n == 0 || !top) return MD5HIP_DESC_XDMA;
  const uint32_t bmax = top - 1;
  if (ngroups <= kLaneGroupsPerCu * (uint64_t)cu_count()) return small_choice(ngroups, bmax);
  if (bmax < kHybridLongBlocks) return MD5HIP_DESC_XDMA;
  return plan_choice(bmax, median, total, (uint32_t)(probe - 1));
}

int md5hip_order_device(const uint32_t* d_lens, uint64_t n, uint32_t kmax, uint32_t* d_next,
                        uint32_t* d_order, void* stream) {
  if (n == 0) return 0;
  if (!d_lens || !d_next || !d_order || kmax > MD5HIP_HIST_KMAX) return -EINVAL;
  if (int e = device_ok()) return e;
  const uint64_t g = (n + 255) / 256;
  if (g > 0x7fffffffull) return -EINVAL;
  hipLaunchKernelGGL(order_scatter, dim3((uint32_t)g), dim3(256), 0, (hipStream_t)stream, d_lens, n,
                     kmax, d_next, d_order);
  return launched();
}

// The stable longest-first order (ABI 5): rocPRIM's LSD radix sort of
// (kmax - key, chunk index) pairs, the key computed from the length as it is
// read (no key array), the index from a counting iterator; radix sort is
// stable, so equal keys keep chunk-index (= address) order -- exactly
// md5hip_plan_desc's host order.  order_scatter's wave-arrival order within a
// key cost a 6-batch C3 BALANCED launch 5-6 % against this order
// (profiles/r06d/, r06e/ order_ab.json).  Scratch: the sorted keys (4 n B,
// 256-B aligned) then rocPRIM's temporary storage.
}  // extern "C"

namespace {
struct BucketOf {
  uint32_t kmax;
  __host__ __device__ uint32_t operator()(uint32_t len) const {
    const uint32_t k = (len >> 6) + 1u;
    return k <= kmax ? kmax - k : kmax;        // a key past kmax: after every bucket
  }
};
unsigned sort_bits(uint32_t kmax) { return 32u - (unsigned)__builtin_clz(kmax | 1u); }
uint64_t keys_bytes(uint64_t n) { return (4 * n + 255) & ~255ull; }
hipError_t order_sort(void* temp, size_t& temp_bytes, const uint32_t* d_lens, uint32_t n, uint32_t kmax,
                      uint32_t* keys_out, uint32_t* d_order, hipStream_t s) {
  auto keys_in = rocprim::make_transform_iterator(d_lens, BucketOf{kmax});
  return rocprim::radix_sort_pairs(temp, temp_bytes, keys_in, keys_out, rocprim::counting_iterator<uint32_t>(0u),
                                   d_order, n, 0u, sort_bits(kmax), s);
}
}  // namespace

extern "C" {

uint64_t md5hip_order_stable_scratch(uint64_t n, uint32_t kmax) {
  if (n == 0) return 0;
  if (n > 0x7fffffffull || kmax > MD5HIP_HIST_KMAX) return 0;
  size_t temp = 0;
  if (order_sort(nullptr, temp, nullptr, (uint32_t)n, kmax ? kmax : MD5HIP_HIST_KMAX, nullptr, nullptr,
                 nullptr) != hipSuccess)
    return 0;
  return keys_bytes(n) + temp;
}

int md5hip_order_device_stable(const uint32_t* d_lens, uint64_t n, uint32_t kmax, void* d_scratch,
                               uint64_t scratch_bytes, uint32_t* d_order, void* stream) {
  if (n == 0) return 0;
  if (!d_lens || !d_order || !d_scratch || kmax == 0 || kmax > MD5HIP_HIST_KMAX || n > 0x7fffffffull)
    return -EINVAL;
  if (int e = device_ok()) return e;
  size_t temp = 0;
  if (order_sort(nullptr, temp, d_lens, (uint32_t)n, kmax, nullptr, d_order, (hipStream_t)stream) != hipSuccess)
    return -EINVAL;
  if (scratch_bytes < keys_bytes(n) + temp) return -ENOSPC;
  uint32_t* keys_out = (uint32_t*)d_scratch;
  void* tmp = (uint8_t*)d_scratch + keys_bytes(n);
  if (order_sort(tmp, temp, d_lens, (uint32_t)n, kmax, keys_out, d_order, (hipStream_t)stream) != hipSuccess)
    return -EIO;
  return launched();
}

}  // extern "C"
