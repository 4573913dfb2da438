// hashers.h -- per-chunk digest policies plugged into the batched loaders of
// md5_kernels.h.  A hasher H provides
//   typename H::State, typename H::Out
//   void setup(uint8_t* lds)            once per workgroup, all threads, before
//                                       any early exit (may __syncthreads)
//   State init()
//   void block(State&, const uint4 (&w)[4])          one full 64-byte block
//   void finish(State&, tail, r, len)                the last len % 64 bytes
//   void store(Out* out, uint64_t i, const State&)
//
//   Md5Hasher<kLat>  md5.c:153-265 (MD5Init / Update / Final per chunk)
//   Crc32Hasher      netcache crc32.c:186-240 (slicing-by-8 over LDS tables)
//   FoldHasher       diagnostics only: 16-word xor fold (load-path ceilings)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "md5_core.h"

namespace md5hip {

__device__ __forceinline__ uint32_t keep_bytes(uint32_t w, int nbytes) {
  // keep the low `nbytes` (0..4) bytes of w
  return nbytes >= 4 ? w : nbytes <= 0 ? 0u : (w & ((1u << (8 * nbytes)) - 1u));
}

// The r (< 64) bytes at `tail` as 16 little-endian words, bytes past r zero.
// Only granules that hold message bytes are read; a 16-B (aligned) or 4-B
// (unaligned) granule never crosses a page, so reading past r cannot fault.
__device__ __forceinline__ void load_tail(const uint8_t* tail, uint32_t r, uint32_t (&w)[16]) {
  const uintptr_t addr = (uintptr_t)tail;
  if ((addr & 15u) == 0) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      uint4 q = make_uint4(0, 0, 0, 0);
      if ((uint32_t)g * 16u < r) q = *reinterpret_cast<const uint4*>(tail + 16 * g);
      w[4 * g + 0] = q.x; w[4 * g + 1] = q.y; w[4 * g + 2] = q.z; w[4 * g + 3] = q.w;
    }
  } else {
    // unaligned tail: aligned dword loads + funnel shift (v_alignbit_b32)
    const uint32_t* base = reinterpret_cast<const uint32_t*>(addr & ~(uintptr_t)3);
    const uint32_t sh = (uint32_t)(addr & 3u) * 8u;
    const uint32_t nwords = (((uint32_t)(addr & 3u)) + r + 3u) >> 2;   // words touched
    uint32_t prev = r ? base[0] : 0u;
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      uint32_t next = ((uint32_t)j + 1u < nwords) ? base[j + 1] : 0u;
      w[j] = __builtin_amdgcn_alignbit(next, prev, sh);
      prev = next;
    }
  }
#pragma unroll
  for (int j = 0; j < 16; ++j) w[j] = keep_bytes(w[j], (int)r - 4 * j);
}

// ---------------------------------------------------------------------------
// MD5 (md5.c).  Digest = A,B,C,D little-endian (md5.c:262-263).
// ---------------------------------------------------------------------------
// kX3 (default): round 3 as v_xad_u32 pairs, 316 instead of 324 VALU per
// block -- measured 1.2 % faster at the board's power cap.
template <bool kLat = false, bool kX3 = true>
struct Md5Hasher {
  using State = md5hip::State;
  using Out = uint4;
  __device__ __forceinline__ void setup(uint8_t*) {}
  __device__ __forceinline__ State init() { return initial_state(); }
  __device__ __forceinline__ void block(State& st, const uint4 (&w)[4]) {
    compress_regs<kLat, kX3>(st, w);
  }
  // 0x80, zeros, 64-bit bit count (md5.c:221-261); one or two final blocks.
  __device__ __forceinline__ void finish(State& st, const uint8_t* tail, uint32_t r,
                                         uint64_t len_bytes) {
    const uint32_t bits_lo = (uint32_t)(len_bytes << 3);
    const uint32_t bits_hi = (uint32_t)(len_bytes >> 29);
    if (r == 0) {
      compress_pad_only(st, bits_lo, bits_hi);
      return;
    }
    uint32_t w[16];
    load_tail(tail, r, w);
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if ((uint32_t)j == (r >> 2)) w[j] |= 0x80u << (8 * (r & 3u));
    if (r < 56) {
      w[14] = bits_lo;
      w[15] = bits_hi;
      compress(st, [&](int i) __attribute__((always_inline)) { return w[i]; });
    } else {
      compress(st, [&](int i) __attribute__((always_inline)) { return w[i]; });
      compress(st, [&](int i) __attribute__((always_inline)) -> uint32_t {
        return i == 14 ? bits_lo : i == 15 ? bits_hi : 0u;
      });
    }
  }
  __device__ __forceinline__ void store(Out* out, uint64_t idx, const State& st) {
    out[idx] = make_uint4(st.a, st.b, st.c, st.d);
  }
};

// Diagnostics: consumes all 16 words with a cheap fold (no MD5).
struct FoldHasher : Md5Hasher<false> {
  __device__ __forceinline__ void block(State& st, const uint4 (&w)[4]) {
    st.a ^= w[0].x ^ w[0].y ^ w[0].z ^ w[0].w;
    st.b ^= w[1].x ^ w[1].y ^ w[1].z ^ w[1].w;
    st.c ^= w[2].x ^ w[2].y ^ w[2].z ^ w[2].w;
    st.d ^= w[3].x ^ w[3].y ^ w[3].z ^ w[3].w;
  }
};

// ---------------------------------------------------------------------------
// CRC-32 (netcache crc32.c): zlib polynomial 0xEDB88320 (crc32.c:22),
// init ~0, final ~, slicing-by-8 little-endian form (crc32.c:186-240).  The
// eight 256-entry tables (crc32.c:251+) are built at compile time and copied
// into 8 KiB of LDS per workgroup; every byte costs one ds_read_b32.
// ---------------------------------------------------------------------------
struct CrcTables {
  uint32_t t[8][256];
  constexpr CrcTables() : t() {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
      t[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; ++i)
      for (int s = 1; s < 8; ++s) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFFu];
  }
};
__constant__ const CrcTables kCrcTables{};

// Zero-byte operators of the CRC-32 register, as zlib's crc32_combine builds
// them: m[l][i] = the register after 256 * 2^l zero bytes (l = 0..6: 256 B
// .. 16 KiB), started from the register 1 << i.  One zero byte is eight
// single-bit steps of the reflected polynomial (crc32.c:22); the larger
// operators are its repeated squares.  The register is linear in its start
// value and in the data, so the CRC of a message cut into segments is the
// XOR of each segment's register (the first started at ~0, the others at 0)
// advanced through the bytes after that segment (crc32_split).
struct CrcShift {
  uint32_t m[7][32];
  static constexpr uint32_t apply(const uint32_t (&op)[32], uint32_t v) {
    uint32_t r = 0;
    for (int i = 0; i < 32; ++i)
      if ((v >> i) & 1u) r ^= op[i];
    return r;
  }
  constexpr CrcShift() : m() {
    uint32_t cur[32] = {};
    for (int i = 0; i < 32; ++i) {
      uint32_t c = 1u << i;
      for (int k = 0; k < 8; ++k) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
      cur[i] = c;
    }
    for (int sq = 0; sq < 14; ++sq) {          // 2^(sq+1) zero bytes after square sq
      uint32_t nx[32] = {};
      for (int i = 0; i < 32; ++i) nx[i] = apply(cur, cur[i]);
      for (int i = 0; i < 32; ++i) cur[i] = nx[i];
      if (sq >= 7)
        for (int i = 0; i < 32; ++i) m[sq - 7][i] = cur[i];
    }
  }
};
__constant__ const CrcShift kCrcShift{};

// The register v advanced through 256 * 2^L zero bytes (L compile-time: the
// 32 columns fold into literals), 2 VALU per column.
template <int L>
__device__ __forceinline__ uint32_t crc_shift(uint32_t v) {
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 32; ++i) r ^= ((v >> i) & 1u) ? kCrcShift.m[L][i] : 0u;
  return r;
}

struct Crc32State {
  uint32_t c;
};

struct Crc32Hasher {
  using State = Crc32State;
  using Out = uint32_t;
  const uint32_t* tab;   // 2048 words in LDS: table s at tab + 256*s
  static constexpr int kLdsBytes = 8192;
  __device__ __forceinline__ void setup(uint8_t* lds) {
    uint32_t* t = reinterpret_cast<uint32_t*>(lds);
    const uint32_t* src = &kCrcTables.t[0][0];
    for (uint32_t k = threadIdx.x; k < 2048u; k += blockDim.x) t[k] = src[k];
    __syncthreads();
    tab = t;
  }
  __device__ __forceinline__ State init() { return State{0xFFFFFFFFu}; }
  // The 8 lookups fold through three 3-input XORs (v_bitop3_b32 0x96) and one
  // v_xor: 4 VALU instead of the 7 two-input XORs hipcc emits for a ^ chain.
  __device__ __forceinline__ uint32_t step8(uint32_t c, uint32_t one, uint32_t two) const {
    one ^= c;
    const uint32_t x = xor3(tab[0 * 256 + (two >> 24)], tab[1 * 256 + ((two >> 16) & 0xFFu)],
                            tab[2 * 256 + ((two >> 8) & 0xFFu)]);
    const uint32_t y = xor3(tab[3 * 256 + (two & 0xFFu)], tab[4 * 256 + (one >> 24)],
                            tab[5 * 256 + ((one >> 16) & 0xFFu)]);
    return xor3(x, tab[6 * 256 + ((one >> 8) & 0xFFu)], tab[7 * 256 + (one & 0xFFu)]) ^ y;
  }
  static __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
  }
  __device__ __forceinline__ void block(State& st, const uint4 (&w)[4]) {
    uint32_t c = st.c;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c = step8(c, w[k].x, w[k].y);
      c = step8(c, w[k].z, w[k].w);
    }
    st.c = c;
  }
  __device__ __forceinline__ void finish(State& st, const uint8_t* tail, uint32_t r, uint64_t) {
    uint32_t c = st.c;
    if (r) {
      uint32_t w[16];
      load_tail(tail, r, w);
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if ((uint32_t)(8 * j + 8) <= r) c = step8(c, w[2 * j], w[2 * j + 1]);
      // remaining 1..7 bytes, one at a time (crc32.c:236-238)
      const uint32_t done = r & ~7u;
#pragma unroll
      for (int b = 0; b < 7; ++b) {
        const uint32_t pos = done + (uint32_t)b;
        if (pos < r) {
          uint32_t wd = w[0];
#pragma unroll
          for (int j = 1; j < 16; ++j)
            if ((uint32_t)j == (pos >> 2)) wd = w[j];
          const uint32_t byte = (wd >> (8 * (pos & 3u))) & 0xFFu;
          c = tab[(c ^ byte) & 0xFFu] ^ (c >> 8);
        }
      }
    }
    st.c = ~c;
  }
  __device__ __forceinline__ void store(Out* out, uint64_t idx, const State& st) {
    out[idx] = st.c;
  }
};

// ---------------------------------------------------------------------------
// CRC-32, slicing-by-4 over LANE-PRIVATE table copies.  Every table entry is
// stored K times, copy c in bank c (LDS word e*K + c), and lane l reads copy
// l % K, so a ds_read_b32 lane group (32 lanes, bank = dword mod 32,
// MI355X_MICROARCH §LDS) hits at most 32/K lanes per bank whatever bytes
// the lanes look up: conflict-free for K = 32 (2 LDS cycles per wave
// lookup), where the shared 8 KiB tables of Crc32Hasher average ~3.5-way.
// Same polynomial and byte order as crc32.c:186-240 (4 bytes per step).
// LDS: 4 tables x 256 entries x K copies x 4 B = K KiB * 4 (128 KiB at K=32).
// Address bits (K=32): lane copy 2..6, entry 7..14, table 15..16 -- disjoint,
// so an address is one OR/shift; table 1/3 come from the ds_read offset.
// ---------------------------------------------------------------------------
template <int K>
struct Crc32LaneHasher {
  static_assert(K == 16 || K == 32, "K copies: 16 or 32");
  using State = Crc32State;
  using Out = uint32_t;
  static constexpr int kLdsBytes = 4 * 256 * K * 4;
  static constexpr uint32_t kEntryShift = K == 32 ? 7 : 6;     // log2(K * 4)
  static constexpr uint32_t kTableBytes = 256u * K * 4u;
  const uint8_t* lds;
  uint32_t lane4;                      // (lane % K) * 4
  __device__ __forceinline__ void setup(uint8_t* l) {
    uint32_t* t = reinterpret_cast<uint32_t*>(l);
    const uint32_t* src = &kCrcTables.t[0][0];
    for (uint32_t k = threadIdx.x; k < 4u * 256u * K; k += blockDim.x)
      t[k] = src[k / K];               // table s entry e copy c at ((s*256 + e)*K + c)
    __syncthreads();
    lds = l;
    lane4 = (threadIdx.x % K) * 4u;
  }
  __device__ __forceinline__ uint32_t look(uint32_t table, uint32_t byte) const {
    return *reinterpret_cast<const uint32_t*>(lds + table * kTableBytes +
                                              ((byte << kEntryShift) | lane4));
  }
  __device__ __forceinline__ uint32_t step4(uint32_t c, uint32_t w) const {
    c ^= w;
    return look(0, c >> 24) ^ look(1, (c >> 16) & 0xFFu) ^ look(2, (c >> 8) & 0xFFu) ^
           look(3, c & 0xFFu);
  }
  __device__ __forceinline__ State init() { return State{0xFFFFFFFFu}; }
  __device__ __forceinline__ void block(State& st, const uint4 (&w)[4]) {
    uint32_t c = st.c;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c = step4(c, w[k].x);
      c = step4(c, w[k].y);
      c = step4(c, w[k].z);
      c = step4(c, w[k].w);
    }
    st.c = c;
  }
  __device__ __forceinline__ void finish(State& st, const uint8_t* tail, uint32_t r, uint64_t) {
    uint32_t c = st.c;
    if (r) {
      uint32_t w[16];
      load_tail(tail, r, w);
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if ((uint32_t)(4 * j + 4) <= r) c = step4(c, w[j]);
      const uint32_t done = r & ~3u;
      uint32_t wd = w[0];
#pragma unroll
      for (int j = 1; j < 16; ++j)
        if ((uint32_t)j == (done >> 2)) wd = w[j];
#pragma unroll
      for (int b = 0; b < 3; ++b)      // the last 1..3 bytes, one at a time
        if (done + (uint32_t)b < r) c = look(0, (c ^ (wd >> (8 * b))) & 0xFFu) ^ (c >> 8);
    }
    st.c = ~c;
  }
  __device__ __forceinline__ void store(Out* out, uint64_t idx, const State& st) {
    out[idx] = st.c;
  }
};

// Slicing-by-4 over 16 lane copies laid out so ONE v_perm_b32 forms each
// lookup address: entry e of table t, copy c at word e*64 + t*16 + c, i.e.
// byte address (e << 8) | (t << 6) | (c << 2) (64 KiB).  v_perm_b32 drops the
// index byte into bits 8..15 next to a per-lane constant byte (t << 6) |
// (c << 2).  ds_read_b32 banks on word mod 32 = (t & 1) * 16 + c over 32-lane
// groups (MI355X_MICROARCH §LDS), so if every lane looked up the same table
// per instruction, lanes l and l + 16 (same copy) would always share a bank
// (the round-1 fixed 2-way conflict, profiles/r01_pmc_summary_final_box2.json).
// Instead lanes with bit 4 set take the four tables in the order 1, 0, 3, 2:
// in every lookup instruction lanes 0-15 read an even (odd) table and lanes
// 16-31 the odd (even) one, i.e. the two halves of the group sit in opposite
// bank halves -- conflict-free.  The four lookups are XORed, so the order is
// free; each lane holds its per-slot constant byte and v_perm selector in
// VGPRs (the table no longer rides in the ds_read immediate).
struct Crc32PermHasher {
  using State = Crc32State;
  using Out = uint32_t;
  static constexpr int kLdsBytes = 256 * 64 * 4;
  const uint8_t* lds;
  uint32_t lane4;                      // (lane % 16) * 4: table 0, for the byte-wise tail
  uint32_t lb[4], sel[4];              // slot k: (t << 6) | (c << 2), and the v_perm selector
  __device__ __forceinline__ void setup(uint8_t* l) {
    // the 16 copies of one (table, entry) value are 64 contiguous bytes: one
    // load and four 16-B LDS writes per value, 1,024 values per workgroup
    // (a load per dword cost a small launch ~2 us of L2 round trips)
    uint4* t = reinterpret_cast<uint4*>(l);
    for (uint32_t j = threadIdx.x; j < 1024u; j += blockDim.x) {
      const uint32_t v = kCrcTables.t[j & 3u][j >> 2];
      const uint4 q = make_uint4(v, v, v, v);
#pragma unroll
      for (int c = 0; c < 4; ++c) t[4u * j + c] = q;
    }
    __syncthreads();
    lds = l;
    lane4 = (threadIdx.x & 15u) * 4u;
    const uint32_t h = (threadIdx.x >> 4) & 1u;
#pragma unroll
    for (uint32_t k = 0; k < 4; ++k) {
      const uint32_t tab = k ^ h;                   // this lane's table in slot k
      lb[k] = (tab << 6) | lane4;
      // byte 0 <- lb byte 0, byte 1 <- c byte (3 - tab), bytes 2-3 <- 0
      sel[k] = 0x0C0C0000u | ((4u + 3u - tab) << 8);
    }
  }
  __device__ __forceinline__ uint32_t slot(uint32_t c, int k) const {
    const uint32_t addr = __builtin_amdgcn_perm(c, lb[k], sel[k]);
    return *reinterpret_cast<const uint32_t*>(lds + addr);
  }
  static __device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
    return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
  }
  __device__ __forceinline__ uint32_t step4(uint32_t c, uint32_t w) const {
    c ^= w;      // T0[b3] ^ T1[b2] ^ T2[b1] ^ T3[b0] (crc32.c slicing), in this lane's slot order
    return xor3(slot(c, 0), slot(c, 1), slot(c, 2)) ^ slot(c, 3);
  }
  // table 0, index = byte 0 of x (the byte-wise tail, crc32.c:236-238)
  __device__ __forceinline__ uint32_t look0(uint32_t x) const {
    const uint32_t addr = __builtin_amdgcn_perm(x, lane4, 0x0C0C0400u);
    return *reinterpret_cast<const uint32_t*>(lds + addr);
  }
  __device__ __forceinline__ State init() { return State{0xFFFFFFFFu}; }
  __device__ __forceinline__ void block(State& st, const uint4 (&w)[4]) {
    uint32_t c = st.c;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      c = step4(c, w[k].x);
      c = step4(c, w[k].y);
      c = step4(c, w[k].z);
      c = step4(c, w[k].w);
    }
    st.c = c;
  }
  __device__ __forceinline__ void finish(State& st, const uint8_t* tail, uint32_t r, uint64_t) {
    uint32_t c = st.c;
    if (r) {
      uint32_t w[16];
      load_tail(tail, r, w);
#pragma unroll
      for (int j = 0; j < 16; ++j)
        if ((uint32_t)(4 * j + 4) <= r) c = step4(c, w[j]);
      const uint32_t done = r & ~3u;
      uint32_t wd = w[0];
#pragma unroll
      for (int j = 1; j < 16; ++j)
        if ((uint32_t)j == (done >> 2)) wd = w[j];
#pragma unroll
      for (int b = 0; b < 3; ++b)      // the last 1..3 bytes, one at a time (crc32.c:236-238)
        if (done + (uint32_t)b < r) c = look0(c ^ (wd >> (8 * b))) ^ (c >> 8);
    }
    st.c = ~c;
  }
  __device__ __forceinline__ void store(Out* out, uint64_t idx, const State& st) {
    out[idx] = st.c;
  }
};

}  // namespace md5hip
