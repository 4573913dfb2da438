// md5_core.h -- the MD5 compression as gfx950 VALU code.
//
// Re-states the block transform of sproxy's md5.c (MD5Transform, md5.c:63-146;
// round functions md5.c:46-52; MD5STEP md5.c:55-56) for ONE lane = ONE chunk.
// Every step is written so that hipcc lowers it to the short CDNA4 sequence
//
//     v_add3_u32   t  = a + M + K            (off the dependency chain)
//     v_bfi_b32 / v_xor3_b32 / (v_bfi_b32 + v_xad_u32)     f(b, c, d)
//     v_add_u32    t += f
//     v_alignbit_b32 t = rotl(t, s)
//     v_add_u32    a  = b + t
//
// i.e. 5 VALU ops per step, 4 of them on the serial chain; the padding-only
// final block folds M + K into one literal.  See DESIGN.md "VALU budget".
#pragma once
#include <stdint.h>

namespace md5hip {

struct State {
  uint32_t a, b, c, d;
};

__device__ __forceinline__ State initial_state() {
  // md5.c:156-159
  return State{0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
}

__device__ __forceinline__ uint32_t rotl(uint32_t x, int s) {
  return __builtin_amdgcn_alignbit(x, x, 32 - s);
}
// Round functions md5.c:49-52 as ONE gfx950 v_bitop3_b32 each (3-input LUT,
// bit index = S0<<2 | S1<<1 | S2):
//   F1 = x ? y : z            -> 0xCA
//   F2 = F1(z, x, y) = z ? x : y -> 0xE4
//   F3 = x ^ y ^ z            -> 0x96
//   F4 = y ^ (x | ~z)         -> 0x39
__device__ __forceinline__ uint32_t f1(uint32_t x, uint32_t y, uint32_t z) {
  return __builtin_amdgcn_bitop3_b32(x, y, z, 0xCA);
}
__device__ __forceinline__ uint32_t f2(uint32_t x, uint32_t y, uint32_t z) {
  return __builtin_amdgcn_bitop3_b32(x, y, z, 0xE4);
}
__device__ __forceinline__ uint32_t f3(uint32_t x, uint32_t y, uint32_t z) {
  return __builtin_amdgcn_bitop3_b32(x, y, z, 0x96);
}
__device__ __forceinline__ uint32_t f4(uint32_t x, uint32_t y, uint32_t z) {
  return __builtin_amdgcn_bitop3_b32(x, y, z, 0x39);
}

// MD5STEP (md5.c:55-56): w += f(x,y,z) + data; w = rotl(w, s); w += x.
// Cost model (profiles/r01_valu_rate_*): v_add_u32 / v_bitop3 ~2.8 cycles,
// v_add3_u32 / v_alignbit ~4.4.  Two orderings of the same 5 instructions:
//  kLat = false: hipcc's choice, add(w,M) off the chain, add3(.,F,K) on it
//                (chain: bitop3 -> add3 -> alignbit -> add, two slow ops);
//  kLat = true : add3(w,M,K) off the chain (an empty asm pins the partial
//                sum so it is not re-associated with F), fast add on it
//                (chain: bitop3 -> add -> alignbit -> add, one slow op).
// The instruction count is equal; kLat shortens the serial chain, which is
// what bounds a lane hashing a long chunk alone (config C3).
template <bool kLat>
__device__ __forceinline__ uint32_t md5_sum(uint32_t w, uint32_t m, uint32_t k, uint32_t f) {
  if constexpr (kLat) {
    uint32_t t = w + m + k;
    asm("" : "+v"(t));
    return t + f;
  } else {
    return (w + m + k) + f;
  }
}

#define MD5HIP_STEP(F, w, x, y, z, m, k, s) \
  w = x + rotl(md5_sum<kLat>(w, (m), (k), F(x, y, z)), s)

// Round 3 (H = x ^ y ^ z, md5.c:51) two steps at a time (kX3): step k uses
// H(b, c, d) and step k+1 H(a', b, c), so b ^ c serves both, and each step's
// "+ H" becomes one v_xad_u32 ((p ^ q) + t): 3 VALU instead of 4 per two
// steps (316 instead of 324 per block), and step k+1's serial chain is
// a' -> xad -> alignbit -> add.
template <bool kLat>
__device__ __forceinline__ uint32_t md5_xsum(uint32_t w, uint32_t m, uint32_t k, uint32_t p,
                                             uint32_t q) {
  const uint32_t t = w + m + k;
  uint32_t r;   // hipcc splits (p ^ q) + t into v_xor + v_add; ask for v_xad_u32
  asm("v_xad_u32 %0, %1, %2, %3" : "=v"(r) : "v"(p), "v"(q), "v"(t));
  return r;
}
#define MD5HIP_STEP3_PAIR(w1, w2, x, y, m1, k1, s1, m2, k2, s2) \
  { const uint32_t cx = x ^ y;                                   \
    w1 = x + rotl(md5_xsum<kLat>(w1, (m1), (k1), cx, w2), s1);     \
    w2 = w1 + rotl(md5_xsum<kLat>(w2, (m2), (k2), cx, w1), s2); }

// One 64-byte block, message words m[0..15] little-endian (byteReverse is a
// no-op on little-endian gfx950, md5.c:24-25).  The 64 K literals are the
// RFC 1321 T table (md5.c:74-139).
template <bool kLat = false, bool kX3 = true, typename MsgFn>
__device__ __forceinline__ void compress(State& st, MsgFn M) {
  uint32_t a = st.a, b = st.b, c = st.c, d = st.d;
  MD5HIP_STEP(f1, a, b, c, d, M(0), 0xd76aa478u, 7);
  MD5HIP_STEP(f1, d, a, b, c, M(1), 0xe8c7b756u, 12);
  MD5HIP_STEP(f1, c, d, a, b, M(2), 0x242070dbu, 17);
  MD5HIP_STEP(f1, b, c, d, a, M(3), 0xc1bdceeeu, 22);
  MD5HIP_STEP(f1, a, b, c, d, M(4), 0xf57c0fafu, 7);
  MD5HIP_STEP(f1, d, a, b, c, M(5), 0x4787c62au, 12);
  MD5HIP_STEP(f1, c, d, a, b, M(6), 0xa8304613u, 17);
  MD5HIP_STEP(f1, b, c, d, a, M(7), 0xfd469501u, 22);
  MD5HIP_STEP(f1, a, b, c, d, M(8), 0x698098d8u, 7);
  MD5HIP_STEP(f1, d, a, b, c, M(9), 0x8b44f7afu, 12);
  MD5HIP_STEP(f1, c, d, a, b, M(10), 0xffff5bb1u, 17);
  MD5HIP_STEP(f1, b, c, d, a, M(11), 0x895cd7beu, 22);
  MD5HIP_STEP(f1, a, b, c, d, M(12), 0x6b901122u, 7);
  MD5HIP_STEP(f1, d, a, b, c, M(13), 0xfd987193u, 12);
  MD5HIP_STEP(f1, c, d, a, b, M(14), 0xa679438eu, 17);
  MD5HIP_STEP(f1, b, c, d, a, M(15), 0x49b40821u, 22);

  MD5HIP_STEP(f2, a, b, c, d, M(1), 0xf61e2562u, 5);
  MD5HIP_STEP(f2, d, a, b, c, M(6), 0xc040b340u, 9);
  MD5HIP_STEP(f2, c, d, a, b, M(11), 0x265e5a51u, 14);
  MD5HIP_STEP(f2, b, c, d, a, M(0), 0xe9b6c7aau, 20);
  MD5HIP_STEP(f2, a, b, c, d, M(5), 0xd62f105du, 5);
  MD5HIP_STEP(f2, d, a, b, c, M(10), 0x02441453u, 9);
  MD5HIP_STEP(f2, c, d, a, b, M(15), 0xd8a1e681u, 14);
  MD5HIP_STEP(f2, b, c, d, a, M(4), 0xe7d3fbc8u, 20);
  MD5HIP_STEP(f2, a, b, c, d, M(9), 0x21e1cde6u, 5);
  MD5HIP_STEP(f2, d, a, b, c, M(14), 0xc33707d6u, 9);
  MD5HIP_STEP(f2, c, d, a, b, M(3), 0xf4d50d87u, 14);
  MD5HIP_STEP(f2, b, c, d, a, M(8), 0x455a14edu, 20);
  MD5HIP_STEP(f2, a, b, c, d, M(13), 0xa9e3e905u, 5);
  MD5HIP_STEP(f2, d, a, b, c, M(2), 0xfcefa3f8u, 9);
  MD5HIP_STEP(f2, c, d, a, b, M(7), 0x676f02d9u, 14);
  MD5HIP_STEP(f2, b, c, d, a, M(12), 0x8d2a4c8au, 20);

  if constexpr (kX3) {
    // pair (a; b,c,d), (d; a,b,c): shared b ^ c; pair (c; d,a,b), (b; c,d,a): shared d ^ a
    MD5HIP_STEP3_PAIR(a, d, b, c, M(5), 0xfffa3942u, 4, M(8), 0x8771f681u, 11);
    MD5HIP_STEP3_PAIR(c, b, d, a, M(11), 0x6d9d6122u, 16, M(14), 0xfde5380cu, 23);
    MD5HIP_STEP3_PAIR(a, d, b, c, M(1), 0xa4beea44u, 4, M(4), 0x4bdecfa9u, 11);
    MD5HIP_STEP3_PAIR(c, b, d, a, M(7), 0xf6bb4b60u, 16, M(10), 0xbebfbc70u, 23);
    MD5HIP_STEP3_PAIR(a, d, b, c, M(13), 0x289b7ec6u, 4, M(0), 0xeaa127fau, 11);
    MD5HIP_STEP3_PAIR(c, b, d, a, M(3), 0xd4ef3085u, 16, M(6), 0x04881d05u, 23);
    MD5HIP_STEP3_PAIR(a, d, b, c, M(9), 0xd9d4d039u, 4, M(12), 0xe6db99e5u, 11);
    MD5HIP_STEP3_PAIR(c, b, d, a, M(15), 0x1fa27cf8u, 16, M(2), 0xc4ac5665u, 23);
  } else {
  MD5HIP_STEP(f3, a, b, c, d, M(5), 0xfffa3942u, 4);
  MD5HIP_STEP(f3, d, a, b, c, M(8), 0x8771f681u, 11);
  MD5HIP_STEP(f3, c, d, a, b, M(11), 0x6d9d6122u, 16);
  MD5HIP_STEP(f3, b, c, d, a, M(14), 0xfde5380cu, 23);
  MD5HIP_STEP(f3, a, b, c, d, M(1), 0xa4beea44u, 4);
  MD5HIP_STEP(f3, d, a, b, c, M(4), 0x4bdecfa9u, 11);
  MD5HIP_STEP(f3, c, d, a, b, M(7), 0xf6bb4b60u, 16);
  MD5HIP_STEP(f3, b, c, d, a, M(10), 0xbebfbc70u, 23);
  MD5HIP_STEP(f3, a, b, c, d, M(13), 0x289b7ec6u, 4);
  MD5HIP_STEP(f3, d, a, b, c, M(0), 0xeaa127fau, 11);
  MD5HIP_STEP(f3, c, d, a, b, M(3), 0xd4ef3085u, 16);
  MD5HIP_STEP(f3, b, c, d, a, M(6), 0x04881d05u, 23);
  MD5HIP_STEP(f3, a, b, c, d, M(9), 0xd9d4d039u, 4);
  MD5HIP_STEP(f3, d, a, b, c, M(12), 0xe6db99e5u, 11);
  MD5HIP_STEP(f3, c, d, a, b, M(15), 0x1fa27cf8u, 16);
  MD5HIP_STEP(f3, b, c, d, a, M(2), 0xc4ac5665u, 23);
  }

  MD5HIP_STEP(f4, a, b, c, d, M(0), 0xf4292244u, 6);
  MD5HIP_STEP(f4, d, a, b, c, M(7), 0x432aff97u, 10);
  MD5HIP_STEP(f4, c, d, a, b, M(14), 0xab9423a7u, 15);
  MD5HIP_STEP(f4, b, c, d, a, M(5), 0xfc93a039u, 21);
  MD5HIP_STEP(f4, a, b, c, d, M(12), 0x655b59c3u, 6);
  MD5HIP_STEP(f4, d, a, b, c, M(3), 0x8f0ccc92u, 10);
  MD5HIP_STEP(f4, c, d, a, b, M(10), 0xffeff47du, 15);
  MD5HIP_STEP(f4, b, c, d, a, M(1), 0x85845dd1u, 21);
  MD5HIP_STEP(f4, a, b, c, d, M(8), 0x6fa87e4fu, 6);
  MD5HIP_STEP(f4, d, a, b, c, M(15), 0xfe2ce6e0u, 10);
  MD5HIP_STEP(f4, c, d, a, b, M(6), 0xa3014314u, 15);
  MD5HIP_STEP(f4, b, c, d, a, M(13), 0x4e0811a1u, 21);
  MD5HIP_STEP(f4, a, b, c, d, M(4), 0xf7537e82u, 6);
  MD5HIP_STEP(f4, d, a, b, c, M(11), 0xbd3af235u, 10);
  MD5HIP_STEP(f4, c, d, a, b, M(2), 0x2ad7d2bbu, 15);
  MD5HIP_STEP(f4, b, c, d, a, M(9), 0xeb86d391u, 21);

  st.a += a;  // feed-forward, md5.c:142-145
  st.b += b;
  st.c += c;
  st.d += d;
}

#undef MD5HIP_STEP
#undef MD5HIP_STEP3_PAIR

// Compress 16 words held in four uint4 registers.
template <bool kLat = false, bool kX3 = true>
__device__ __forceinline__ void compress_regs(State& st, const uint4 (&w)[4]) {
  compress<kLat, kX3>(st, [&](int i) __attribute__((always_inline)) -> uint32_t {
    const uint4& q = w[i >> 2];
    switch (i & 3) {
      case 0: return q.x;
      case 1: return q.y;
      case 2: return q.z;
      default: return q.w;
    }
  });
}

// The final padding block of a message whose length is a multiple of 64:
// 0x80, 52 zero bytes, then the 64-bit bit count (md5.c:221-261).  All but
// words 14/15 are compile-time constants, so M + K folds into one literal.
template <bool kLat = false, bool kX3 = true>
__device__ __forceinline__ void compress_pad_only(State& st, uint32_t bits_lo, uint32_t bits_hi) {
  compress<kLat, kX3>(st, [&](int i) __attribute__((always_inline)) -> uint32_t {
    return i == 0 ? 0x80u : i == 14 ? bits_lo : i == 15 ? bits_hi : 0u;
  });
}

}  // namespace md5hip
