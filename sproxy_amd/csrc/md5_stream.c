/*
 * md5_stream.c -- the per-message MD5Init / MD5Update / MD5Final entries of
 * libmd5hip.so (include/md5.h), i.e. the ABI of /root/reference/md5.h:31-51.
 *
 * These serve sproxy's per-request callers (soluri2.c:711-713 token check,
 * streaming.c:7840-7842 HLS key), which hash tens to hundreds of bytes on an
 * MHD worker thread; they stay on the host CPU by design (a device round trip
 * costs more than the whole hash).  Everything chunk-sized goes through the
 * batched device entries of include/md5hip.h instead.
 *
 * Behaviour follows md5.c:153-265 exactly: 32-bit `len`, 64-bit bit counter
 * kept as two u32 words with carry (md5.c:179-182), partial block buffered in
 * ctx->in, MD5Final pads 0x80 / zeros / LE bit count and zeroes the context.
 */
#include <stdint.h>
#include <string.h>

#include "../../include/md5.h"

_Static_assert(sizeof(struct MD5Context) == 88, "md5.h:33-38 layout");

static const uint32_t k_add[64] = {
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

static inline uint32_t rol32(uint32_t v, unsigned s) { return (v << s) | (v >> (32u - s)); }

static inline uint32_t get_le32(const unsigned char *p)
{
    uint32_t v;
    memcpy(&v, p, 4); /* little-endian host; the reference's HIGHFIRST path is not needed */
    return v;
}

/* One 64-byte block.  Each step is written for a short serial chain (the
 * host MD5 is one dependent chain, so latency, not throughput, bounds it):
 * the parts of f that do not involve the newest word are computed off the
 * chain, as is w + M + K, so the chain per step is f-tail -> add -> rotate ->
 * add.  Round 2 adds its two disjoint halves (G = (b & d) + (c & ~d)) so only
 * b & d waits for b.  The rounds are loops the compiler fully unrolls
 * (constant tables fold into immediates). */
#define STEP1(a, b, c, d, m, k, s) \
    { uint32_t t_ = a + (m) + (k); t_ += d ^ (b & (c ^ d)); a = b + rol32(t_, s); }
#define STEP2(a, b, c, d, m, k, s) \
    { uint32_t t_ = a + (m) + (k) + (c & ~d); t_ += b & d; a = b + rol32(t_, s); }
#define STEP3(a, b, c, d, m, k, s) \
    { uint32_t t_ = a + (m) + (k); t_ += b ^ (c ^ d); a = b + rol32(t_, s); }
#define STEP4(a, b, c, d, m, k, s) \
    { uint32_t t_ = a + (m) + (k); t_ += c ^ (b | ~d); a = b + rol32(t_, s); }

static void md5_blocks(uint32_t st[4], const unsigned char *p, size_t nblocks)
{
    while (nblocks--) {
        uint32_t m[16];
        for (int i = 0; i < 16; i++) m[i] = get_le32(p + 4 * i);
        uint32_t a = st[0], b = st[1], c = st[2], d = st[3];
#pragma GCC unroll 16
        for (int i = 0; i < 16; i += 4) {
            STEP1(a, b, c, d, m[i], k_add[i], 7);
            STEP1(d, a, b, c, m[i + 1], k_add[i + 1], 12);
            STEP1(c, d, a, b, m[i + 2], k_add[i + 2], 17);
            STEP1(b, c, d, a, m[i + 3], k_add[i + 3], 22);
        }
#pragma GCC unroll 16
        for (int i = 0; i < 16; i += 4) {
            STEP2(a, b, c, d, m[(5 * i + 1) & 15], k_add[16 + i], 5);
            STEP2(d, a, b, c, m[(5 * i + 6) & 15], k_add[17 + i], 9);
            STEP2(c, d, a, b, m[(5 * i + 11) & 15], k_add[18 + i], 14);
            STEP2(b, c, d, a, m[(5 * i) & 15], k_add[19 + i], 20);
        }
#pragma GCC unroll 16
        for (int i = 0; i < 16; i += 4) {
            STEP3(a, b, c, d, m[(3 * i + 5) & 15], k_add[32 + i], 4);
            STEP3(d, a, b, c, m[(3 * i + 8) & 15], k_add[33 + i], 11);
            STEP3(c, d, a, b, m[(3 * i + 11) & 15], k_add[34 + i], 16);
            STEP3(b, c, d, a, m[(3 * i + 14) & 15], k_add[35 + i], 23);
        }
#pragma GCC unroll 16
        for (int i = 0; i < 16; i += 4) {
            STEP4(a, b, c, d, m[(7 * i) & 15], k_add[48 + i], 6);
            STEP4(d, a, b, c, m[(7 * i + 7) & 15], k_add[49 + i], 10);
            STEP4(c, d, a, b, m[(7 * i + 14) & 15], k_add[50 + i], 15);
            STEP4(b, c, d, a, m[(7 * i + 21) & 15], k_add[51 + i], 21);
        }
        st[0] += a;
        st[1] += b;
        st[2] += c;
        st[3] += d;
        p += 64;
    }
}
#undef STEP1
#undef STEP2
#undef STEP3
#undef STEP4

void MD5Init(struct MD5Context *ctx)
{
    static const uint32_t iv[4] = {0x67452301u, 0xefcdab89u, 0x98badcfeu, 0x10325476u};
    memcpy(ctx->buf, iv, sizeof iv);
    ctx->bits[0] = ctx->bits[1] = 0;
}

void MD5Update(struct MD5Context *ctx, const void *buf, unsigned len)
{
    const unsigned char *src = (const unsigned char *)buf;
    const uint32_t old = ctx->bits[0];
    const unsigned fill = (old >> 3) & 63u;
    ctx->bits[0] = old + ((uint32_t)len << 3);
    ctx->bits[1] += (len >> 29) + (ctx->bits[0] < old);
    if (fill) {
        const unsigned room = 64u - fill;
        if (len < room) {
            memcpy(ctx->in + fill, src, len);
            return;
        }
        memcpy(ctx->in + fill, src, room);
        md5_blocks(ctx->buf, ctx->in, 1);
        src += room;
        len -= room;
    }
    const unsigned whole = len >> 6;
    md5_blocks(ctx->buf, src, whole);
    src += len & ~63u;
    /* md5.c:204-214 copies every whole block through ctx->in before it is
     * transformed, so in[] ends as the last whole block with the tail copied
     * over its first bytes.  Hashing straight from the source and copying that
     * block once leaves the same 88 bytes. */
    if (whole)
        memcpy(ctx->in, src - 64, 64);
    memcpy(ctx->in, src, len & 63u);
}

void MD5Final(unsigned char digest[MD5_DIGEST_SIZE], struct MD5Context *ctx)
{
    const unsigned used = (ctx->bits[0] >> 3) & 63u;
    ctx->in[used] = 0x80;
    if (used >= 56) { /* no room for the length: pad this block out, then one more */
        memset(ctx->in + used + 1, 0, 63u - used);
        md5_blocks(ctx->buf, ctx->in, 1);
        memset(ctx->in, 0, 56);
    } else {
        memset(ctx->in + used + 1, 0, 55u - used);
    }
    memcpy(ctx->in + 56, &ctx->bits[0], 4);
    memcpy(ctx->in + 60, &ctx->bits[1], 4);
    md5_blocks(ctx->buf, ctx->in, 1);
    memcpy(digest, ctx->buf, 16);
    memset(ctx, 0, sizeof *ctx);
}
