/*
 * oracle/md5_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker).
 *
 * Clean-room CPU restatement of sproxy's in-tree MD5 (Colin Plumb's public
 * domain md5.c, /root/reference/md5.c + md5.h).  Only tests/, smoke() in
 * __graft_entry__.py and the cpu_baseline leg of bench.py may load this
 * library; the product (sproxy_amd/) never links or calls it.
 *
 * Parity is PINNED: tests/test_oracle.py checks this file against every
 * golden vector in tests/golden/ (RFC 1321 suite, the MHD test_md5.c units,
 * curl unit1601, edge lengths 0..1 MiB, the 65,536 x 16 KiB batch fold), and
 * those fixtures were produced by the reference md5.c itself compiled from
 * /root/reference (oracle/Makefile -> oracle/_ref/, tests/golden/make_golden.py).
 *
 * Written table-driven on purpose (the reference is 64 unrolled macro steps),
 * so that a bug shared by the two shapes is unlikely.
 *
 *   reference                        here
 *   md5.c:46-52  F1..F4             o_round_fn()
 *   md5.c:55-56  MD5STEP            o_compress() loop body
 *   md5.c:63-146 MD5Transform       o_compress()
 *   md5.c:153-163 MD5Init           oracle_md5_init()
 *   md5.c:169-215 MD5Update         oracle_md5_update()
 *   md5.c:221-265 MD5Final          oracle_md5_final()
 *   md5.h:33-38  struct MD5Context  struct oracle_md5_ctx (same 88-byte layout)
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>

struct oracle_md5_ctx {          /* md5.h:33-38: buf[4], bits[2], in[64] */
    uint32_t state[4];
    uint32_t nbits[2];           /* [0] low word, [1] high word (md5.c:179-182) */
    uint8_t  pending[64];
};

/* Additive constants, RFC 1321 §3.4 table T[1..64] (= the literals of md5.c:74-139). */
static const uint32_t o_T[64] = {
    0xd76aa478u, 0xe8c7b756u, 0x242070dbu, 0xc1bdceeeu, 0xf57c0fafu, 0x4787c62au,
    0xa8304613u, 0xfd469501u, 0x698098d8u, 0x8b44f7afu, 0xffff5bb1u, 0x895cd7beu,
    0x6b901122u, 0xfd987193u, 0xa679438eu, 0x49b40821u, 0xf61e2562u, 0xc040b340u,
    0x265e5a51u, 0xe9b6c7aau, 0xd62f105du, 0x02441453u, 0xd8a1e681u, 0xe7d3fbc8u,
    0x21e1cde6u, 0xc33707d6u, 0xf4d50d87u, 0x455a14edu, 0xa9e3e905u, 0xfcefa3f8u,
    0x676f02d9u, 0x8d2a4c8au, 0xfffa3942u, 0x8771f681u, 0x6d9d6122u, 0xfde5380cu,
    0xa4beea44u, 0x4bdecfa9u, 0xf6bb4b60u, 0xbebfbc70u, 0x289b7ec6u, 0xeaa127fau,
    0xd4ef3085u, 0x04881d05u, 0xd9d4d039u, 0xe6db99e5u, 0x1fa27cf8u, 0xc4ac5665u,
    0xf4292244u, 0x432aff97u, 0xab9423a7u, 0xfc93a039u, 0x655b59c3u, 0x8f0ccc92u,
    0xffeff47du, 0x85845dd1u, 0x6fa87e4fu, 0xfe2ce6e0u, 0xa3014314u, 0x4e0811a1u,
    0xf7537e82u, 0xbd3af235u, 0x2ad7d2bbu, 0xeb86d391u};

/* Per-round rotate amounts (md5.c step literals 7/12/17/22, 5/9/14/20, ...). */
static const unsigned o_S[4][4] = {
    {7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};

/* Round functions, md5.c:49-52. */
static uint32_t o_round_fn(int round, uint32_t x, uint32_t y, uint32_t z)
{
    switch (round) {
    case 0:  return z ^ (x & (y ^ z));  /* F1 */
    case 1:  return y ^ (z & (x ^ y));  /* F2 = F1(z, x, y) */
    case 2:  return x ^ y ^ z;          /* F3 */
    default: return y ^ (x | ~z);       /* F4 */
    }
}

/* Message-word schedule: round r, step i (md5.c:74-139 'in[...]' indices). */
static unsigned o_word_index(int round, unsigned i)
{
    switch (round) {
    case 0:  return i;
    case 1:  return (5u * i + 1u) & 15u;
    case 2:  return (3u * i + 5u) & 15u;
    default: return (7u * i) & 15u;
    }
}

static uint32_t o_load_le32(const uint8_t *p)
{
    return (uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 |
           (uint32_t)p[3] << 24;
}

/* MD5Transform, md5.c:63-146.  The 64-byte block is read little-endian
 * (byteReverse is a no-op on LE hosts, md5.c:24-25). */
static void o_compress(uint32_t st[4], const uint8_t block[64])
{
    uint32_t m[16];
    uint32_t v[4];   /* v[0..3] = a, b, c, d */
    for (unsigned k = 0; k < 16; k++)
        m[k] = o_load_le32(block + 4 * k);
    for (unsigned k = 0; k < 4; k++)
        v[k] = st[k];
    for (unsigned step = 0; step < 64; step++) {
        int r = (int)(step >> 4);
        unsigned i = step & 15u;
        /* the register being written rotates a, d, c, b (md5.c:74-77) */
        unsigned w = (4u - (step & 3u)) & 3u;
        uint32_t x = v[(w + 1) & 3], y = v[(w + 2) & 3], z = v[(w + 3) & 3];
        uint32_t t = v[w] + o_round_fn(r, x, y, z) + m[o_word_index(r, i)] + o_T[step];
        unsigned s = o_S[r][step & 3u];
        t = (t << s) | (t >> (32u - s));
        v[w] = t + x;                      /* MD5STEP, md5.c:55-56 */
    }
    for (unsigned k = 0; k < 4; k++)       /* md5.c:142-145 */
        st[k] += v[k];
}

void oracle_md5_init(struct oracle_md5_ctx *c)
{
    c->state[0] = 0x67452301u;   /* md5.c:156-159 */
    c->state[1] = 0xefcdab89u;
    c->state[2] = 0x98badcfeu;
    c->state[3] = 0x10325476u;
    c->nbits[0] = 0;
    c->nbits[1] = 0;
}

void oracle_md5_update(struct oracle_md5_ctx *c, const void *data, unsigned len)
{
    const uint8_t *p = (const uint8_t *)data;
    uint32_t lo = c->nbits[0];
    unsigned have = (lo >> 3) & 63u;           /* md5.c:184 */
    /* 64-bit bit counter with carry, md5.c:179-182 */
    c->nbits[0] = lo + ((uint32_t)len << 3);
    if (c->nbits[0] < lo)
        c->nbits[1]++;
    c->nbits[1] += len >> 29;

    while (len > 0) {
        unsigned take = 64u - have;
        if (take > len)
            take = len;
        if (have == 0 && len >= 64) {          /* whole block straight from input */
            o_compress(c->state, p);
            p += 64;
            len -= 64;
            continue;
        }
        memcpy(c->pending + have, p, take);
        have += take;
        p += take;
        len -= take;
        if (have == 64) {
            o_compress(c->state, c->pending);
            have = 0;
        }
    }
}

void oracle_md5_final(unsigned char digest[16], struct oracle_md5_ctx *c)
{
    unsigned used = (c->nbits[0] >> 3) & 63u;  /* md5.c:228 */
    uint8_t blk[128];
    unsigned total = (used < 56) ? 64u : 128u; /* md5.c:240: < 8 bytes free -> 2 blocks */
    memset(blk, 0, sizeof blk);
    memcpy(blk, c->pending, used);
    blk[used] = 0x80;                          /* md5.c:232-233 */
    for (unsigned k = 0; k < 4; k++) {         /* bit length LE in the last 8 bytes, md5.c:258-259 */
        blk[total - 8 + k] = (uint8_t)(c->nbits[0] >> (8 * k));
        blk[total - 4 + k] = (uint8_t)(c->nbits[1] >> (8 * k));
    }
    o_compress(c->state, blk);
    if (total == 128)
        o_compress(c->state, blk + 64);
    for (unsigned k = 0; k < 16; k++)          /* md5.c:262-263 */
        digest[k] = (uint8_t)(c->state[k >> 2] >> (8 * (k & 3)));
    memset(c, 0, sizeof *c);                   /* md5.c:264 */
}

/* ---- convenience entry points for the Python test harness (ctypes) ---- */

size_t oracle_md5_ctx_size(void) { return sizeof(struct oracle_md5_ctx); }

void oracle_md5(const void *data, uint64_t len, unsigned char digest[16])
{
    struct oracle_md5_ctx c;
    const uint8_t *p = (const uint8_t *)data;
    oracle_md5_init(&c);
    while (len > 0) {                 /* 'len' is 32-bit in md5.h:47; split big inputs */
        unsigned part = len > 0x40000000u ? 0x40000000u : (unsigned)len;
        oracle_md5_update(&c, p, part);
        p += part;
        len -= part;
    }
    oracle_md5_final(digest, &c);
}

/* digest[i] = MD5(base + offs[i], lens[i]) for i in [0, n). */
void oracle_md5_batch(const void *base, const uint64_t *offs, const uint32_t *lens,
                      uint64_t n, unsigned char *digests)
{
    const uint8_t *b = (const uint8_t *)base;
    for (uint64_t i = 0; i < n; i++)
        oracle_md5(b + offs[i], lens[i], digests + 16 * i);
}

/* Fixed-stride batch: chunk i is base[i*len .. i*len+len). */
void oracle_md5_batch_fixed(const void *base, uint64_t n, uint32_t len,
                            unsigned char *digests)
{
    const uint8_t *b = (const uint8_t *)base;
    for (uint64_t i = 0; i < n; i++)
        oracle_md5(b + i * (uint64_t)len, len, digests + 16 * i);
}

/* ---- deterministic test-data generators (shared with tests/gen.py) ---- */

/* xorshift64 (13/7/17) stream, each state stored little-endian, as SURVEY.md
 * §8(c)/(d) specifies for the C1 buffers.  The first 8 bytes are the state
 * after ONE update of the seed. */
void oracle_xorshift_fill(void *dst, uint64_t nbytes, uint64_t seed)
{
    uint8_t *d = (uint8_t *)dst;
    uint64_t s = seed;
    uint64_t off = 0;
    while (off < nbytes) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        for (unsigned k = 0; k < 8 && off < nbytes; k++, off++)
            d[off] = (uint8_t)(s >> (8 * k));
    }
}
