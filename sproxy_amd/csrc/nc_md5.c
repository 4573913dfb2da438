/*
 * nc_md5.c -- netcache-compatible nc_MD5 (include/nc_md5.h), host path.
 *
 * Behaviour of /root/reference/netcache/netcache/md5.c on an LP64 host, where
 * UINT4 is 64 bits wide (netcache/include/md5.h:40): every add, the four
 * round functions and ROTATE_LEFT(x, n) = (x << n) | (x >> (32 - n))
 * (md5.c:116-122) run in 64-bit arithmetic, the message words are the 32-bit
 * little-endian input words zero-extended (md5.c:192-195), and the digest is
 * the low 32 bits of each state word (md5.c:232-238).  Written as a
 * table-driven loop that the compiler unrolls; parity with the reference
 * build is pinned by tests/test_nc_md5.py.
 */
#include <stdint.h>
#include <string.h>

#include "../../include/nc_md5.h"

_Static_assert(sizeof(nc_MD5_CTX) == 128, "LP64 layout of netcache md5.h:43-49");

static const uint32_t nc_k[64] = {
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
static const unsigned nc_s[4][4] = {{7, 12, 17, 22}, {5, 9, 14, 20}, {4, 11, 16, 23}, {6, 10, 15, 21}};

/* Fully unrolled (the pragma): every index below is then a constant, v[]
 * lives in registers and the switch folds away: 1.4-1.6x faster than the
 * rolled loop and 2-17 % faster than the reference md5.c for 32 B-1 KiB keys
 * (scripts/nc_md5_speed.sh, profiles/r01_nc_md5_speed_container.txt). */
__attribute__((optimize("O3"))) static void nc_transform(unsigned long st[4],
                                                          const unsigned long m[16])
{
    unsigned long v[4] = {st[0], st[1], st[2], st[3]};
#pragma GCC unroll 64
    for (unsigned j = 0; j < 64; j++) {
        const unsigned r = j >> 4, i = j & 15u;
        const unsigned w = (4u - (j & 3u)) & 3u;            /* a, d, c, b, ... */
        const unsigned long x = v[(w + 1) & 3], y = v[(w + 2) & 3], z = v[(w + 3) & 3];
        unsigned long f;
        unsigned g;
        switch (r) {
        case 0:  f = (x & y) | (~x & z);  g = i; break;                  /* F */
        case 1:  f = (x & z) | (y & ~z);  g = (5 * i + 1) & 15u; break;  /* G */
        case 2:  f = x ^ y ^ z;           g = (3 * i + 5) & 15u; break;  /* H */
        default: f = y ^ (x | ~z);        g = (7 * i) & 15u; break;      /* I */
        }
        unsigned long a = v[w] + f + m[g] + (unsigned long)nc_k[j];
        const unsigned s = nc_s[r][j & 3u];
        a = (a << s) | (a >> (32 - s));                 /* 64-bit, high bits kept */
        v[w] = a + x;
    }
    for (int k = 0; k < 4; k++) st[k] += v[k];
}

static void nc_words(const unsigned char *p, unsigned long *m, int n)
{
    for (int k = 0; k < n; k++)
        m[k] = (unsigned long)p[4 * k] | (unsigned long)p[4 * k + 1] << 8 |
               (unsigned long)p[4 * k + 2] << 16 | (unsigned long)p[4 * k + 3] << 24;
}

void nc_MD5Init(nc_MD5_CTX *c)
{
    c->i[0] = c->i[1] = 0;
    c->buf[0] = 0x67452301ul;
    c->buf[1] = 0xefcdab89ul;
    c->buf[2] = 0x98badcfeul;
    c->buf[3] = 0x10325476ul;
    memset(c->digest, 0, sizeof c->digest);
}

void nc_MD5Update(nc_MD5_CTX *c, unsigned char *in, unsigned int n)
{
    unsigned fill = (unsigned)((c->i[0] >> 3) & 0x3F);
    const unsigned long add = (unsigned long)n << 3;
    if (c->i[0] + add < c->i[0]) c->i[1]++;             /* md5.c:180-183, 64-bit */
    c->i[0] += add;
    c->i[1] += (unsigned long)n >> 29;
    while (n > 0) {
        unsigned take = 64 - fill < n ? 64 - fill : n;
        memcpy(c->in + fill, in, take);
        in += take;
        n -= take;
        fill += take;
        if (fill == 64) {
            unsigned long m[16];
            nc_words(c->in, m, 16);
            nc_transform(c->buf, m);
            fill = 0;
        }
    }
}

void nc_MD5Final(nc_MD5_CTX *c)
{
    static unsigned char pad[64] = {0x80};
    unsigned long m[16];
    m[14] = c->i[0];                                     /* full 64-bit words (md5.c:211-212) */
    m[15] = c->i[1];
    const unsigned fill = (unsigned)((c->i[0] >> 3) & 0x3F);
    nc_MD5Update(c, pad, fill < 56 ? 56 - fill : 120 - fill);
    nc_words(c->in, m, 14);
    nc_transform(c->buf, m);
    for (int k = 0; k < 4; k++)
        for (int b = 0; b < 4; b++) c->digest[4 * k + b] = (unsigned char)(c->buf[k] >> (8 * b));
}
