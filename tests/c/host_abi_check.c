/*
 * host_abi_check.c -- exercises the host-side C entries of libmd5hip
 * (include/md5.h, nc_md5.h, nc_digest.h, md5hip_pool_plan) from plain C, built
 * by tests/test_host_sanitize.py with -fsanitize=address,undefined.  Prints
 * one result per line; the test compares them with the oracle and goldens.
 *
 *   md5 <len> <hex>      MD5Update in random-sized pieces of mul_pattern[0:len]
 *   ncmd5 <len> <hex>    nc_MD5 of the same bytes
 *   crc <len> <hex>      nc_crc32 of the same bytes
 *   hdr <hex> <ok>       nc_header_crc / nc_header_verify of a sealed header
 *   plan <G> <first...>  md5hip_pool_plan over a fixed length list
 *   arr <rc...>          nc_digest_update / verify bound cases
 *   ctx <seq> <off> <n> <hex88>  the whole context after each MD5Update of
 *                        buf[off:off+n] (stale in[] preset to 0x5a), for the
 *                        test to replay through the reference md5.c
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "md5.h"
#include "md5hip.h"
#include "nc_digest.h"
#include "nc_md5.h"

static unsigned char *mul_pattern(size_t n)
{
    unsigned char *b = malloc(n ? n : 1);
    for (size_t i = 0; i < n; i++) b[i] = (unsigned char)((uint32_t)(i * 2654435761u) >> 24);
    return b;
}

static void hex(const unsigned char *d, int n)
{
    for (int i = 0; i < n; i++) printf("%02x", d[i]);
}

int main(void)
{
    static const unsigned lens[] = {0, 1, 55, 56, 57, 63, 64, 65, 119, 120, 127, 128, 4096, 16384,
                                    16385, 65536};
    const size_t maxlen = 65536;
    unsigned char *buf = mul_pattern(maxlen);
    uint64_t rng = 0x1234567;
    for (size_t k = 0; k < sizeof lens / sizeof lens[0]; k++) {
        const unsigned L = lens[k];
        struct MD5Context ctx;
        unsigned char dig[16];
        MD5Init(&ctx);
        for (unsigned at = 0; at < L;) {
            rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
            unsigned take = (unsigned)(rng % 200);
            if (take > L - at) take = L - at;
            MD5Update(&ctx, buf + at, take);
            at += take;
        }
        MD5Final(dig, &ctx);
        printf("md5 %u ", L); hex(dig, 16); printf("\n");
        nc_MD5_CTX nctx;
        nc_MD5Init(&nctx);
        nc_MD5Update(&nctx, buf, L);
        nc_MD5Final(&nctx);
        printf("ncmd5 %u ", L); hex(nctx.digest, 16); printf("\n");
        printf("crc %u %08x\n", L, nc_crc32(buf, L));
    }
    /* a sealed header, then the verify result after the skipped fields change */
    const int32_t hs = 1000;
    unsigned char *h = calloc(1, hs);
    const uint32_t magic = NC_MAGIC_V30;
    memcpy(h, &magic, 4);
    memcpy(h + NC_HDR_OFF_HEADER_SIZE, &hs, 4);
    memcpy(h + NC_HDR_MIN_SIZE, buf, hs - NC_HDR_MIN_SIZE);
    if (nc_header_seal(h) != 0) return 2;
    const int32_t dhs = 321;
    const uint32_t flag = 0x10000000u;
    memcpy(h + NC_HDR_OFF_DISK_HEADER_SIZE, &dhs, 4);
    memcpy(h + NC_HDR_OFF_FLAG, &flag, 4);
    printf("hdr %08x %d\n", nc_header_crc(h), nc_header_verify(h));
    h[500] ^= 1;
    printf("hdrbad %d\n", nc_header_verify(h));
    free(h);
    /* call-by-call context bytes (md5.c:204-214 leaves the last whole block in in[]) */
    for (int seq = 0; seq < 40; seq++) {
        struct MD5Context ctx;
        MD5Init(&ctx);
        memset(ctx.in, 0x5a, sizeof ctx.in);
        for (int call = 0; call < 6; call++) {
            rng ^= rng << 13; rng ^= rng >> 7; rng ^= rng << 17;
            const unsigned n = (unsigned)(rng % (call & 1 ? 300u : 5000u));
            const unsigned off = (unsigned)((rng >> 20) % (maxlen - n));
            MD5Update(&ctx, buf + off, n);
            printf("ctx %d %u %u ", seq, off, n); hex((const unsigned char *)&ctx, sizeof ctx); printf("\n");
        }
    }
    /* pool split */
    uint32_t pl[100];
    for (int i = 0; i < 100; i++) pl[i] = (uint32_t)((i * 7919u) % 5000u);
    uint64_t first[9];
    if (md5hip_pool_plan(pl, 100, 8, first) != 0) return 3;
    printf("plan 8");
    for (int g = 0; g <= 8; g++) printf(" %llu", (unsigned long long)first[g]);
    printf("\n");
    /* digest array bounds (dsz 16 on an array of 3 entries) */
    unsigned char arr[48] = {0}, d16[16];
    memset(d16, 0xab, 16);
    const int u0 = nc_digest_update(arr, 48, 16, 3, 2, d16);      /* in order: C leaves */
    const int u1 = nc_digest_update(arr, 48, 16, 3, 3, d16);      /* argument evaluation */
    const int u2 = nc_digest_update(arr, 48, 16, 9, 3, d16);      /* order unspecified */
    const int v0 = nc_digest_verify(arr, 48, 16, 2, d16);
    const int v1 = nc_digest_verify(arr, 48, 16, 1, d16);
    printf("arr %d %d %d %d %d\n", u0, u1, u2, v0, v1);
    free(buf);
    return 0;
}
