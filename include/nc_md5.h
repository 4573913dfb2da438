/*
 * include/nc_md5.h -- drop-in for netcache's nc_MD5 (netcache/include/md5.h,
 * implementation netcache/netcache/md5.c), the RSA-reference MD5 whose UINT4
 * is `unsigned long int` (md5.h:40): 64-bit on LP64 hosts, so state, counters
 * and rotates carry high bits and the digests are NOT RFC 1321 MD5
 * (nc_MD5("") = e4c23762ed2823a27e62a64b95c024e7).  Existing cache-key
 * variant suffixes (diskcache.c:3443-3452) and the consistent-hash ring
 * (plugins/common/lb.c:1041-1054, 1396-1410) depend on those exact values,
 * so this keeps them.  Host path only: the inputs are short keys.
 *
 * Layout as md5.h:43-49 on LP64: 128 bytes (i[2] at 0, buf[4] at 16,
 * in[64] at 48, digest[16] at 112).
 */
#ifndef SPROXY_AMD_NC_MD5_H
#define SPROXY_AMD_NC_MD5_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct {
    unsigned long i[2];       /* bit count (carried as in md5.c:180-183) */
    unsigned long buf[4];     /* state */
    unsigned char in[64];     /* input buffer */
    unsigned char digest[16]; /* result after nc_MD5Final */
} nc_MD5_CTX;

/* replaces netcache/netcache/md5.c:147-165 */
void nc_MD5Init(nc_MD5_CTX *ctx);
/* replaces md5.c:167-200 */
void nc_MD5Update(nc_MD5_CTX *ctx, unsigned char *inBuf, unsigned int inLen);
/* replaces md5.c:202-239; the digest lands in ctx->digest */
void nc_MD5Final(nc_MD5_CTX *ctx);

#ifdef __cplusplus
}
#endif

#endif /* SPROXY_AMD_NC_MD5_H */
