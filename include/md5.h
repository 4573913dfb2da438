/*
 * include/md5.h -- drop-in replacement header for sproxy's md5.h.
 *
 * Same ABI as /root/reference/md5.h:31-51 so that soluri2.c:711-713 and
 * streaming.c:7840-7842 recompile unchanged against libmd5hip.so:
 *   - MD5_DIGEST_SIZE 16                         (md5.h:31)
 *   - struct MD5Context { buf[4]; bits[2]; in[64] }, 88 bytes, 4-byte aligned
 *     (md5.h:33-38; buf at offset 0, bits at 16, in at 24)
 *   - MD5Init / MD5Update(ctx, buf, unsigned len) / MD5Final(digest, ctx)
 *     (md5.h:41-51; note the digest is MD5Final's FIRST argument)
 * Semantics as md5.c:153-265: void returns, no failure mode, reentrant per
 * context, MD5Final zeroes the context.  These per-message entries run on
 * the host CPU in libmd5hip.so (sproxy_amd/csrc/md5_stream.c): the callers
 * hash tens-to-hundreds of bytes per request, where a device round trip
 * would be a latency regression.  Chunk batches go through
 * the device API in md5hip.h.
 */
#ifndef SPROXY_AMD_MD5_H
#define SPROXY_AMD_MD5_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MD5_DIGEST_SIZE 16

struct MD5Context {
    uint32_t buf[4];      /* running A, B, C, D */
    uint32_t bits[2];     /* message length in bits, low word first */
    unsigned char in[64]; /* pending partial block */
};

/* replaces md5.h:41-42 / md5.c:153-163 */
void MD5Init(struct MD5Context *ctx);
/* replaces md5.h:44-47 / md5.c:169-215 */
void MD5Update(struct MD5Context *ctx, const void *buf, unsigned len);
/* replaces md5.h:49-51 / md5.c:221-265 */
void MD5Final(unsigned char digest[MD5_DIGEST_SIZE], struct MD5Context *ctx);

#ifdef __cplusplus
}
#endif

#endif /* SPROXY_AMD_MD5_H */
