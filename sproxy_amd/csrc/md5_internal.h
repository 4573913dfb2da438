/* md5_internal.h -- entries shared between the library's own objects
 * (hidden: not part of the C ABI in include/). */
#ifndef SPROXY_AMD_MD5_INTERNAL_H
#define SPROXY_AMD_MD5_INTERNAL_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* One copy of the device-side gather: `len` bytes from the device-visible
 * address `src` (registered host memory) to d_dst + dst. */
struct md5hip_seg {
    uint64_t src;
    uint64_t dst;
    uint32_t len;
    uint32_t pad;
};

/* Gather kernel (md5_kernels.hip): one workgroup per segment. */
__attribute__((visibility("hidden")))
int md5hip_gather_launch(const struct md5hip_seg *d_segs, uint64_t nseg, unsigned char *d_dst,
                         void *stream);

/* Batched verify with a digest kind of its own (md5_submit.c): the
 * batcher's setting is not touched, so concurrent submitters keep theirs. */
struct md5hip_batcher;
struct md5hip_iov;
__attribute__((visibility("hidden")))
int md5hip_verify_iov_as(struct md5hip_batcher *b, int kind, uint32_t fastcrc,
                         const struct md5hip_iov *segs, const uint64_t *seg_first, uint64_t n,
                         const void *expected, unsigned char *ok);

#ifdef __cplusplus
}
#endif

#endif
