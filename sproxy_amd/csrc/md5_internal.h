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

/* CRC kernel variant (enum crc32hip_variant) for a full-CRC descriptor batch
 * of n chunks whose mean length is known (md5_kernels.hip). */
__attribute__((visibility("hidden")))
int md5hip_crc_desc_choice(uint64_t n, uint64_t mean_len);

/* MD5 descriptor variant for a planned batch of `bytes` payload of which
 * `unlined_bytes` lie in chunks starting 16-B but not 128-B aligned: XDMA
 * becomes LINES past half (md5_kernels.hip). */
__attribute__((visibility("hidden")))
int md5hip_lines_choice(int variant, uint64_t unlined_bytes, uint64_t bytes);

/* Batched verify with a digest kind of its own (md5_submit.c): the
 * batcher's setting is not touched, so concurrent submitters keep theirs. */
struct md5hip_batcher;
struct md5hip_iov;
__attribute__((visibility("hidden")))
int md5hip_verify_iov_as(struct md5hip_batcher *b, int kind, uint32_t fastcrc,
                         const struct md5hip_iov *segs, const uint64_t *seg_first, uint64_t n,
                         const void *expected, unsigned char *ok);

/* For the multi-GPU pool's router (md5_pool.c), all in md5_submit.c:
 *   md5hip_batcher_load    weight (len + 64 per chunk) reserved in the
 *                          batcher's open and in-flight slots, read lock-free
 *   md5hip_batcher_slice   staging bytes per slot
 *   md5hip_submit_as       host chunks (ptrs/lens, or segs/seg_first when
 *                          ptrs is NULL) with an explicit digest kind;
 *                          ticket NULL = synchronous; urgent = launched at
 *                          once like a synchronous call (the caller waits
 *                          on the ticket right away)
 *   md5hip_host_fixed_as   md5hip_batch_host_fixed with an explicit kind,
 *                          optionally asynchronous
 *   md5hip_batcher_ticket_state  1 done (*err = its error), 0 pending,
 *                          -EINVAL unknown; never launches anything */
__attribute__((visibility("hidden")))
uint64_t md5hip_batcher_load(const struct md5hip_batcher *b);
__attribute__((visibility("hidden")))
uint64_t md5hip_batcher_slice(const struct md5hip_batcher *b);
__attribute__((visibility("hidden")))
int md5hip_submit_as(struct md5hip_batcher *b, int kind, uint32_t fastcrc, const void *const *ptrs,
                     const uint32_t *lens, const struct md5hip_iov *segs, const uint64_t *seg_first,
                     uint64_t n, unsigned char *digests, uint64_t *ticket, int urgent);
__attribute__((visibility("hidden")))
int md5hip_host_fixed_as(struct md5hip_batcher *b, int kind, uint32_t fastcrc, const void *h_base,
                         uint64_t n, uint32_t len, uint64_t stride, unsigned char *digests,
                         uint64_t *ticket);
__attribute__((visibility("hidden")))
int md5hip_batcher_ticket_state(struct md5hip_batcher *b, uint64_t ticket, int *err);

#ifdef __cplusplus
}
#endif

#endif
