/*
 * include/md5hip.h -- batched MD5 on MI355X (gfx950): the C-ABI boundary.
 *
 * sproxy has no batched digest entry; its chunk-granular checksum call site is
 *   nc_crc_t blk_make_crc(fc_inode_t *inode, fc_blk_t *blk, ssize_t len, int fastcrc)
 *   (netcache/common/blk_io.c:354-430, called from blk_io.c:665-704 on cache
 *    read, blk_io.c:851-863 on origin read, bc_mgr.c:1464-1492 on write verify)
 * which checksums ONE cache block per call.  The entries below replace that
 * per-block call with a batch of independent chunks; every digest equals
 * MD5Init/MD5Update(chunk)/MD5Final from md5.c:153-265 bit for bit.
 *
 * Conventions (all entries):
 *   - plain C types only; `stream` is a hipStream_t passed as void* (NULL =
 *     the null stream of the current device); device pointers are memory of
 *     the current HIP device (hipMalloc, or a torch CUDA tensor's data_ptr);
 *   - asynchronous w.r.t. the host unless stated; errors are returned as
 *     0 / negative errno, checked BEFORE anything is enqueued:
 *       -EINVAL  bad argument (NULL pointer with n > 0, len > stride, ...)
 *       -ENODEV  no usable gfx950 device / HIP runtime failure
 *       -EIO     the kernel launch itself failed
 *   - digest i is 16 bytes, MD5 byte order (md5.c:262-263), at digests+16*i.
 */
#ifndef SPROXY_AMD_MD5HIP_H
#define SPROXY_AMD_MD5HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI 5 (round 6): md5hip_order_stable_scratch / md5hip_order_device_stable
 * (appended; the batcher's large slots use them); md5hip_batch_host_fixed
 * reads a source in place only if it is pinned over its whole range.
 * ABI 4 (round 5): device failure -- md5hip_batcher_health /
 * md5hip_batcher_inject_fault, md5hip_pool_get_health / _device_health /
 * _inject_fault -- and md5_batch_submit_device_fixed (appended); md5hip_batcher_set_chain rejects modes outside
 * 0..2 with -EINVAL.
 * ABI 3 (round 4): md5_batch_submit_device_after (an ordering flag apart from
 * the producer stream, so the null stream can be ordered on), the LINES
 * descriptor kernel and md5hip_plan_desc_at (appended); round 3 had
 * already grown MD5HIP_DESC_NUM_VARIANTS 6 -> 7 (FED) and CRC32HIP_NUM_VARIANTS
 * 7 -> 8 (SPLIT) -- appended values, compatible -- and made the pool route a
 * submission whole (same results; set_digest no longer drains). */
#define MD5HIP_ABI_VERSION 5

/* Fixed-length kernels for md5hip_digest_fixed_variant.  ABI 2: the round-1
 * A/B variants (values 2-9) moved to the diagnostic library (removed in round 4;
 * git history at 993ee7d, sproxy_amd/csrc/md5_diag.hip);
 * the library ships the default and one fallback, and no environment
 * variable re-routes a launch. */
enum md5hip_variant {
    MD5HIP_AUTO = 0,        /* the default: XDMA1NT */
    MD5HIP_DIRECT2 = 1,     /* lane-direct dwordx4 loads, 2-block register ring (used for
                               strides >= 2^31/64, where XDMA1NT's 32-bit offsets end) */
    MD5HIP_XDMA1NT = 10,    /* 8 chunks x 128 B per wave-instruction by LDS-DMA into a per-wave
                               transpose image, non-temporal; DESIGN.md §4 */
    MD5HIP_NUM_VARIANTS = 11
};

int md5hip_abi_version(void);
const char *md5hip_variant_name(int variant);
/* The concrete variant MD5HIP_AUTO resolves to. */
int md5hip_resolve_variant(int variant);

/*
 * Fixed-length device batch (the hot path):
 *   digests[i] = MD5(d_base + i*stride, len),  i in [0, n).
 * Requires len <= stride.  Fast path: d_base and stride 16-byte aligned;
 * otherwise the descriptor kernel is used.  Replaces n calls of
 * blk_make_crc (blk_io.c:354) over equal-sized blocks.
 */
int md5hip_digest_fixed(const void *d_base, uint64_t n, uint32_t len, uint64_t stride,
                        unsigned char *d_digests, void *stream);
int md5hip_digest_fixed_variant(const void *d_base, uint64_t n, uint32_t len, uint64_t stride,
                                unsigned char *d_digests, void *stream, int variant);

/*
 * Descriptor device batch (mixed lengths, any alignment; config C3):
 *   digests[i] = MD5(d_base + d_offsets[i], d_lens[i]).
 * d_order (optional, may be NULL) is a permutation of [0, n) giving the order
 * in which chunks are packed onto lanes; pass md5hip_plan_order()'s output
 * (longest first) so that a wave's 64 lanes carry similar block counts.
 */
int md5hip_digest_desc(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
                       const uint32_t *d_order, uint64_t n, unsigned char *d_digests,
                       void *stream);
/* Descriptor-batch kernels for md5hip_digest_desc_variant. */
enum md5hip_desc_variant {
    MD5HIP_DESC_AUTO = 0,   /* the default: XDMA */
    MD5HIP_DESC_LANE = 1,   /* each lane streams its own chunk (8-block register ring):
                               the planner's choice for small batches */
    /* 2: the register-staged XPOSE loader, retired (round-1 A/B) */
    MD5HIP_DESC_HYBRID = 3, /* XDMA, but the first waves (one per CU) go lane-direct when
                               they hold a chunk >= 256 KiB (md5hip_plan_desc's choice for
                               batches whose longest chunks bound the launch) */
    MD5HIP_DESC_XDMA = 4,   /* whole-line loads of 8 chunks x 128 B by LDS-DMA into a
                               transpose image; waves holding an unaligned chunk go LANE */
    MD5HIP_DESC_BALANCED = 5, /* XDMA's loader in a persistent grid of one wave per SIMD
                               taking 64-chunk groups longest-first (LPT list scheduling):
                               the planner's choice for mixed batches holding several
                               waves of work per SIMD (coalesced submissions) */
    MD5HIP_DESC_FED = 6,    /* one 2-wave workgroup per 64-chunk group: a feeder wave forms
                               each step's message word + constant, so the chain wave runs
                               4 VALU per step instead of 5; groups holding an unaligned
                               chunk start (or no chunk of >= 128 B) go LANE.  The
                               planner's choice for small batches (round 3) */
    MD5HIP_DESC_LINES = 7,  /* XDMA whose waves holding a chunk that does not start on a
                               128-B line load whole lines, each once, instead of
                               chunk-relative 128-B stages straddling two lines (ABI 3;
                               md5hip_plan_desc_at's choice for such batches) */
    MD5HIP_DESC_NUM_VARIANTS = 8
};
int md5hip_digest_desc_variant(const void *d_base, const uint64_t *d_offsets,
                               const uint32_t *d_lens, const uint32_t *d_order, uint64_t n,
                               unsigned char *d_digests, void *stream, int variant);

/*
 * MD5Init / MD5Update / MD5Final on many caller-owned contexts at once
 * (md5.c:153-265, batched; the "init/update/final behind the C-ABI shim" of
 * north_star for concurrent objects).  d_ctxs: n struct MD5Context (md5.h,
 * 88 bytes each, 4-byte aligned) in device memory.  Every context ends
 * byte-for-byte as the same sequence of host calls leaves it:
 *   md5hip_init_ctx    ctx i as MD5Init (md5.c:153-163; in[] untouched);
 *   md5hip_update_ctx  ctx i as MD5Update(ctx i, d_ptrs[i], d_lens[i]): the
 *                      bit count with its carry (md5.c:177-182), the pending
 *                      partial block completed, whole blocks compressed, the
 *                      tail left in ctx->in (md5.c:184-214); d_ptrs is a DEVICE
 *                      array of device addresses, any alignment, d_lens a
 *                      device array (one update per context per call; 0 = none);
 *   md5hip_final_ctx   digest i (16 B, 16-B aligned array) as MD5Final, ctx i
 *                      zeroed (md5.c:221-265).
 * Calls on one stream apply in order, so k updates are k launches.  An update
 * over at most 64 contexts per CU lasts one context's serial chain and runs its
 * whole blocks as fed pairs: keep each context's data 16-B
 * aligned past its pending bytes to stay on that path.
 */
struct MD5Context;
int md5hip_init_ctx(struct MD5Context *d_ctxs, uint64_t n, void *stream);
int md5hip_update_ctx(struct MD5Context *d_ctxs, const void *const *d_ptrs, const uint32_t *d_lens,
                      uint64_t n, void *stream);
int md5hip_final_ctx(struct MD5Context *d_ctxs, uint64_t n, unsigned char *d_digests, void *stream);

/*
 * CRC-32 block checksums -- the checksum netcache itself computes at the
 * block-completion site: nc_crc_t blk_make_crc(inode, blk, len, fastcrc)
 * (netcache/common/blk_io.c:354-430, compiled with NC_ENABLE_CRC), CRC-32
 * from netcache/netcache/crc32.c (zlib polynomial 0xEDB88320, crc32.c:22).
 *   crcs[i] = fastcrc == 0 || len_i <= fastcrc ? crc32(chunk_i)
 *           : crc32(first fastcrc bytes) ^ crc32(last fastcrc bytes)
 * exactly as blk_io.c:408-424 combines them.  Same conventions as the MD5
 * entries; fastcrc must be a multiple of 4 (cfs_apix.c:2222-2236).
 */
int crc32hip_fixed(const void *d_base, uint64_t n, uint32_t len, uint64_t stride,
                   uint32_t fastcrc, uint32_t *d_crcs, void *stream);
/* CRC-32 kernels for crc32hip_fixed_variant (ABI 2: values 1-5, the round-1
 * A/B variants, retired; their measurements stay in profiles/). */
enum crc32hip_variant {
    CRC32HIP_AUTO = 0,      /* the default: XDMA16 */
    CRC32HIP_XDMA16 = 6,    /* slicing-by-4 over 16 v_perm-addressed LDS table copies, 8 KiB
                               images filled by LDS-DMA, 12 waves/CU */
    CRC32HIP_SPLIT = 7,     /* one wave per chunk: 256-B segments per lane, registers combined
                               with crc32_combine's zero-byte operators (CRC-32 is linear);
                               AUTO's choice for full-CRC batches of up to 128 chunks per CU
                               of >= 2 KiB (12 per CU shorter; 16 per CU when the lengths
                               are device-side only); fastcrc windows of >= 2 KiB split as
                               two messages per chunk, shorter ones keep the window kernels */
    CRC32HIP_NUM_VARIANTS = 8
};
int crc32hip_fixed_variant(const void *d_base, uint64_t n, uint32_t len, uint64_t stride,
                           uint32_t fastcrc, uint32_t *d_crcs, void *stream, int variant);
/* The variant CRC32HIP_AUTO resolves to (same for any other value). */
int crc32hip_resolve_variant(int variant);
int crc32hip_desc(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
                  const uint32_t *d_order, uint64_t n, uint32_t fastcrc, uint32_t *d_crcs,
                  void *stream);
/* The same with the kernel named (CRC32HIP_AUTO = crc32hip_desc's choice). */
int crc32hip_desc_variant(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
                          const uint32_t *d_order, uint64_t n, uint32_t fastcrc, uint32_t *d_crcs,
                          void *stream, int variant);

/*
 * Host helper: order[] = indices of lens[] sorted by MD5 block count,
 * descending (stable counting sort, O(n)).  Synchronous, host memory.
 */
int md5hip_plan_order(const uint32_t *lens, uint64_t n, uint32_t *order);

/*
 * Batch arena: `bytes` of device memory on `device` at a 1 GiB-aligned
 * virtual address (reserved + mapped through the HIP virtual memory API), so
 * the GPU page tables can use large fragments for the whole range.  Chunks
 * hashed by lane-direct chains (HYBRID's long waves) touch 64 pages per load;
 * they run faster from an arena than from a 2 MiB-aligned hipMalloc buffer.
 * 0 / -EINVAL / -ENODEV / -ENOMEM / -EIO; free with md5hip_arena_free, which
 * first synchronizes the arena's device (a kernel still queued on any stream
 * may read it), so it may be called right after an asynchronous launch.
 */
int md5hip_arena_alloc(int device, uint64_t bytes, void **d_ptr);
int md5hip_arena_free(void *d_ptr);

/*
 * Host planner for a descriptor batch: fills order[] as md5hip_plan_order and
 * returns the enum md5hip_desc_variant to launch it with (>= 0), or -errno.
 * FED for a small batch of at most one 64-chunk group per CU of the current
 * device whose longest chunk has >= 2 whole blocks, LANE for one of at most
 * two groups per CU (the launch is one chunk's serial chain: FED takes an
 * instruction per step off it, lane-direct loads keep it free of load
 * waits).  Otherwise, with the longest chunk >= 256 KiB and the median 64-chunk group at most an
 * eighth of the longest (a mixed batch): BALANCED when the batch holds at
 * least 0.4 x (SIMDs x the longest chain) of work, so the placement of waves
 * on SIMDs decides the time; else HYBRID when the longest chunks stand out
 * (the chunk two waves per CU deep in the order is at most a quarter as
 * long), so their serial chains bound the launch; else XDMA.
 */
int md5hip_plan_desc(const uint32_t *lens, uint64_t n, uint32_t *order);
/* ABI 3: the same for chunks whose device addresses (or offsets from a
 * 128-B-aligned base) the caller holds on the host, addrs[i]: an XDMA batch
 * becomes MD5HIP_DESC_LINES when more than half its bytes lie in chunks that
 * start 16-B but not 128-B aligned (device-resident blocks packed at 16 B),
 * whose chunk-relative 128-B stages would straddle lines. */
int md5hip_plan_desc_at(const uint32_t *lens, const uint64_t *addrs, uint64_t n, uint32_t *order);

/* Planning without sorting on the host, for producers that count lengths as
 * chunks arrive (the batcher does): hist[k] = number of chunks whose key
 * k = (len >> 6) + 1, for k in [1, kmax] (kmax <= MD5HIP_HIST_KMAX, chunks
 * up to 8 MiB).  Returns md5hip_plan_desc's variant for such a batch and, if
 * bucket_start is not NULL, fills bucket_start[kmax - k] with the first
 * position of key k in the longest-first order (kmax + 1 entries).
 * md5hip_order_device then builds that order on the device: with
 * d_bucket_next holding bucket_start, d_order[d_bucket_next[kmax - k]++] = i
 * for every chunk i of key k (positions within one key in wave-arrival
 * order -- correct for every kernel, but BALANCED over large mixed batches
 * runs 5-6 % faster in the stable order below).  Asynchronous on `stream`; 0 or -errno.  The
 * histogram must cover every chunk: a chunk whose key exceeds kmax is left
 * out of the order (its position keeps what it held), never written past
 * d_bucket_next. */
#define MD5HIP_HIST_KMAX (1u << 17)
int md5hip_plan_hist(const uint32_t *hist, uint32_t kmax, uint64_t n, uint32_t *bucket_start);
int md5hip_order_device(const uint32_t *d_lens, uint64_t n, uint32_t kmax, uint32_t *d_bucket_next,
                        uint32_t *d_order, void *stream);
/* ABI 5: the same order, STABLE -- equal keys in chunk-index order, exactly
 * md5hip_plan_desc's host order -- built by a device radix sort (rocPRIM)
 * of (kmax - key, index) pairs.  The positions within a key matter after
 * all: BALANCED over 6 coalesced C3 batches ran 5-6 % longer with
 * md5hip_order_device's wave-arrival order; the batcher
 * uses this one.  Device scratch of md5hip_order_stable_scratch(n, kmax)
 * bytes (0 = unsupported n or kmax; kmax 0 sizes for any kmax up to
 * MD5HIP_HIST_KMAX); a chunk whose key exceeds kmax goes after every
 * bucket.  Asynchronous on `stream`; 0, -EINVAL, -ENOSPC (scratch too
 * small), -ENODEV, -EIO. */
uint64_t md5hip_order_stable_scratch(uint64_t n, uint32_t kmax);
int md5hip_order_device_stable(const uint32_t *d_lens, uint64_t n, uint32_t kmax, void *d_scratch,
                               uint64_t scratch_bytes, uint32_t *d_order, void *stream);

/*
 * Synthetic-data generator for benches/tests: fills nbytes (multiple of 16)
 * of device memory with word i = mix32(seed, i) (md5hip_kernels.hip).
 */
int md5hip_fill_synthetic(void *d_dst, uint64_t nbytes, uint64_t seed, void *stream);

/*
 * The batcher: a thread-safe, coalescing submission queue (md5_submit.c) for
 * the blk_make_crc call site (blk_io.c:354; configs C3 and C5).  It owns
 * `nslots` pipeline slots (HIP stream + pinned staging of `slice_bytes` +
 * device buffers + descriptors).  Submissions from any number of threads
 * append their chunks to the one OPEN slot -- host chunks are gathered into
 * its pinned staging, device-resident chunks add only a descriptor -- and
 * the slot is launched as ONE planned descriptor batch when it is full, when
 * fewer than `inflight target` slots are running (an idle device takes work
 * at once), when it is chained behind a launch about to end
 * (md5hip_batcher_set_chain), or when a caller waits on, polls or flushes a
 * ticket in it while nothing runs.  A synchronous submission's slot goes at
 * once while fewer than nslots - 1 launches run; past that it coalesces with
 * the other callers' work in the last slot.
 * While the device is busy, everything submitted meanwhile is therefore
 * coalesced into the next launch.  A progress thread per batcher retires
 * finished slots, delivers digests and launches the open slot.
 * slice_bytes = 0 / nslots = 0 select the defaults, 128 MiB x 4: MD5 is one
 * serial chain per chunk, so the bytes in flight must cover the PCIe rate
 * times one chunk's hashing time.
 * Every entry saves and restores the calling thread's HIP device.
 */
typedef struct md5hip_batcher md5hip_batcher;

/* What a batcher computes per chunk (default MD5, 16 bytes).  CRC32 gives
 * netcache's own 4-byte block checksum, with the fastcrc head^tail window
 * (0 = whole block), i.e. exactly what blk_make_crc returns. */
enum md5hip_digest_kind { MD5HIP_DIGEST_MD5 = 0, MD5HIP_DIGEST_CRC32 = 1 };

int md5hip_batcher_create(int device, uint64_t slice_bytes, uint32_t nslots,
                          md5hip_batcher **out);
/* A batcher sized for device-resident chunks (md5_batch_submit_device*):
 * `max_chunks` descriptors per launch (0 = 1,048,576), 16 MiB of staging per
 * slot for the odd host-memory submission. */
int md5hip_queue_create(int device, uint64_t max_chunks, uint32_t nslots, md5hip_batcher **out);
/* Launches what is still open, waits for everything in flight, frees. */
void md5hip_batcher_destroy(md5hip_batcher *b);
/* Waits until nothing is queued, then switches (concurrent submitters see
 * the new kind on their next call; md5hip_batch_verify_iov returns -EAGAIN
 * if the kind changed between its read and its submit). */
int md5hip_batcher_set_digest(md5hip_batcher *b, int kind, uint32_t fastcrc);
int md5hip_batcher_get_digest(const md5hip_batcher *b, int *kind, uint32_t *fastcrc);
/* The open slot is launched at once while fewer than `target` slots are in
 * flight (1..nslots; default 2, or 1 with fewer than 3 slots).  1 coalesces
 * hardest; nslots never waits to coalesce. */
int md5hip_batcher_set_inflight(md5hip_batcher *b, uint32_t target);
/* Linger: with nothing in flight, an asynchronous submission's slot is held
 * up to min(max_us, 1/8 of the recent launches' wall time) for more work to
 * join it, so a burst of vectors goes out as one launch.  A wait, poll or
 * flush on one of its tickets, a full slot or a synchronous submission still
 * launches at once.  Default max_us 5000; 0 = launch at once. */
int md5hip_batcher_set_linger(md5hip_batcher *b, uint32_t max_us);
/* ABI 3: chained launches.  With the pipeline at its target and the running
 * launch due to end within min(2 ms, a quarter of a launch), the open slot --
 * planned, no chunk arrived since the last poll -- is launched at once with
 * its hash kernel waiting on the running launch's event, so it starts when
 * that one ends instead of after the host has seen it end (a C3 stream step
 * lost ~1.3 ms to that).  mode 1: that; mode 2 (the
 * default): the same, except that when both launches are BALANCED the hash
 * kernel does not wait -- its workgroups take CUs as the running launch's
 * finish (one BALANCED workgroup fills a CU's LDS, so the two never share a
 * CU); 0: off.  Other values: -EINVAL. */
int md5hip_batcher_set_chain(md5hip_batcher *b, int mode);

/* ABI 4: device failure.  blk_make_crc cannot fail (blk_io.c:354-430); a
 * batcher can.  When HIP reports an error back -- a launch's completion
 * event does (a lost or reset device), or an enqueue fails and the slot's
 * stream then reports one -- the batcher is FAILED for good:
 *   - the tickets of that launch complete with -EIO;
 *   - tickets still coalescing in the open slot complete with -ENODEV;
 *   - every later submission returns -ENODEV at once, touching nothing;
 *   - no digest of a failed launch is copied into a HOST digest array; a
 *     DEVICE digest array (digests_on_device) the launch wrote in place, or
 *     the scatter kernel had filled, is undefined after -EIO / -ENODEV.
 * A kernel memory fault on ROCm usually ends the process through the HSA
 * queue's error handler before any event reports it, so the policy covers
 * what the runtime returns, and was checked by injection
 * (md5hip_batcher_inject_fault, the fake runtime of tests/c/), not against
 * a real fault.
 * Launches already in flight complete as their own events say.  The library
 * never falls back to the host: what the call site does instead (and that a
 * device error is never a checksum mismatch) is INTEGRATION.md §2j.
 * md5hip_batcher_health: 0 healthy, -ENODEV failed.
 * md5hip_batcher_inject_fault: test control for that policy -- the
 * after-th launch from now (1 = the next) is reported as a device fault once
 * it has really finished (its event is still waited for); 0 cancels;
 * returns -ENODEV if the batcher has failed already. */
int md5hip_batcher_health(const md5hip_batcher *b);
int md5hip_batcher_inject_fault(md5hip_batcher *b, uint64_t after);

struct md5hip_batcher_stats {
    uint64_t submissions;             /* tickets issued */
    uint64_t launches;                /* slots launched */
    uint64_t coalesced_launches;      /* launches holding chunks of > 1 ticket */
    uint64_t chunks;                  /* chunks launched */
    uint64_t bytes_staged;            /* host bytes moved through staging (host_fixed: a pageable
                                         source's; a wholly pinned one is DMA'd in place, 0) */
    uint64_t max_chunks_per_launch;
    uint64_t max_tickets_per_launch;
    uint64_t inflight_target, nslots, max_chunks_per_slot;
};
int md5hip_batcher_get_stats(md5hip_batcher *b, struct md5hip_batcher_stats *out);

/* digests[i] = MD5(ptrs[i], lens[i]); any host memory.  -E2BIG if one chunk
 * exceeds slice_bytes.  Synchronous. */
int md5_batch_submit(md5hip_batcher *b, const void *const *ptrs, const uint32_t *lens,
                     uint64_t n, unsigned char *digests);

/* One segment of a chunk that lives in several buffers -- e.g. a netcache
 * block, which is a list of 16 KiB pages (netcache/include/block.h:143-146,
 * bc_mgr.c:1251) read through bs_read (bc_mgr.c:1117-1157). */
struct md5hip_iov {
    const void *base;
    uint32_t len;
};

/* digests[i] = MD5(concat(segs[seg_first[i]] .. segs[seg_first[i+1]-1])),
 * seg_first has n+1 entries (seg_first[0] = 0).  The segments are gathered
 * into the pinned staging slice; -E2BIG if one chunk exceeds slice_bytes. */
int md5_batch_submit_iov(md5hip_batcher *b, const struct md5hip_iov *segs,
                         const uint64_t *seg_first, uint64_t n, unsigned char *digests);

/* Asynchronous forms: the
 * call returns once the chunks are staged -- the caller's buffers may be
 * reused, except in the zero-copy gather modes (registered memory is read
 * by the device until the work is done) -- and *ticket names the
 * submission (0 for an empty one).  `digests` must stay valid until
 * md5_batch_wait(b, ticket) returns or md5_batch_poll(b, ticket) returns 1.
 * Tickets complete independently and out of order: a ticket is done when
 * the slots holding ITS chunks are, whatever earlier tickets still run.
 * Submissions larger than the free pipeline block inside the call until
 * slots free up. */
int md5_batch_submit_async(md5hip_batcher *b, const void *const *ptrs, const uint32_t *lens,
                           uint64_t n, unsigned char *digests, uint64_t *ticket);
int md5_batch_submit_iov_async(md5hip_batcher *b, const struct md5hip_iov *segs,
                               const uint64_t *seg_first, uint64_t n, unsigned char *digests,
                               uint64_t *ticket);
/* Device-resident chunks: d_ptrs[i] (a HOST array of device addresses on the
 * batcher's device, any alignment) and lens[i]; no bytes are copied.  The
 * digests go to `digests`, device memory of the batcher's device when
 * digests_on_device != 0, else host memory.  Same ticket semantics. */
int md5_batch_submit_device_async(md5hip_batcher *b, const uint64_t *d_ptrs, const uint32_t *lens,
                                  uint64_t n, unsigned char *digests, int digests_on_device,
                                  uint64_t *ticket);
int md5_batch_submit_device(md5hip_batcher *b, const uint64_t *d_ptrs, const uint32_t *lens,
                            uint64_t n, unsigned char *digests, int digests_on_device);
/* The two forms above run on the batcher's own streams with NO ordering
 * against the caller's: the chunks must be written (and the digest memory
 * free to overwrite) before the call, e.g. after hipStreamSynchronize on the
 * producer's stream.  This form takes the producer's stream instead: the
 * kernel that reads the chunks (and writes device digests) runs after all
 * work enqueued on `producer_stream` before the call, with no host sync.
 * producer_stream NULL = no ordering; it must belong to the batcher's device
 * (-EINVAL otherwise).  ticket NULL = synchronous, else as the _async form. */
int md5_batch_submit_device_on(md5hip_batcher *b, const uint64_t *d_ptrs, const uint32_t *lens,
                               uint64_t n, unsigned char *digests, int digests_on_device,
                               void *producer_stream, uint64_t *ticket);
/* ABI 3: the same with the ordering named apart from the stream, so that the
 * null stream can be the producer: order != 0 = after all work enqueued on
 * producer_stream before the call, where producer_stream NULL is the null
 * (default) stream of the batcher's device -- the stream HIP and torch use
 * when the producer names none, which the batcher's non-blocking streams do
 * NOT wait for on their own; order == 0 = no ordering (producer_stream is
 * ignored).  md5_batch_submit_device_on(.., s, ..) is this with
 * order = (s != NULL). */
int md5_batch_submit_device_after(md5hip_batcher *b, const uint64_t *d_ptrs, const uint32_t *lens,
                                  uint64_t n, unsigned char *digests, int digests_on_device,
                                  void *producer_stream, int order, uint64_t *ticket);
/* ABI 4: fixed-length device-resident chunks, digest i of (d_base +
 * i*stride, len) -- the queue form of md5hip_digest_fixed / crc32hip_fixed:
 * no per-chunk descriptor crosses PCIe (12 B per chunk through the other
 * device entries, more than a fastcrc window's HBM bytes cost), each slice
 * of at most max_chunks chunks is one launch of its own on the queue's
 * streams (several in flight overlap), digests in the batcher's kind.
 * producer_stream / order as md5_batch_submit_device_after; ticket NULL =
 * synchronous. */
int md5_batch_submit_device_fixed(md5hip_batcher *b, const void *d_base, uint64_t n, uint32_t len,
                                  uint64_t stride, unsigned char *digests, int digests_on_device,
                                  void *producer_stream, int order, uint64_t *ticket);
/* Block until submission `ticket` has delivered its digests: 0 or -errno.
 * A ticket still coalescing in the open slot is launched at once when
 * nothing is in flight (no linger); otherwise its slot goes out as soon as a
 * running launch retires (it is never forced out beside one). */
int md5_batch_wait(md5hip_batcher *b, uint64_t ticket);
/* Non-blocking: 1 = `ticket` delivered, 0 = still running (its slot is
 * hastened as by md5_batch_wait), <0 = error. */
int md5_batch_poll(md5hip_batcher *b, uint64_t ticket);
/* Launch the open slot now, whatever the in-flight count. */
int md5_batch_flush(md5hip_batcher *b);

/* Batched verify (cache read / write verify sites, blk_io.c:665-704,
 * bc_mgr.c:1464-1492): ok[i] = (digest of chunk i == expected[i]), expected
 * holding 16 (MD5) or 4 (CRC32) bytes per chunk.  Returns the number of
 * mismatches (>= 0) or -errno; the caller keeps its per-block EAGAIN /
 * inode-reset policy (blk_io.c:693-703). */
int md5hip_batch_verify_iov(md5hip_batcher *b, const struct md5hip_iov *segs,
                            const uint64_t *seg_first, uint64_t n, const void *expected,
                            unsigned char *ok);

/*
 * Zero-copy input.  md5hip_host_register pins and device-maps host memory
 * for every device (hipHostRegister, portable + mapped) -- e.g. each bulk of
 * netcache's page heap as it is allocated (bc_mgr.c:1260-1290).  A batcher
 * whose gather mode is not HOST then skips the host memcpy into its staging
 * slice for any call whose segments all lie in registered memory:
 *   DEVICE  a gather kernel reads the segments over PCIe into HBM;
 *   DMA     one async DMA copy per run of contiguous segments;
 *   AUTO    (default) per slice, DMA when the runs average >= 256 KiB,
 *           else DEVICE.
 * Other calls (or mode HOST) gather on the host into the pinned slice.
 * Ranges must not overlap (-EEXIST); unregister with the same base.
 */
enum md5hip_gather_mode {
    MD5HIP_GATHER_HOST = 0,
    MD5HIP_GATHER_DEVICE = 1,
    MD5HIP_GATHER_DMA = 2,
    MD5HIP_GATHER_AUTO = 3
};
int md5hip_host_register(void *base, uint64_t bytes);
int md5hip_host_unregister(void *base);
int md5hip_batcher_set_gather(md5hip_batcher *b, int mode);

/* digests[i] = MD5(h_base + i*stride, len) from one contiguous host buffer,
 * copied slice by slice with no host gather.  A source the runtime has
 * page-locked over its WHOLE range (hipHostMalloc, hipHostRegister, or
 * md5hip_host_register) is DMA'd in place at full PCIe rate; any other --
 * pageable, or pinned only in part -- is copied through the slot's pinned
 * staging by the calling thread first. */
int md5hip_batch_host_fixed(md5hip_batcher *b, const void *h_base, uint64_t n, uint32_t len,
                            uint64_t stride, unsigned char *digests);

/*
 * Multi-GPU host pool: a router over one coalescing batcher
 * per listed device (a device may be listed more than once).  Chunks are
 * independent, so no collective is needed.  Each submission goes WHOLE to
 * the device whose batcher holds the least outstanding work (bytes reserved
 * and not yet delivered), so a netcache vector keeps its one launch and
 * coalesces there with other threads' vectors.  Only a submission larger than
 * the split threshold (default: one batcher slice) is cut into contiguous
 * byte-balanced ranges (md5hip_pool_plan) over the least-loaded devices.
 * No pool-wide lock is held across device work and no thread is created per
 * call: any number of threads (the ASIO pool, asio_mgr.c:205, :1050-1057)
 * may submit concurrently.  Same results and errors as the batcher entries.
 */
typedef struct md5hip_pool md5hip_pool;

int md5hip_pool_create(const int *devices, uint32_t ndev, uint64_t slice_bytes, uint32_t nslots,
                       md5hip_pool **out);
/* Waits for everything in flight, then frees. */
void md5hip_pool_destroy(md5hip_pool *p);
int md5hip_pool_ndev(const md5hip_pool *p);
/* The digest kind of later submissions (submissions already made keep
 * theirs); MD5 or CRC32 with a fastcrc window as md5hip_batcher_set_digest. */
int md5hip_pool_set_digest(md5hip_pool *p, int kind, uint32_t fastcrc);
int md5hip_pool_set_gather(md5hip_pool *p, int mode);
/* Submissions above `bytes` (sum of chunk lengths) are split over devices;
 * 0 = one batcher slice (the default). */
int md5hip_pool_set_split(md5hip_pool *p, uint64_t bytes);
int md5hip_pool_submit(md5hip_pool *p, const void *const *ptrs, const uint32_t *lens, uint64_t n,
                       unsigned char *digests);
int md5hip_pool_submit_iov(md5hip_pool *p, const struct md5hip_iov *segs,
                           const uint64_t *seg_first, uint64_t n, unsigned char *digests);
int md5hip_pool_verify_iov(md5hip_pool *p, const struct md5hip_iov *segs,
                           const uint64_t *seg_first, uint64_t n, const void *expected,
                           unsigned char *ok);
int md5hip_pool_host_fixed(md5hip_pool *p, const void *h_base, uint64_t n, uint32_t len,
                           uint64_t stride, unsigned char *digests);
/* Asynchronous forms, ticket semantics as md5_batch_submit_async: the call
 * returns once the chunks are staged, *ticket (0 for an empty submission)
 * completes when every device holding its chunks has delivered them, and
 * `digests` must stay valid until then.  A pool ticket is only meaningful to
 * the pool that issued it. */
int md5hip_pool_submit_async(md5hip_pool *p, const void *const *ptrs, const uint32_t *lens,
                             uint64_t n, unsigned char *digests, uint64_t *ticket);
int md5hip_pool_submit_iov_async(md5hip_pool *p, const struct md5hip_iov *segs,
                                 const uint64_t *seg_first, uint64_t n, unsigned char *digests,
                                 uint64_t *ticket);
/* 0 or the ticket's own -errno (first failing part); -EINVAL if unknown. */
int md5hip_pool_wait(md5hip_pool *p, uint64_t ticket);
/* 1 = delivered, 0 = running, <0 = its error. */
int md5hip_pool_poll(md5hip_pool *p, uint64_t ticket);

struct md5hip_pool_stats {
    uint64_t submissions;             /* non-empty submissions */
    uint64_t routed_whole;            /* went whole to one device */
    uint64_t split;                   /* cut over several devices */
    uint64_t parts;                   /* device submissions made in all */
};
int md5hip_pool_get_stats(md5hip_pool *p, struct md5hip_pool_stats *out);
/* Device g's batcher counters (launches, coalesced launches, ...). */
int md5hip_pool_device_stats(md5hip_pool *p, uint32_t g, struct md5hip_batcher_stats *out);

/* ABI 4: failed devices (md5hip_batcher_health).  The router never picks a
 * failed device.  A submission that finds its device failed before the
 * device took its chunks (-ENODEV) is routed to another one; a synchronous
 * submission (or split part) whose launch then fails is resubmitted on a
 * healthy device from the caller's still-valid buffers, so it returns 0 as
 * long as one device is left.  An asynchronous ticket on a device that
 * fails completes with -EIO (its launch failed) or -ENODEV (it had not
 * been launched yet): it is not moved, as its buffers may be gone by the
 * wait.  With every device failed, submissions return -ENODEV.
 * md5hip_pool_device_health: 0 / -ENODEV for device index g (-EINVAL
 * past ndev); md5hip_pool_inject_fault: md5hip_batcher_inject_fault on
 * device index g. */
struct md5hip_pool_health {
    uint32_t ndev;
    uint32_t nfailed;                 /* devices failed */
    uint64_t failed_mask;             /* bit g: device index g failed (g < 64) */
    uint64_t failovers;               /* submissions or parts moved off a failed device */
};
int md5hip_pool_get_health(md5hip_pool *p, struct md5hip_pool_health *out);
int md5hip_pool_device_health(md5hip_pool *p, uint32_t g);
int md5hip_pool_inject_fault(md5hip_pool *p, uint32_t g, uint64_t after);

/* The pool's split, exposed for callers and tests (host only, synchronous):
 * first[0..nparts] such that part g is chunks [first[g], first[g+1]).
 * lens == NULL: equal counts, first[g] = g*n/nparts.  Otherwise contiguous
 * ranges of near-equal weight, weight(chunk) = len + 64. */
int md5hip_pool_plan(const uint32_t *lens, uint64_t n, uint32_t nparts, uint64_t *first);

#ifdef __cplusplus
}
#endif

#endif /* SPROXY_AMD_MD5HIP_H */
