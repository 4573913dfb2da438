/*
 * fake_hip.c -- TEST INFRASTRUCTURE: just enough of the HIP runtime, and of
 * the library's device entries, for the batcher (sproxy_amd/csrc/md5_submit.c)
 * and the pool to run on a machine with no GPU, under ASan or TSan
 * (tests/test_batcher_host.py, tests/c/batcher_check.c).
 *
 *   - "device" memory is host memory; device pointers are host pointers;
 *   - a stream executes each operation when it is enqueued (copies and
 *     "kernels" run at once, on the calling thread);
 *   - an event recorded on a stream reports hipErrorNotReady for 0-3 queries
 *     (a per-event pseudo-random count) before hipSuccess, so slots stay in
 *     flight for a while and the batcher's progress thread, coalescing and
 *     out-of-order completion all run;
 *   - the "kernels" compute the digests on the CPU with the library's own
 *     host MD5 (md5_stream.c) and CRC-32 (nc_digest.c);
 *   - a stream remembers the device current at its creation, and every copy
 *     or "kernel" enqueued on it from a thread whose current device differs
 *     is counted in fake_hip_wrong_device (the real runtime keys state such
 *     as the BALANCED counter and CU counts on hipGetDevice);
 *   - test controls: fake_hip_hold keeps every event NotReady; for an
 *     event recorded while fake_hip_slow_query is set, the first query made from a
 *     thread marked by fake_hip_mark_thread() takes 600 us and answers
 *     NotReady while the event turns ready for every other caller (until
 *     then it answers NotReady to unmarked threads) -- a
 *     waiter's bounded spin then ends on NotReady just after the kernel
 *     finished, and the progress thread retires the launch before the waiter
 *     holds the lock again (the lost-wakeup race of a blocked caller);
 *   - device lost after launch K (fake_hip_lose_device): the K-th kernel
 *     enqueued on a device from then on faults.  how 0: it is enqueued, and
 *     every event recorded on that device from then on reports
 *     hipErrorLaunchFailure when it completes; once one has, every copy,
 *     kernel and stream wait on the device fails too.  how 1: that kernel's
 *     launch itself fails, and everything after it.  hipStreamQuery reports
 *     the loss either way (what the batcher classifies an enqueue error by).
 * Nothing here is part of the product.
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "md5.h"
#include "md5hip.h"
#include "nc_digest.h"
#include "../../sproxy_amd/csrc/md5_internal.h"

struct ihipEvent_t {
    int left;                     /* queries still answered NotReady */
    int bad;                      /* recorded on a device that had faulted: completes with an error */
    int device;
    unsigned seed;
    int slow;                     /* recorded while fake_hip_slow_query was set */
    int slow_done;                /* the slow query of this record happened */
};
struct ihipStream_t {
    int device;
};

static __thread int t_device;
static __thread int t_marked;
unsigned long fake_hip_wrong_device;
int fake_hip_hold, fake_hip_slow_query;
void fake_hip_mark_thread(void) { t_marked = 1; }

static void on_stream(hipStream_t stream)
{
    if (stream && stream->device != t_device)
        __atomic_fetch_add(&fake_hip_wrong_device, 1, __ATOMIC_RELAXED);
}

/* device loss (all under g_lose_mu) */
static pthread_mutex_t g_lose_mu = PTHREAD_MUTEX_INITIALIZER;
static int g_lose_after[8], g_lose_how[8], g_kernels[8];
static int g_faulted[8];          /* the fault happened */
static int g_reported[8];         /* ... and the runtime has said so: enqueues fail */
static unsigned long g_lost_kernels;

static int stream_dev(hipStream_t s) { return s ? s->device : t_device; }

void fake_hip_lose_device(int dev, int after_kernels, int how)
{
    pthread_mutex_lock(&g_lose_mu);
    g_lose_after[dev] = g_kernels[dev] + after_kernels;
    g_lose_how[dev] = how;
    pthread_mutex_unlock(&g_lose_mu);
}

int fake_hip_device_faulted(int dev)
{
    pthread_mutex_lock(&g_lose_mu);
    const int f = g_faulted[dev];
    pthread_mutex_unlock(&g_lose_mu);
    return f;
}

/* an enqueue on `s`: hipErrorLaunchFailure once its device's loss is known */
static hipError_t enqueue_ok(hipStream_t s)
{
    pthread_mutex_lock(&g_lose_mu);
    const int bad = g_reported[stream_dev(s)];
    pthread_mutex_unlock(&g_lose_mu);
    return bad ? hipErrorLaunchFailure : hipSuccess;
}

/* a kernel enqueued on `stream`: 0, or -EIO if the launch fails */
static int kernel_begin(hipStream_t stream)
{
    on_stream(stream);
    const int d = stream_dev(stream);
    pthread_mutex_lock(&g_lose_mu);
    int rc = g_reported[d] ? -EIO : 0;
    if (!rc && g_lose_after[d] && ++g_kernels[d] >= g_lose_after[d] && !g_faulted[d]) {
        g_faulted[d] = 1;
        if (g_lose_how[d]) {
            g_reported[d] = 1;
            rc = -EIO;
        }
    } else if (!rc && !g_lose_after[d]) {
        g_kernels[d]++;
    }
    if (rc) g_lost_kernels++;
    pthread_mutex_unlock(&g_lose_mu);
    return rc;
}
/* a launch holding a chunk of this length fails with -EIO (error paths) */
uint32_t fake_hip_fail_len = 0xffffffffu;
static pthread_mutex_t g_ev_mu = PTHREAD_MUTEX_INITIALIZER;

hipError_t hipGetDevice(int *deviceId) { *deviceId = t_device; return hipSuccess; }
hipError_t hipSetDevice(int deviceId) { if (deviceId < 0 || deviceId > 7) return hipErrorInvalidDevice; t_device = deviceId; return hipSuccess; }
hipError_t hipGetDeviceCount(int *count) { *count = 8; return hipSuccess; }

/* page-locked host ranges the "runtime" knows (hipHostMalloc, hipHostRegister):
 * what hipPointerGetAttributes / the RANGE attributes / hipMemGetAddressRange
 * answer from.  An H2D copy whose source overlaps a watched range
 * (fake_hip_watch) but is not wholly inside one page-locked range is DMA
 * from pageable memory, counted in fake_hip_pageable_dma (every H2D copy
 * from the watched range: fake_hip_watched_h2d). */
#define NPIN 256
static pthread_mutex_t g_pin_mu = PTHREAD_MUTEX_INITIALIZER;
static uintptr_t g_pin_lo[NPIN], g_pin_hi[NPIN];
static uintptr_t g_watch_lo, g_watch_hi;
unsigned long fake_hip_pageable_dma, fake_hip_watched_h2d;

static void pin_add(const void *p, size_t len)
{
    pthread_mutex_lock(&g_pin_mu);
    for (int i = 0; i < NPIN; i++)
        if (!g_pin_hi[i]) {
            g_pin_lo[i] = (uintptr_t)p;
            g_pin_hi[i] = (uintptr_t)p + (len ? len : 1);
            break;
        }
    pthread_mutex_unlock(&g_pin_mu);
}

static void pin_del(const void *p)
{
    pthread_mutex_lock(&g_pin_mu);
    for (int i = 0; i < NPIN; i++)
        if (g_pin_hi[i] && g_pin_lo[i] == (uintptr_t)p) g_pin_lo[i] = g_pin_hi[i] = 0;
    pthread_mutex_unlock(&g_pin_mu);
}

/* the page-locked range holding p: its index, or -1 */
static int pin_find(uintptr_t p)
{
    for (int i = 0; i < NPIN; i++)
        if (g_pin_hi[i] && g_pin_lo[i] <= p && p < g_pin_hi[i]) return i;
    return -1;
}

/* test controls: a page-locked range with no allocation of its own (a block
 * pinned by someone else), and the range whose H2D copies are checked */
void fake_hip_pin(const void *p, size_t len) { pin_add(p, len); }
void fake_hip_unpin(const void *p) { pin_del(p); }
void fake_hip_watch(const void *p, size_t len)
{
    pthread_mutex_lock(&g_pin_mu);
    g_watch_lo = (uintptr_t)p;
    g_watch_hi = (uintptr_t)p + len;
    pthread_mutex_unlock(&g_pin_mu);
}

static void h2d_check(const void *src, size_t len)
{
    const uintptr_t lo = (uintptr_t)src, hi = lo + len;
    pthread_mutex_lock(&g_pin_mu);
    if (len && lo < g_watch_hi && g_watch_lo < hi) {
        fake_hip_watched_h2d++;
        const int i = pin_find(lo);
        if (i < 0 || hi > g_pin_hi[i]) fake_hip_pageable_dma++;
    }
    pthread_mutex_unlock(&g_pin_mu);
}

hipError_t hipMalloc(void **ptr, size_t size) { *ptr = malloc(size ? size : 1); return *ptr ? hipSuccess : hipErrorOutOfMemory; }
hipError_t hipHostMalloc(void **ptr, size_t size, unsigned int flags)
{
    (void)flags;
    const hipError_t e = hipMalloc(ptr, size);
    if (e == hipSuccess) pin_add(*ptr, size);
    return e;
}
hipError_t hipFree(void *ptr) { free(ptr); return hipSuccess; }
hipError_t hipHostFree(void *ptr) { pin_del(ptr); free(ptr); return hipSuccess; }
hipError_t hipHostRegister(void *hostPtr, size_t sizeBytes, unsigned int flags) { (void)flags; pin_add(hostPtr, sizeBytes); return hipSuccess; }
hipError_t hipHostUnregister(void *hostPtr) { pin_del(hostPtr); return hipSuccess; }
hipError_t hipHostGetDevicePointer(void **devPtr, void *hstPtr, unsigned int flags) { (void)flags; *devPtr = hstPtr; return hipSuccess; }
/* page-locked memory answers hipMemoryTypeHost; any other pointer is unknown
 * to the runtime (pageable malloc memory: hipErrorInvalidValue) */
hipError_t hipPointerGetAttributes(hipPointerAttribute_t *attributes, const void *ptr)
{
    pthread_mutex_lock(&g_pin_mu);
    const int i = pin_find((uintptr_t)ptr);
    pthread_mutex_unlock(&g_pin_mu);
    if (i < 0) return hipErrorInvalidValue;
    memset(attributes, 0, sizeof *attributes);
    attributes->type = hipMemoryTypeHost;
    attributes->hostPointer = (void *)ptr;
    attributes->devicePointer = (void *)ptr;
    return hipSuccess;
}
/* extent of the page-locked allocation holding ptr; fake_hip_no_range: the
 * runtime will not say (the batcher then stages) */
int fake_hip_no_range;
hipError_t hipPointerGetAttribute(void *data, hipPointer_attribute attribute, hipDeviceptr_t ptr)
{
    pthread_mutex_lock(&g_pin_mu);
    const int i = pin_find((uintptr_t)ptr);
    const uintptr_t lo = i < 0 ? 0 : g_pin_lo[i], hi = i < 0 ? 0 : g_pin_hi[i];
    pthread_mutex_unlock(&g_pin_mu);
    if (i < 0 || __atomic_load_n(&fake_hip_no_range, __ATOMIC_RELAXED)) return hipErrorInvalidValue;
    if (attribute == HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR) *(void **)data = (void *)lo;
    else if (attribute == HIP_POINTER_ATTRIBUTE_RANGE_SIZE) *(size_t *)data = hi - lo;
    else return hipErrorInvalidValue;
    return hipSuccess;
}
hipError_t hipMemGetAddressRange(hipDeviceptr_t *pbase, size_t *psize, hipDeviceptr_t dptr)
{
    pthread_mutex_lock(&g_pin_mu);
    const int i = pin_find((uintptr_t)dptr);
    const uintptr_t lo = i < 0 ? 0 : g_pin_lo[i], hi = i < 0 ? 0 : g_pin_hi[i];
    pthread_mutex_unlock(&g_pin_mu);
    if (i < 0 || __atomic_load_n(&fake_hip_no_range, __ATOMIC_RELAXED)) return hipErrorInvalidValue;
    *pbase = (hipDeviceptr_t)lo;
    *psize = hi - lo;
    return hipSuccess;
}
hipError_t hipGetLastError(void) { return hipSuccess; }

hipError_t hipStreamCreateWithFlags(hipStream_t *stream, unsigned int flags)
{
    (void)flags;
    *stream = calloc(1, sizeof(struct ihipStream_t));
    if (!*stream) return hipErrorOutOfMemory;
    (*stream)->device = t_device;
    return hipSuccess;
}
hipError_t hipStreamDestroy(hipStream_t stream) { free(stream); return hipSuccess; }
hipError_t hipStreamWaitEvent(hipStream_t stream, hipEvent_t event, unsigned int flags) { (void)event; (void)flags; return enqueue_ok(stream); }
hipError_t hipStreamQuery(hipStream_t stream)
{
    pthread_mutex_lock(&g_lose_mu);
    const int f = g_faulted[stream_dev(stream)];
    pthread_mutex_unlock(&g_lose_mu);
    return f ? hipErrorLaunchFailure : hipSuccess;
}

hipError_t hipEventCreateWithFlags(hipEvent_t *event, unsigned flags)
{
    (void)flags;
    *event = calloc(1, sizeof(struct ihipEvent_t));
    if (!*event) return hipErrorOutOfMemory;
    (*event)->seed = (unsigned)(uintptr_t)*event;
    return hipSuccess;
}
hipError_t hipEventDestroy(hipEvent_t event) { free(event); return hipSuccess; }
hipError_t hipEventRecord(hipEvent_t event, hipStream_t stream)
{
    pthread_mutex_lock(&g_lose_mu);
    const int bad = g_faulted[stream_dev(stream)];
    pthread_mutex_unlock(&g_lose_mu);
    pthread_mutex_lock(&g_ev_mu);
    event->bad = bad;
    event->device = stream_dev(stream);
    event->seed = event->seed * 1103515245u + 12345u;
    event->left = (int)((event->seed >> 16) % 4u);
    event->slow = __atomic_load_n(&fake_hip_slow_query, __ATOMIC_RELAXED);
    event->slow_done = 0;
    pthread_mutex_unlock(&g_ev_mu);
    return hipSuccess;
}
hipError_t hipEventQuery(hipEvent_t event)
{
    pthread_mutex_lock(&g_ev_mu);
    if (__atomic_load_n(&fake_hip_hold, __ATOMIC_RELAXED)) {
        pthread_mutex_unlock(&g_ev_mu);
        return hipErrorNotReady;
    }
    if (event->slow && !event->slow_done && !t_marked) {
        pthread_mutex_unlock(&g_ev_mu);             /* running until a marked thread has looked */
        return hipErrorNotReady;
    }
    if (event->slow && !event->slow_done && t_marked) {
        event->slow_done = 1;
        event->left = 0;                          /* ready for everyone else from now */
        pthread_mutex_unlock(&g_ev_mu);
        const struct timespec ts = {0, 600000};
        nanosleep(&ts, NULL);
        return hipErrorNotReady;                  /* ... but this caller saw it running */
    }
    const int ready = event->left == 0;
    if (!ready) event->left--;
    const int bad = ready && event->bad;
    const int dev = event->device;
    pthread_mutex_unlock(&g_ev_mu);
    if (bad) {                                    /* the runtime has seen the fault now */
        pthread_mutex_lock(&g_lose_mu);
        g_reported[dev] = 1;
        pthread_mutex_unlock(&g_lose_mu);
        return hipErrorLaunchFailure;
    }
    return ready ? hipSuccess : hipErrorNotReady;
}
hipError_t hipEventSynchronize(hipEvent_t event)
{
    while (__atomic_load_n(&fake_hip_hold, __ATOMIC_RELAXED)) {
        const struct timespec ts = {0, 100000};
        nanosleep(&ts, NULL);
    }
    pthread_mutex_lock(&g_ev_mu);
    event->left = 0;
    const int bad = event->bad;
    pthread_mutex_unlock(&g_ev_mu);
    return bad ? hipErrorLaunchFailure : hipSuccess;
}

hipError_t hipMemcpyAsync(void *dst, const void *src, size_t sizeBytes, hipMemcpyKind kind, hipStream_t stream)
{
    on_stream(stream);
    const hipError_t e = enqueue_ok(stream);
    if (e != hipSuccess) return e;
    if (kind == hipMemcpyHostToDevice) h2d_check(src, sizeBytes);
    if (sizeBytes) memmove(dst, src, sizeBytes);
    return hipSuccess;
}

/* ------------------------------------------------------------------ "kernels" */
static void md5_of(const unsigned char *p, uint32_t len, unsigned char *out)
{
    struct MD5Context c;
    MD5Init(&c);
    MD5Update(&c, p, len);
    MD5Final(out, &c);
}

static uint32_t blk_crc(const unsigned char *p, uint32_t len, uint32_t F)
{
    if (F == 0 || len <= F) return nc_crc32(p, len);                   /* blk_io.c:408-424 */
    return nc_crc32(p, F) ^ nc_crc32(p + (len - F), F);
}

int md5hip_digest_fixed(const void *d_base, uint64_t n, uint32_t len, uint64_t stride,
                        unsigned char *d_digests, void *stream)
{
    if (kernel_begin((hipStream_t)stream)) return -EIO;
    for (uint64_t i = 0; i < n; i++) md5_of((const unsigned char *)d_base + i * stride, len, d_digests + 16 * i);
    return 0;
}

int crc32hip_fixed(const void *d_base, uint64_t n, uint32_t len, uint64_t stride, uint32_t fastcrc,
                   uint32_t *d_crcs, void *stream)
{
    if (kernel_begin((hipStream_t)stream)) return -EIO;
    for (uint64_t i = 0; i < n; i++) d_crcs[i] = blk_crc((const unsigned char *)d_base + i * stride, len, fastcrc);
    return 0;
}

int md5hip_digest_desc_variant(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
                               const uint32_t *d_order, uint64_t n, unsigned char *d_digests,
                               void *stream, int variant)
{
    if (kernel_begin((hipStream_t)stream)) return -EIO;
    (void)variant;
    if (((uintptr_t)d_digests & 15u) != 0) return -EINVAL;
    for (uint64_t k = 0; k < n; k++)
        if (d_lens[k] == fake_hip_fail_len) return -EIO;
    if (getenv("FAKE_HIP_NOHASH")) return 0;         /* host-side cost probes: no digests */
    for (uint64_t k = 0; k < n; k++) {               /* lanes in `order`, digests by chunk */
        const uint64_t c = d_order ? d_order[k] : k;
        if (c >= n) return -EINVAL;
        md5_of((const unsigned char *)((uintptr_t)d_base + d_offsets[c]), d_lens[c], d_digests + 16 * c);
    }
    return 0;
}

int crc32hip_desc(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
                  const uint32_t *d_order, uint64_t n, uint32_t fastcrc, uint32_t *d_crcs, void *stream)
{
    if (kernel_begin((hipStream_t)stream)) return -EIO;
    for (uint64_t k = 0; k < n; k++) {
        const uint64_t c = d_order ? d_order[k] : k;
        if (c >= n) return -EINVAL;
        d_crcs[c] = blk_crc((const unsigned char *)((uintptr_t)d_base + d_offsets[c]), d_lens[c], fastcrc);
    }
    return 0;
}

int crc32hip_desc_variant(const void *d_base, const uint64_t *d_offsets, const uint32_t *d_lens,
                          const uint32_t *d_order, uint64_t n, uint32_t fastcrc, uint32_t *d_crcs,
                          void *stream, int variant)
{
    if (variant != 0 && variant != 6 && variant != 7) return -EINVAL;
    return crc32hip_desc(d_base, d_offsets, d_lens, d_order, n, fastcrc, d_crcs, stream);
}

int md5hip_lines_choice(int variant, uint64_t unlined_bytes, uint64_t bytes)
{
    return variant == MD5HIP_DESC_XDMA && 2 * unlined_bytes > bytes ? MD5HIP_DESC_LINES : variant;
}

int md5hip_crc_desc_choice(uint64_t n, uint64_t mean_len)
{
    return (mean_len >= 2048 ? n <= 128 * 256 : n <= 12 * 256) ? 7 : 6;
}

int md5hip_gather_launch(const struct md5hip_seg *d_segs, uint64_t nseg, unsigned char *d_dst, void *stream)
{
    on_stream((hipStream_t)stream);
    if (enqueue_ok((hipStream_t)stream) != hipSuccess) return -EIO;
    for (uint64_t k = 0; k < nseg; k++)
        memmove((void *)((uintptr_t)d_dst + d_segs[k].dst), (const void *)(uintptr_t)d_segs[k].src, d_segs[k].len);
    return 0;
}

/* longest-first by key (len >> 6) + 1, stable (md5hip_plan_order) */
int md5hip_plan_desc(const uint32_t *lens, uint64_t n, uint32_t *order)
{
    if (!lens || !order) return n ? -EINVAL : 0;
    uint32_t kmax = 0;
    for (uint64_t i = 0; i < n; i++) if ((lens[i] >> 6) + 1 > kmax) kmax = (lens[i] >> 6) + 1;
    uint64_t at = 0;
    for (int64_t k = kmax; k >= 1; k--)               /* O(n * keys): test sizes only */
        for (uint64_t i = 0; i < n; i++)
            if ((lens[i] >> 6) + 1 == (uint32_t)k) order[at++] = (uint32_t)i;
    return MD5HIP_DESC_XDMA;
}

int md5hip_plan_hist(const uint32_t *hist, uint32_t kmax, uint64_t n, uint32_t *bucket_start)
{
    if (!hist) return -EINVAL;
    uint64_t sum = 0;                                 /* the batcher's histogram counts every chunk */
    for (uint32_t k = 1; k <= kmax; k++) sum += hist[k];
    if (sum != n) return -EBADMSG;
    if (bucket_start) {
        uint64_t at = 0;
        for (int64_t k = kmax; k >= 1; k--) {
            bucket_start[kmax - k] = (uint32_t)at;
            at += hist[k];
        }
        bucket_start[kmax] = (uint32_t)n;
    }
    return MD5HIP_DESC_XDMA;
}

int md5hip_order_device(const uint32_t *d_lens, uint64_t n, uint32_t kmax, uint32_t *d_bucket_next,
                        uint32_t *d_order, void *stream)
{
    on_stream((hipStream_t)stream);
    if (enqueue_ok((hipStream_t)stream) != hipSuccess) return -EIO;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t k = (d_lens[i] >> 6) + 1;
        if (k > kmax) continue;
        const uint32_t pos = d_bucket_next[kmax - k]++;
        if (pos < n) d_order[pos] = (uint32_t)i;
    }
    return 0;
}

/* the stable longest-first order: a counting sort by key, equal keys in
 * chunk order (md5hip_order_device_stable's contract).  Every third call is
 * refused with -ENOSPC (scratch too small), so the batcher's fallback to
 * order_scatter runs too. */
static unsigned long g_sort_calls;
unsigned long fake_hip_sort_refused;
uint64_t md5hip_order_stable_scratch(uint64_t n, uint32_t kmax)
{
    (void)kmax;
    return n ? 4 * n + 256 : 0;
}

int md5hip_order_device_stable(const uint32_t *d_lens, uint64_t n, uint32_t kmax, void *d_scratch,
                               uint64_t scratch_bytes, uint32_t *d_order, void *stream)
{
    on_stream((hipStream_t)stream);
    if (enqueue_ok((hipStream_t)stream) != hipSuccess) return -EIO;
    if (n == 0) return 0;
    if (!d_lens || !d_order || !d_scratch || !kmax || scratch_bytes < 4 * n) return -EINVAL;
    if (__atomic_add_fetch(&g_sort_calls, 1, __ATOMIC_RELAXED) % 3 == 0) {
        __atomic_fetch_add(&fake_hip_sort_refused, 1, __ATOMIC_RELAXED);
        return -ENOSPC;
    }
    uint64_t *start = calloc((size_t)kmax + 2, sizeof *start);     /* by bucket kmax - key */
    if (!start) return -ENOMEM;
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t k = (d_lens[i] >> 6) + 1;
        start[(k <= kmax ? kmax - k : kmax) + 1]++;
    }
    for (uint32_t b = 1; b <= kmax + 1; b++) start[b] += start[b - 1];
    for (uint64_t i = 0; i < n; i++) {
        const uint32_t k = (d_lens[i] >> 6) + 1;
        d_order[start[k <= kmax ? kmax - k : kmax]++] = (uint32_t)i;
    }
    free(start);
    return 0;
}

