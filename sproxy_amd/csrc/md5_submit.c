/*
 * md5_submit.c -- the batcher: a thread-safe, coalescing submission queue in
 * front of the batched kernels (include/md5hip.h).
 *
 * Serves the netcache block-completion checksum site (blk_make_crc,
 * netcache/common/blk_io.c:354-430, called from ASIO pool threads,
 * asio_mgr.c:1054-1057): chunks live in host memory (cache pages, socket
 * buffers) or already in HBM, and each caller wants its own digests back.
 *
 * A batcher owns `nslots` pipeline slots.  Slot k has its own HIP stream,
 * pinned staging, device buffers, descriptor arrays and completion event.
 * At most one slot is OPEN at a time: submissions (from any thread) append
 * their chunks to it -- host chunks are gathered into its pinned staging,
 * device-resident chunks only add a descriptor -- and the slot is launched
 * as ONE planned descriptor batch (md5hip_plan_desc) when
 *   - it is full (bytes, descriptors or gather segments), or
 *   - fewer than `target` slots are in flight (an idle pipeline takes work at
 *     once: no added latency when the device is not busy), or
 *   - a caller waits on / polls / flushes a ticket it holds.
 * So while the device is busy, everything submitted meanwhile is coalesced
 * into the next launch: a 1 MiB chunk's serial chain (~10 ms) then runs
 * beside the bytes of many later submissions instead of ending its launch
 * alone.
 *
 * Completion is per ticket and out of order: a ticket completes when every
 * slot holding its chunks has finished, whatever earlier tickets are doing.
 * A progress thread per batcher polls the in-flight slots' events, delivers
 * host digests (D2H staging -> the caller's array), retires slots and
 * launches the open slot when the pipeline drains below `target`.
 *
 * Locking: b->mu guards all batcher state; HIP enqueue calls are made under
 * it (they are asynchronous); host gathers (memcpy) run outside it, the slot
 * held open by a writer count.  Lock order: b->mu, then g_reg_lock.
 *
 * Every entry saves and restores the calling thread's HIP device.
 * Errors: 0 / negative errno (include/md5hip.h); -E2BIG when one chunk
 * exceeds the slot's staging; -EFAULT when registered memory vanished
 * under a zero-copy submission.
 *
 * Device failure.  blk_make_crc cannot fail (blk_io.c:354-430); this can.
 * A launch whose completion event reports an error, or an enqueue failure
 * after which the slot's stream reports one, marks the batcher FAILED
 * (sticky): that launch's tickets get -EIO, tickets still coalescing in the
 * open slot and every later submission get -ENODEV at once, and nothing is
 * enqueued on the device again.  Launches already in flight complete as
 * their events say.  No digest of a failed launch is delivered.  The pool
 * (md5_pool.c) routes around a failed batcher; what the call site does with
 * -EIO / -ENODEV is INTEGRATION.md §2j.
 */
#include <errno.h>
#include <pthread.h>
#include <sys/prctl.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include <hip/hip_runtime_api.h>

#include "../../include/md5hip.h"
#include "md5_internal.h"
#include "md5_tickets.h"

/* ------------------------------------------------------------------------
 * Registered host ranges (zero-copy input).  netcache allocates its cache
 * pages in 4 KiB-aligned bulks (bc_mgr.c:1260-1290); a bulk registered here
 * is pinned and mapped for every device, so the batcher can let the device
 * (or the DMA engine) pull the pages directly instead of memcpy'ing them into
 * the pinned staging slice on the host.
 * ------------------------------------------------------------------------ */
#define REG_MAXDEV 16
struct reg_range {
    uintptr_t lo, hi;
    intptr_t delta[REG_MAXDEV];       /* device-visible address - host address */
};
static struct reg_range *g_reg;
static size_t g_nreg, g_capreg;
static pthread_rwlock_t g_reg_lock = PTHREAD_RWLOCK_INITIALIZER;

/* index of the range containing [p, p+len), or -1 (caller holds the lock) */
static long reg_find(uintptr_t p, uint64_t len)
{
    size_t lo = 0, hi = g_nreg;
    while (lo < hi) {
        const size_t mid = (lo + hi) / 2;
        if (g_reg[mid].hi <= p) lo = mid + 1;
        else hi = mid;
    }
    if (lo < g_nreg && g_reg[lo].lo <= p && p + len <= g_reg[lo].hi) return (long)lo;
    return -1;
}

/* The caller's HIP device, restored on every exit from an entry. */
struct dev_guard { int prev; int ok; };
static int dev_enter(struct dev_guard *g, int device)
{
    g->ok = hipGetDevice(&g->prev) == hipSuccess;
    if (hipSetDevice(device) != hipSuccess) {
        (void)hipGetLastError();      /* ours: returned as -ENODEV, not left for the caller's next check */
        if (g->ok) (void)hipSetDevice(g->prev);
        return -ENODEV;
    }
    return 0;
}
static void dev_leave(const struct dev_guard *g)
{
    if (g->ok) (void)hipSetDevice(g->prev);
}

int md5hip_host_register(void *base, uint64_t bytes)
{
    if (!base || bytes == 0) return -EINVAL;
    const uintptr_t lo = (uintptr_t)base, hi = lo + bytes;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -ENODEV;
    if (ndev > REG_MAXDEV) ndev = REG_MAXDEV;
    struct dev_guard g;
    (void)hipGetDevice(&g.prev);
    g.ok = 1;
    pthread_rwlock_wrlock(&g_reg_lock);
    int rc = 0;
    size_t at = 0;
    while (at < g_nreg && g_reg[at].hi <= lo) at++;
    if (at < g_nreg && g_reg[at].lo < hi) { rc = -EEXIST; goto out; }     /* overlap */
    if (g_nreg == g_capreg) {
        size_t cap = g_capreg ? 2 * g_capreg : 64;
        struct reg_range *r = realloc(g_reg, cap * sizeof *r);
        if (!r) { rc = -ENOMEM; goto out; }
        g_reg = r;
        g_capreg = cap;
    }
    /* coarse-grained: the batcher reads a range only between the caller's
     * writes, and DMA from coarse-grained pages runs 44 vs 34 GB/s
     * (DESIGN.md §5); MD5HIP_REGISTER_COARSE=0 turns it off */
    unsigned flags = hipHostRegisterPortable | hipHostRegisterMapped;
    const char *coarse = getenv("MD5HIP_REGISTER_COARSE");
    if (!coarse || atoi(coarse)) flags |= hipExtHostRegisterCoarseGrained;
    if (hipHostRegister(base, bytes, flags) != hipSuccess) {
        rc = -ENODEV;
        goto out;
    }
    struct reg_range r = {lo, hi, {0}};
    for (int d = 0; d < ndev; d++) {
        void *dp = NULL;
        if (hipSetDevice(d) == hipSuccess && hipHostGetDevicePointer(&dp, base, 0) == hipSuccess)
            r.delta[d] = (intptr_t)((uintptr_t)dp - lo);
    }
    memmove(&g_reg[at + 1], &g_reg[at], (g_nreg - at) * sizeof *g_reg);
    g_reg[at] = r;
    g_nreg++;
out:
    pthread_rwlock_unlock(&g_reg_lock);
    dev_leave(&g);
    return rc;
}

int md5hip_host_unregister(void *base)
{
    if (!base) return -EINVAL;
    pthread_rwlock_wrlock(&g_reg_lock);
    int rc = -ENOENT;
    for (size_t k = 0; k < g_nreg; k++) {
        if (g_reg[k].lo == (uintptr_t)base) {
            rc = hipHostUnregister(base) == hipSuccess ? 0 : -EIO;
            memmove(&g_reg[k], &g_reg[k + 1], (g_nreg - k - 1) * sizeof *g_reg);
            g_nreg--;
            break;
        }
    }
    pthread_rwlock_unlock(&g_reg_lock);
    return rc;
}

/* ------------------------------------------------------------------------
 * Slots and tickets
 * ------------------------------------------------------------------------ */
enum slot_state { SLOT_FREE = 0, SLOT_OPEN, SLOT_INFLIGHT };
enum slot_mode { MODE_NONE = 0, MODE_STAGED, MODE_ZEROCOPY, MODE_FIXED };

/* One ticket's chunks in one slot: slot chunks [first, first+count) deliver
 * into `user` (host array, or device memory when on_device). */
struct seg {
    uint64_t ticket, first, count;
    unsigned char *user;
    int on_device;
};

struct slot {
    hipStream_t stream;
    hipEvent_t done;
    hipEvent_t kdone;                 /* right after the hash kernel: what a chained launch waits on
                                         (the digest scatter / D2H behind it need not) */
    unsigned char *h_data, *d_data;   /* staging, `cap` bytes */
    uint64_t *h_off, *d_off;          /* descriptors, `maxn` entries */
    uint32_t *h_len, *d_len;
    const uint64_t *dh_off;           /* h_off / h_len as the device sees them (fine-grained) */
    const uint32_t *dh_len;
    int desc_direct;                  /* the planned launch reads dh_off / dh_len in place */
    uint32_t *h_ord, *d_ord;
    unsigned char *h_dig, *d_dig;     /* 16 * maxn */
    int direct;                       /* the kernel wrote the one device segment in place */
    struct md5hip_seg *h_seg, *d_seg; /* zero-copy gather table, `segcap` entries */
    void **b_dst, **b_src;            /* DMA-batch gather arrays (plain host memory) */
    size_t *b_len;
    long *b_reg;                      /* registration each DMA entry lies in */
    struct md5hip_seg *h_dsc, *d_dsc; /* device-digest scatter table, `segcap` entries */
    struct seg *segs;                 /* ticket segments */
    uint32_t nsegs, capsegs;
    int state, mode, writers, full, flush, err;
    uint64_t n, used, nseg, ndma, ndsc;
    uint32_t kind, fastcrc, dsz;
    /* MODE_FIXED (md5hip_batch_host_fixed): one contiguous host range, or
     * (fx_dev, md5_batch_submit_device_fixed) one device range read in place */
    const unsigned char *fx_src;
    int fx_dev;
    uint64_t fx_bytes, fx_stride;
    uint32_t fx_len;
    uint64_t tickets_in;              /* distinct tickets (stats) */
    /* descriptors already on the device / the plan they were ordered by:
     * prepared ahead while another slot's launch runs (slot_prepare) */
    uint64_t copied_n, planned_n, seen_n;
    int plan_var;
    /* key histogram of the reserved chunks (k = (len >> 6) + 1, md5hip.h
     * md5hip_plan_hist): the plan is made from counts and the order built on
     * the device; hovf = a chunk past MD5HIP_HIST_KMAX (host sort instead) */
    uint32_t *hh, hkmax, *h_bkt, *d_bkt;
    void *d_sort;                     /* md5hip_order_device_stable scratch (NULL: order_scatter) */
    uint64_t sort_bytes;
    int hovf;
    /* keys already non-increasing in reservation order (a vector of full
     * blocks with a short last one, a single equal-length batch): then the
     * identity IS the longest-first order, and no order is built or used */
    uint32_t last_key;
    int unsorted, use_order;
    uint64_t opened_us, launched_us;  /* first chunk reserved / went in flight */
    uint64_t gen;                     /* launches of this slot so far (a waiter's check) */
    uint64_t load;                    /* this slot's share of b->load_bytes */
    /* payload bytes, and those in device-resident chunks starting 16-B but not
     * 128-B aligned (md5hip_lines_choice: LINES instead of XDMA) */
    uint64_t payload, unlined;
    /* callers blocked on tickets held here sleep on `cv` (nwait of them):
     * broadcast when the slot retires, signalled once when it goes in flight
     * (one sleeper then watches the launch).  watch: WATCH_NONE / _ACTIVE (one
     * waiter sleeps through or spins on this launch) / _GAVE_UP (the spin
     * ended first: the progress thread retires it, polling fast) */
    pthread_cond_t cv;
    uint32_t nwait;
    int watch;
    /* chained launch: its hash kernel waits on the last launch's event
     * (device-side order), so it starts the moment that one ends instead of
     * after the host has seen it end and enqueued it (~1.3 ms per C3 step,
     * profiles/r04b/c3q_gaps.json); chain_at = when it should start */
    hipEvent_t chain_ev;
    uint64_t chain_at;
    /* chain mode 2, both launches BALANCED: no device-side wait -- this
     * launch's workgroups take CUs as the running one's finish (a BALANCED
     * workgroup holds 96 KiB of LDS, so two never share a CU) */
    int chain_overlap;
    /* a synchronous caller's chunks are here: the slot goes while a slot is
     * left over to coalesce the callers behind it (slot_try_launch) */
    int urgent;
    /* md5hip_batcher_inject_fault: this launch completes as a device fault */
    int inject;
};
enum { WATCH_NONE = 0, WATCH_ACTIVE, WATCH_GAVE_UP };
enum watch_policy { WATCH_POLICY_SPIN = 0, WATCH_POLICY_TAIL = 1, WATCH_POLICY_BLOCK = 2 };

struct md5hip_batcher {
    int device;
    int kind;          /* MD5HIP_DIGEST_MD5 or MD5HIP_DIGEST_CRC32 */
    uint32_t fastcrc;  /* CRC-32 head^tail window (blk_io.c:408-424), 0 = whole block */
    uint32_t dsz;      /* digest bytes per chunk: 16 or 4 */
    uint32_t nslots;
    uint64_t cap;      /* staging bytes per slot */
    uint64_t maxn;     /* chunks per slot */
    uint64_t segcap;   /* gather segments per slot (zero-copy modes) */
    int gather;        /* enum md5hip_gather_mode */
    uint32_t target;   /* launch the open slot at once while fewer slots are in flight */
    uint32_t linger_max_us;  /* idle pipeline: hold a slot up to this long for more work */
    double launch_ema_us;    /* recent launches' wall time (submit to retire) */
    struct slot *s;
    int open;          /* index of the OPEN slot new chunks go to, -1 = none */
    uint32_t inflight;
    struct tk_ring tk; /* tickets: live ids, their references and errors (md5_tickets.h) */
    uint64_t load_bytes;      /* weight (len + 64 per chunk) reserved and not yet retired:
                                 read without the lock by md5hip_batcher_load (the pool's router) */
    struct md5hip_batcher_stats st;
    pthread_mutex_t mu;
    pthread_cond_t done_cv;   /* a slot retired / a ticket completed */
    pthread_cond_t work_cv;   /* a slot went in flight / stop */
    pthread_t progress;
    int progress_started, stop;
    int poll_fast;            /* the progress thread polls launches every 10 us now */
    uint32_t slot_waiters;    /* submitters waiting for a slot to retire (slot_wait) */
    int chain;                /* chain the open slot behind the running launch: 0 off, 1 on, 2 (default) on + BALANCED tails overlap */
    hipEvent_t after_ev;     /* recorded on a producer's stream (md5_batch_submit_device_on) */
    int failed;               /* 0, or -ENODEV once the device failed (sticky; read lock-free by the pool) */
    int watch_policy;         /* enum watch_policy (watch_launch), MD5HIP_WATCH at create */
    uint64_t inject_at;       /* md5hip_batcher_inject_fault: launch number that faults, 0 = none */
};

#define CK(x) do { if ((x) != hipSuccess) { rc = -ENODEV; goto fail; } } while (0)

/* the earliest a slot is chained behind the running launch: this long
 * before that launch's expected end (at most; a quarter of a launch for
 * short ones), so late submissions still coalesce into it */
#define CHAIN_LEAD_MAX_US 2000.0

static uint64_t now_us(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return (uint64_t)ts.tv_sec * 1000000u + (uint64_t)ts.tv_nsec / 1000u;
}

/* How long an idle pipeline holds an open slot for more work: 1/8 of the
 * recent launches' wall time, at most linger_max_us.  A burst of vectors
 * submitted back to back then goes out as one launch instead of its first
 * vector alone (a mixed vector alone is bound by its longest chains, DESIGN.md
 * §5.4), and the added latency stays a fraction of the work itself. */
static uint64_t linger_us(const md5hip_batcher *b)
{
    const double l = b->launch_ema_us / 8.0;
    return l < (double)b->linger_max_us ? (uint64_t)l : (uint64_t)b->linger_max_us;
}

/* pthread_cond_timedwait on cv until `us` microseconds from now (mu held) */
static void wait_cv_us(md5hip_batcher *b, pthread_cond_t *cv, uint64_t us)
{
    struct timespec ts;
    clock_gettime(CLOCK_REALTIME, &ts);
    ts.tv_sec += (time_t)(us / 1000000u);
    ts.tv_nsec += (long)(us % 1000000u) * 1000;
    if (ts.tv_nsec >= 1000000000L) { ts.tv_sec++; ts.tv_nsec -= 1000000000L; }
    pthread_cond_timedwait(cv, &b->mu, &ts);
}
static void wait_work_us(md5hip_batcher *b, uint64_t us) { wait_cv_us(b, &b->work_cv, us); }

/* ticket table (md5_tickets.h), all under b->mu */
static int tk_new(md5hip_batcher *b, uint64_t *t) { return tk_ring_new(&b->tk, t); }
static int tk_done(const md5hip_batcher *b, uint64_t t, int *err) { return tk_ring_done(&b->tk, t, err); }
static void tk_put(md5hip_batcher *b, uint64_t t, int err) { tk_ring_put(&b->tk, t, err); }

/* One segment per (ticket, slot): a submission fills a slot until it is full
 * before it moves on, so its chunks in one slot are one contiguous run. */
static int seg_push(struct slot *sl, struct seg sg)
{
    if (sl->nsegs == sl->capsegs) {
        const uint32_t nc = sl->capsegs ? 2 * sl->capsegs : 64;
        struct seg *p = realloc(sl->segs, nc * sizeof *p);
        if (!p) return -ENOMEM;
        sl->segs = p;
        sl->capsegs = nc;
    }
    sl->segs[sl->nsegs++] = sg;
    sl->tickets_in++;
    return 0;
}

static int seg_has(const struct slot *sl, uint64_t t)
{
    for (uint32_t k = 0; k < sl->nsegs; k++)
        if (sl->segs[k].ticket == t) return 1;
    return 0;
}

/* Descriptors in and the plan (mu held): the new descriptor entries
 * [copied_n, n) go to the device, the whole slot is ordered longest-first
 * (md5hip_plan_desc) and the order follows, all on the slot's own stream.
 * Descriptors are final once reserved (append-only), so this may run while
 * the slot is still OPEN -- the progress thread does it while another slot's
 * launch keeps the device busy, and the launch then only enqueues the kernel.
 * Chunks appended after it are copied and the slot re-planned at launch (an
 * order copy still in flight is overwritten by the later one, same stream). */
/* Small slots (a netcache vector) skip the two descriptor copies: the kernel
 * reads the fine-grained pinned arrays in place, one PCIe round trip per wave
 * instead of two copy operations ahead of the launch on the slot's stream. */
enum { DESC_DIRECT_MAX = 4096, EARLY_COPY_MIN = 8192 };

/* The stable device order of a large slot: 0 done; 1 = refused before any
 * device work (scratch sized at creation too small for this slot's n /
 * kmax, an argument the sort does not take): fall back to order_scatter,
 * never a failed ticket for it; < 0 = the sort's launch failed (-EIO): the
 * slot fails, and no hash kernel runs on an order never written. */
static int stable_order(struct slot *sl, uint64_t n)
{
    const int e = md5hip_order_device_stable(sl->d_len, n, sl->hkmax, sl->d_sort, sl->sort_bytes,
                                             sl->d_ord, sl->stream);
    return e == -ENOSPC || e == -EINVAL ? 1 : e;
}

static int slot_prepare(md5hip_batcher *b, struct slot *sl)
{
    (void)b;
    const uint64_t n = sl->n;
    if (sl->planned_n == n) return 0;
    sl->desc_direct = n <= DESC_DIRECT_MAX;
    if (!sl->desc_direct && n > sl->copied_n) {
        const uint64_t c0 = sl->copied_n;
        if (hipMemcpyAsync(sl->d_off + c0, sl->h_off + c0, 8 * (n - c0), hipMemcpyHostToDevice, sl->stream) ||
            hipMemcpyAsync(sl->d_len + c0, sl->h_len + c0, 4 * (n - c0), hipMemcpyHostToDevice, sl->stream))
            return -EIO;
        sl->copied_n = n;
    }
    int dvar, e = 0;
    if (!sl->unsorted) {
        dvar = sl->hovf ? md5hip_plan_desc(sl->h_len, n, sl->h_ord)
                        : md5hip_plan_hist(sl->hh, sl->hkmax, n, NULL);
        if (dvar < 0) return dvar;
        sl->use_order = 0;
    } else if (!sl->hovf && !sl->desc_direct && sl->d_sort &&
               (dvar = md5hip_plan_hist(sl->hh, sl->hkmax, n, NULL)) >= 0 &&
               (e = stable_order(sl, n)) <= 0) {
        /* from the histogram: O(keys) on the host; the STABLE order on the
         * device (equal keys in chunk order: a 6-batch C3 BALANCED launch
         * ran 5-6 % longer in order_scatter's wave-arrival order,
         * profiles/r06e/order_ab.json) */
        if (e) return e;
    } else if (!sl->hovf) {
        /* small slots (lengths read in place from mapped host memory), and
         * large ones whose stable sort was refused: one scatter launch */
        dvar = md5hip_plan_hist(sl->hh, sl->hkmax, n, sl->h_bkt);
        if (dvar < 0) return dvar;
        if (hipMemcpyAsync(sl->d_bkt, sl->h_bkt, 4 * ((size_t)sl->hkmax + 1), hipMemcpyHostToDevice,
                           sl->stream))
            return -EIO;
        e = md5hip_order_device(sl->desc_direct ? sl->dh_len : sl->d_len, n, sl->hkmax, sl->d_bkt,
                                sl->d_ord, sl->stream);
        if (e) return e;
    } else {
        dvar = md5hip_plan_desc(sl->h_len, n, sl->h_ord);
        if (dvar < 0) return dvar;
        if (hipMemcpyAsync(sl->d_ord, sl->h_ord, 4 * n, hipMemcpyHostToDevice, sl->stream)) return -EIO;
    }
    if (sl->unsorted) sl->use_order = 1;
    /* host-staged chunks sit on 128-B lines; device-resident ones as placed */
    sl->plan_var = md5hip_lines_choice(dvar, sl->unlined, sl->payload);
    sl->planned_n = n;
    return 0;
}

/* Enqueue slot `sl` (mu held, writers == 0): bytes in, kernel, digests out. */
static int slot_enqueue(md5hip_batcher *b, struct slot *sl)
{
    int rc = 0;
    const uint64_t n = sl->n;
    /* one submission whose digests stay on the device and fill the slot in
     * order: the kernel writes them in place (no scatter launch) */
    const struct seg *g0 = sl->nsegs == 1 ? &sl->segs[0] : NULL;
    unsigned char *dst = sl->d_dig;
    if (g0 && g0->on_device && g0->first == 0 && g0->count == n && ((uintptr_t)g0->user & 15u) == 0) {
        dst = g0->user;
        sl->direct = 1;
    }
    if (sl->mode == MODE_FIXED) {
        /* host_fixed: the bytes are on their way already (its copy was
         * enqueued on this stream outside b->mu); device_fixed: they are
         * read where the caller keeps them */
        const void *src = sl->fx_dev ? (const void *)sl->fx_src : (const void *)sl->d_data;
        if (sl->chain_ev && hipStreamWaitEvent(sl->stream, sl->chain_ev, 0) != hipSuccess) return -EIO;
        rc = sl->kind == MD5HIP_DIGEST_CRC32
                 ? crc32hip_fixed(src, n, sl->fx_len, sl->fx_stride, sl->fastcrc, (uint32_t *)dst, sl->stream)
                 : md5hip_digest_fixed(src, n, sl->fx_len, sl->fx_stride, dst, sl->stream);
        if (rc) return rc;
        if (hipEventRecord(sl->kdone, sl->stream)) return -EIO;
    } else {
        if ((rc = slot_prepare(b, sl))) return rc;
        const int dvar = sl->plan_var;
        if (sl->mode == MODE_STAGED && sl->used) {
            if (hipMemcpyAsync(sl->d_data, sl->h_data, sl->used, hipMemcpyHostToDevice, sl->stream))
                return -EIO;
        } else if (sl->mode == MODE_ZEROCOPY && sl->nseg) {
            int mode = b->gather;
            if (mode == MD5HIP_GATHER_AUTO)
                /* measured: per-copy DMA beats the PCIe-reading
                 * gather kernel once copies average more than ~192 KiB */
                mode = sl->ndma * (256u << 10) <= sl->used ? MD5HIP_GATHER_DMA : MD5HIP_GATHER_DEVICE;
            if (mode == MD5HIP_GATHER_DEVICE) {
                if (hipMemcpyAsync(sl->d_seg, sl->h_seg, sizeof(struct md5hip_seg) * sl->nseg,
                                   hipMemcpyHostToDevice, sl->stream))
                    return -EIO;
                if ((rc = md5hip_gather_launch(sl->d_seg, sl->nseg, sl->d_data, sl->stream))) return rc;
            } else {
                /* one async copy per run (hipMemcpyBatchAsync is newer than the
                 * HIP runtime torch ships, which this library shares) */
                for (uint64_t q = 0; q < sl->ndma; q++)
                    if (hipMemcpyAsync(sl->b_dst[q], sl->b_src[q], sl->b_len[q], hipMemcpyHostToDevice,
                                       sl->stream) != hipSuccess)
                        return -EIO;
            }
        }
        /* a chained launch: bytes in and plan made beside the running
         * launch, the hash kernel after it */
        if (sl->chain_ev && !sl->chain_overlap && hipStreamWaitEvent(sl->stream, sl->chain_ev, 0) != hipSuccess)
            return -EIO;
        const uint32_t *ord = sl->use_order ? sl->d_ord : NULL;
        const uint64_t *doff = sl->desc_direct ? sl->dh_off : sl->d_off;
        const uint32_t *dlen = sl->desc_direct ? sl->dh_len : sl->d_len;
        rc = sl->kind == MD5HIP_DIGEST_CRC32
                 ? crc32hip_desc_variant(sl->d_data, doff, dlen, ord, n, sl->fastcrc,
                                         (uint32_t *)dst, sl->stream,
                                         md5hip_crc_desc_choice(sl->fastcrc ? 2 * n : n,
                                                                sl->fastcrc ? sl->fastcrc
                                                                            : sl->load / n - 64))
                 : md5hip_digest_desc_variant(sl->d_data, doff, dlen, ord, n,
                                              dst, sl->stream, dvar);
        if (rc) return rc;
        if (hipEventRecord(sl->kdone, sl->stream)) return -EIO;
    }
    /* digests out: one D2H for the host segments, one scatter for the device
     * ones.  The scatter kernel runs one workgroup per entry, so a long
     * segment is cut into pieces of DSC_PIECE bytes as the table has room
     * (6 tickets of 79 K digests as 6 entries took 145 us) */
    enum { DSC_PIECE = 64 << 10 };
    int any_host = 0;
    sl->ndsc = 0;
    uint64_t ndev = 0;
    for (uint32_t k = 0; k < sl->nsegs && !sl->direct; k++) ndev += sl->segs[k].on_device;
    uint64_t spare = b->segcap - ndev;                   /* nsegs < segcap (slot_open) */
    for (uint32_t k = 0; k < sl->nsegs && !sl->direct; k++) {
        const struct seg *g = &sl->segs[k];
        if (!g->on_device) { any_host = 1; continue; }
        const uint64_t len = (uint64_t)sl->dsz * g->count;
        if (len == 0) continue;
        uint64_t extra = (len + DSC_PIECE - 1) / DSC_PIECE - 1;
        if (extra > spare) extra = spare;
        spare -= extra;
        const uint64_t piece = ((len + extra) / (extra + 1) + 15) & ~15ull;   /* 16-B multiples */
        for (uint64_t at = 0; at < len; at += piece) {
            const uint64_t l = len - at < piece ? len - at : piece;
            sl->h_dsc[sl->ndsc++] = (struct md5hip_seg){
                (uint64_t)(uintptr_t)(sl->d_dig + (size_t)sl->dsz * g->first + at),
                (uint64_t)((uintptr_t)g->user + at - (uintptr_t)sl->d_dig),   /* relative to d_dig (mod 2^64) */
                (uint32_t)l, 0};
        }
    }
    if (sl->ndsc) {
        if (hipMemcpyAsync(sl->d_dsc, sl->h_dsc, sizeof(struct md5hip_seg) * sl->ndsc,
                           hipMemcpyHostToDevice, sl->stream))
            return -EIO;
        if ((rc = md5hip_gather_launch(sl->d_dsc, sl->ndsc, sl->d_dig, sl->stream))) return rc;
    }
    if (any_host &&
        hipMemcpyAsync(sl->h_dig, sl->d_dig, (size_t)sl->dsz * n, hipMemcpyDeviceToHost, sl->stream))
        return -EIO;
    if (hipEventRecord(sl->done, sl->stream)) return -EIO;
    return 0;
}

static void slot_reset(struct slot *sl)
{
    sl->state = SLOT_FREE;
    sl->watch = WATCH_NONE;
    sl->chain_ev = NULL;
    sl->chain_at = 0;
    sl->chain_overlap = 0;
    sl->urgent = 0;
    sl->inject = 0;
    sl->fx_dev = 0;
    sl->mode = MODE_NONE;
    sl->writers = sl->full = sl->flush = sl->err = sl->direct = 0;
    sl->n = sl->used = sl->nseg = sl->ndma = sl->ndsc = 0;
    sl->nsegs = 0;
    sl->tickets_in = 0;
    sl->copied_n = sl->planned_n = sl->seen_n = 0;
    sl->load = 0;
    sl->payload = sl->unlined = 0;
    sl->last_key = UINT32_MAX;
    sl->unsorted = sl->use_order = 0;
    if (sl->hh) memset(sl->hh, 0, sizeof(uint32_t) * ((size_t)sl->hkmax + 1));
    sl->hkmax = 0;
    sl->hovf = 0;
}

/* Deliver a finished (or failed) slot to its tickets and free it (mu held). */
static void slot_retire(md5hip_batcher *b, struct slot *sl, int err)
{
    for (uint32_t k = 0; k < sl->nsegs; k++) {
        const struct seg *g = &sl->segs[k];
        if (!err && !g->on_device)
            memcpy(g->user, sl->h_dig + (size_t)sl->dsz * g->first, (size_t)sl->dsz * g->count);
        tk_put(b, g->ticket, err);
    }
    __atomic_store_n(&b->load_bytes, b->load_bytes - sl->load, __ATOMIC_RELAXED);
    sl->load = 0;
    if (sl->state == SLOT_INFLIGHT) {
        b->inflight--;
        /* a chained launch's start is estimated (chain_at): one that retires
         * before it (a BALANCED overlap started early) gives no sample */
        const uint64_t t = now_us();
        if (t > sl->launched_us) {
            const double d = (double)(t - sl->launched_us);
            b->launch_ema_us = b->launch_ema_us > 0 ? 0.75 * b->launch_ema_us + 0.25 * d : d;
        }
    }
    slot_reset(sl);
    if (sl->nwait) pthread_cond_broadcast(&sl->cv);   /* its waiters only */
    pthread_cond_broadcast(&b->done_cv);              /* slot_take / drain / destroy */
}

/* Is the device behind this HIP status gone (a fault, a lost or reset
 * device) rather than the call merely refused?  Completion events report
 * only these; an enqueue error is classified by the stream's state after it. */
static int hip_lost(hipError_t e)
{
    switch (e) {
    case hipSuccess: case hipErrorNotReady:
    case hipErrorInvalidValue: case hipErrorOutOfMemory: case hipErrorInvalidDevicePointer:
    case hipErrorInvalidMemcpyDirection: case hipErrorInvalidConfiguration:
    case hipErrorInvalidResourceHandle: case hipErrorNotSupported:
        return 0;
    default:
        return 1;
    }
}

/* The device failed (mu held): sticky.  Tickets coalescing in the open slot
 * are retired with -ENODEV (or when their writers are done: sl->err); slots
 * in flight finish as their events say; callers blocked on a slot are woken
 * by its retire, everything waiting for a free slot by done_cv. */
static void batcher_fail(md5hip_batcher *b)
{
    if (b->failed) return;
    __atomic_store_n(&b->failed, -ENODEV, __ATOMIC_RELEASE);
    b->inject_at = 0;
    for (uint32_t k = 0; k < b->nslots; k++) {
        struct slot *sl = &b->s[k];
        if (sl->state != SLOT_OPEN) continue;
        if (b->open == (int)k) b->open = -1;
        sl->full = 1;
        if (!sl->err) sl->err = -ENODEV;
        if (!sl->writers) slot_retire(b, sl, sl->err);
    }
    pthread_cond_broadcast(&b->done_cv);
    pthread_cond_broadcast(&b->work_cv);
}

/* A launch's completion (mu not needed): its event, or the injected fault
 * once the launch has really finished. */
static hipError_t launch_status(hipEvent_t ev, int inject)
{
    const hipError_t e = hipEventQuery(ev);
    return e == hipSuccess && inject ? hipErrorLaunchFailure : e;
}

/* Retire in-flight slot `sl` whose completion status is `e` (mu held). */
static void slot_complete(md5hip_batcher *b, struct slot *sl, hipError_t e)
{
    slot_retire(b, sl, e == hipSuccess ? 0 : -EIO);
    if (e != hipSuccess) batcher_fail(b);
}

/* Launch slot `sl` if it may go now (mu held). */
static void slot_try_launch(md5hip_batcher *b, struct slot *sl)
{
    if (sl->state != SLOT_OPEN || sl->writers) return;
    /* callers blocked on its tickets: no linger once the device is idle (as
     * md5_batch_wait's hasten, re-applied whenever the slot is looked at,
     * since they sleep until it goes) */
    if (sl->nwait && b->inflight == 0) sl->flush = 1;
    /* synchronous callers: up to nslots - 1 launches run at once (a netcache
     * vector is a wave or two: concurrent small launches cost the device
     * nothing), the last slot coalesces whoever comes while they run */
    if (sl->urgent && b->inflight + 1 < b->nslots) sl->flush = 1;
    if (sl->n == 0) {                 /* nothing reserved (all chunks failed) */
        if (b->open == (int)(sl - b->s)) b->open = -1;
        slot_retire(b, sl, sl->err);
        return;
    }
    if (!(sl->full || sl->flush || sl->chain_ev || b->inflight < b->target)) return;
    if (!sl->full && !sl->flush && b->inflight == 0 && now_us() - sl->opened_us < linger_us(b)) {
        pthread_cond_broadcast(&b->work_cv);        /* the progress thread times the linger */
        return;
    }
    if (b->open == (int)(sl - b->s)) b->open = -1;
    const int rc = sl->err ? sl->err : b->failed ? b->failed : slot_enqueue(b, sl);
    if (rc) {
        /* an enqueue (here, or a descriptor copy or ordering made earlier:
         * sl->err) that failed because the device did: the stream says so */
        const int lost = !b->failed && rc != -ENODEV && hip_lost(hipStreamQuery(sl->stream));
        slot_retire(b, sl, rc);
        if (lost) batcher_fail(b);
        return;
    }
    if (b->inject_at && b->st.launches + 1 == b->inject_at) {
        sl->inject = 1;
        b->inject_at = 0;
    }
    sl->state = SLOT_INFLIGHT;
    sl->launched_us = now_us();
    if (sl->chain_ev && sl->chain_at > sl->launched_us) sl->launched_us = sl->chain_at;   /* its real start */
    sl->gen++;
    b->inflight++;
    b->st.launches++;
    b->st.chunks += sl->n;
    b->st.bytes_staged += sl->used;
    if (sl->n > b->st.max_chunks_per_launch) b->st.max_chunks_per_launch = sl->n;
    if (sl->tickets_in > 1) b->st.coalesced_launches++;
    if (sl->tickets_in > b->st.max_tickets_per_launch) b->st.max_tickets_per_launch = sl->tickets_in;
    if (sl->nwait) pthread_cond_signal(&sl->cv);      /* one sleeper becomes its watcher */
    pthread_cond_broadcast(&b->work_cv);
}

/* A submitter waits for a slot to retire (mu held).  The progress thread
 * polls the launches every 10 us meanwhile instead of its idle 20-200 us:
 * nobody else may be waiting on a ticket (an asynchronous stream whose
 * every slot is in flight), and the retire it waits for gates its whole
 * submission -- a stream of 1 M-block fastcrc launches (~55 us each) lost
 * half its time to that poll before. */
static void slot_wait(md5hip_batcher *b)
{
    b->slot_waiters++;
    if (!b->poll_fast) pthread_cond_broadcast(&b->work_cv);
    pthread_cond_wait(&b->done_cv, &b->mu);
    b->slot_waiters--;
}

/* A FREE slot made OPEN in `mode` for digests of `kind` (mu held; waits
 * for one to retire). */
static struct slot *slot_take(md5hip_batcher *b, int mode, int kind, uint32_t fastcrc)
{
    for (;;) {
        for (uint32_t k = 0; k < b->nslots; k++) {
            struct slot *sl = &b->s[k];
            if (sl->state != SLOT_FREE) continue;
            slot_reset(sl);
            sl->state = SLOT_OPEN;
            sl->mode = mode;
            sl->kind = (uint32_t)kind;
            sl->fastcrc = fastcrc;
            sl->dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
            return sl;
        }
        /* all busy: make sure the open slot can go, then wait for a retire */
        if (b->open >= 0) {
            struct slot *o = &b->s[b->open];
            o->full = 1;
            slot_try_launch(b, o);
        }
        slot_wait(b);
    }
}

/* The OPEN slot that accepts chunks of `mode` and digest `kind` (mu held). */
/* The open slot is re-examined after every wait for a free one: another
 * submitter may have opened one meanwhile, and taking a second slot then
 * would leave the first OPEN but no longer b->open -- launched by nobody
 * (its asynchronous tickets stranded until a wait on them). */
static struct slot *slot_open(md5hip_batcher *b, int mode, int kind, uint32_t fastcrc)
{
    for (;;) {
        if (b->open >= 0) {
            struct slot *o = &b->s[b->open];
            const int compatible = (o->mode == mode || mode == MODE_NONE || o->mode == MODE_NONE) &&
                                   o->kind == (uint32_t)kind && o->fastcrc == fastcrc;
            if (!o->full && compatible && o->nsegs < b->segcap) {
                if (o->mode == MODE_NONE) o->mode = mode;
                return o;
            }
            o->full = 1;                 /* closes: launched once its writers are done */
            b->open = -1;
            slot_try_launch(b, o);
        }
        for (uint32_t k = 0; k < b->nslots; k++) {
            struct slot *sl = &b->s[k];
            if (sl->state != SLOT_FREE) continue;
            slot_reset(sl);
            sl->state = SLOT_OPEN;
            sl->mode = mode;
            sl->kind = (uint32_t)kind;
            sl->fastcrc = fastcrc;
            sl->dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
            b->open = (int)k;
            return sl;
        }
        slot_wait(b);                                 /* all busy: wait for a retire */
    }
}

/* ------------------------------------------------------------------------
 * Progress thread: retire finished slots, launch coalesced work.
 * ------------------------------------------------------------------------ */
static void *progress_main(void *arg)
{
    md5hip_batcher *b = arg;
    (void)hipSetDevice(b->device);
    /* this thread's timed waits are the event polls (10 us while a caller
     * waits): the default 50 us timer slack would stretch each to ~60 us and
     * deliver a finished launch that much late */
    (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
    pthread_mutex_lock(&b->mu);
    unsigned idle_us = 20;
    while (!b->stop) {
        int any = 0;
        b->poll_fast = 0;
        for (uint32_t k = 0; k < b->nslots; k++) {
            struct slot *sl = &b->s[k];
            if (sl->state != SLOT_INFLIGHT) continue;
            const hipError_t e = launch_status(sl->done, sl->inject);
            if (e == hipErrorNotReady) continue;
            slot_complete(b, sl, e);
            any = 1;
        }
        if (any) {
            if (b->open >= 0) slot_try_launch(b, &b->s[b->open]);
            idle_us = 20;
            continue;
        }
        if (b->inflight == 0) {
            struct slot *o = b->open >= 0 ? &b->s[b->open] : NULL;
            if (o && o->state == SLOT_OPEN && o->n > 0 && !o->writers) {
                const uint64_t waited = now_us() - o->opened_us, l = linger_us(b);
                if (waited >= l) slot_try_launch(b, o);    /* lingered long enough */
                else wait_work_us(b, l - waited);
            } else {
                pthread_cond_wait(&b->work_cv, &b->mu);
            }
            idle_us = 20;
        } else {
            /* the device is busy: get the open slot's descriptors over and its
             * plan made now, once no chunk arrived since the last poll, so
             * its launch is only the kernel when the running one retires */
            if (b->open >= 0) {
                struct slot *o = &b->s[b->open];
                if (o->state == SLOT_OPEN && o->mode != MODE_FIXED && o->n > o->planned_n) {
                    if (o->n == o->seen_n) {
                        const int e = slot_prepare(b, o);
                        if (e && !o->err) o->err = e;
                    }
                    o->seen_n = o->n;
                }
                /* planned and quiet, the pipeline at its target, and the last
                 * launch due to end within min(2 ms, a quarter of a launch):
                 * chain it there (its kernel waits on that launch's event).
                 * Not behind a launch overdue by more than that: its end is
                 * unknown, and the open slot keeps coalescing until it retires */
                if (b->chain && o->state == SLOT_OPEN && o->n && !o->writers && !o->err && !o->chain_ev &&
                    o->mode != MODE_FIXED && o->planned_n == o->n && b->inflight == b->target &&
                    b->launch_ema_us > 0) {
                    struct slot *last = NULL;
                    for (uint32_t k = 0; k < b->nslots; k++)
                        if (b->s[k].state == SLOT_INFLIGHT && (!last || b->s[k].launched_us > last->launched_us))
                            last = &b->s[k];
                    const double lead = b->launch_ema_us / 4 < CHAIN_LEAD_MAX_US ? b->launch_ema_us / 4
                                                                                 : CHAIN_LEAD_MAX_US;
                    const uint64_t end = last ? last->launched_us + (uint64_t)b->launch_ema_us : 0;
                    const uint64_t now = now_us();
                    if (last && (double)now + lead >= (double)end && (double)now <= (double)end + lead) {
                        o->chain_ev = last->kdone;
                        o->chain_at = end > now ? end : now;
                        o->chain_overlap = b->chain == 2 && last->mode != MODE_FIXED &&
                                           last->kind == MD5HIP_DIGEST_MD5 && o->kind == MD5HIP_DIGEST_MD5 &&
                                           last->plan_var == MD5HIP_DESC_BALANCED &&
                                           o->plan_var == MD5HIP_DESC_BALANCED;
                        slot_try_launch(b, o);
                    }
                }
            }
            /* poll interval: 20 -> 200 us while nobody waits; blocked callers
             * pin it at 10 us (a short launch is not delivered up to 200 us
             * late) unless each of their launches has a watcher of its own:
             * callers on an open slot (it goes when a launch retires), or on
             * a launch with no watcher yet or whose watcher's spin ran out */
            int fast = b->slot_waiters > 0;
            for (uint32_t k = 0; k < b->nslots; k++)
                fast |= b->s[k].nwait && !(b->s[k].state == SLOT_INFLIGHT && b->s[k].watch == WATCH_ACTIVE);
            b->poll_fast = fast;
            const unsigned us = fast ? 10u : idle_us;
            struct timespec ts;
            clock_gettime(CLOCK_REALTIME, &ts);
            ts.tv_nsec += (long)us * 1000;
            if (ts.tv_nsec >= 1000000000L) { ts.tv_sec++; ts.tv_nsec -= 1000000000L; }
            pthread_cond_timedwait(&b->work_cv, &b->mu, &ts);
            if (idle_us < 200) idle_us += 20;
        }
    }
    pthread_mutex_unlock(&b->mu);
    return NULL;
}

/* ------------------------------------------------------------------------
 * Blocked callers.  A caller blocked on ticket t sleeps on the condition
 * variable of a slot holding t, so a retire wakes only that slot's callers
 * (the netcache ASIO pool runs 4-512 threads into this site at once,
 * asio_mgr.c:86-91, :205, :1050-1057, and a coalesced launch holds many of
 * their vectors).  Waiting for the progress thread alone, a synchronous call
 * returns up to one poll (10 us) plus a wake-up after its kernel ends -- for
 * a netcache vector (a ~140 us kernel) 20-30 us of each call -- so ONE caller
 * per launch watches it: a launch expected to end soon (recent launches' wall
 * time) has its event polled by that caller, who retires the slot the moment
 * it completes; a longer one is slept through first.  Every other caller on
 * the launch sleeps until the retire.  The spin is bounded; past it the
 * watcher sleeps too and the progress thread (polling fast meanwhile)
 * retires the launch.  Every sleep re-checks its condition under b->mu, and
 * every state change that ends one (retire, launch) is made under b->mu and
 * broadcast or signalled, so no wake-up is lost.
 * ------------------------------------------------------------------------ */
enum { WATCH_SPIN_US = 300, WATCH_LEAD_US = 200 };   /* WATCH_POLICY_SPIN */
enum { WATCH_TAIL_US = 50, WATCH_TAIL_SPIN_US = 150 };  /* WATCH_POLICY_TAIL */

static void cpu_relax(void)
{
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}

/* The watcher's sleep on the slot's condition variable until `us` from now
 * ends within a few us of its deadline, not the default 50 us timer slack
 * later (the caller's own slack is put back after). */
static void watch_sleep(md5hip_batcher *b, struct slot *sl, uint64_t us)
{
    const int old = prctl(PR_GET_TIMERSLACK, 0, 0, 0, 0);
    if (old > 2000) (void)prctl(PR_SET_TIMERSLACK, 2000UL, 0, 0, 0);
    sl->nwait++;
    wait_cv_us(b, &sl->cv, us);
    sl->nwait--;
    if (old > 2000) (void)prctl(PR_SET_TIMERSLACK, (unsigned long)old, 0, 0, 0);
}

/* Watch in-flight slot `sl` (mu held on entry and exit, watch == NONE).
 * The policy (b->watch_policy, MD5HIP_WATCH at create; profiles/r05e/):
 *   TAIL   (default) sleep on the slot until 50 us before the launch is due
 *          (recent launches' wall time), then poll its event for at most
 *          150 us; past that the watcher gives up and sleeps too, and the
 *          progress thread (polling every 10 us meanwhile) retires it.  At
 *          8 callers a call costs its thread 33-39 us of CPU instead of
 *          SPIN's 122 (the whole ~150 us launch polled), same latency;
 *   SPIN   round 4: a launch due within 300 us is polled for up to 500 us
 *          (a longer one slept through until 200 us before its end);
 *   BLOCK  hipEventSynchronize on a blocking-sync event: measured, not
 *          kept -- the wake-up after the interrupt costs ~1 ms per call
 *          and ~190 us of CPU (r05e/asio_watch.json). */
static void watch_launch(md5hip_batcher *b, struct slot *sl)
{
    const uint64_t gen = sl->gen;
    const int pol = b->watch_policy;
    const uint64_t spin = pol == WATCH_POLICY_SPIN ? WATCH_SPIN_US : WATCH_TAIL_US;
    const uint64_t lead = pol == WATCH_POLICY_SPIN ? WATCH_LEAD_US : WATCH_TAIL_US;
    sl->watch = WATCH_ACTIVE;
    for (; pol != WATCH_POLICY_BLOCK;) {        /* long launch: sleep most of it */
        const uint64_t now = now_us(), end = sl->launched_us + (uint64_t)b->launch_ema_us;
        if (end <= now + spin) break;
        watch_sleep(b, sl, end - now - lead);
        if (sl->state != SLOT_INFLIGHT || sl->gen != gen) return;     /* retired meanwhile */
    }
    const hipEvent_t ev = sl->done;
    const int inject = sl->inject;
    pthread_mutex_unlock(&b->mu);
    hipError_t e = hipErrorNotReady;
    if (pol != WATCH_POLICY_BLOCK) {
        const uint64_t t0 = now_us(), limit = pol == WATCH_POLICY_SPIN ? WATCH_SPIN_US + WATCH_LEAD_US
                                                                       : WATCH_TAIL_SPIN_US;
        while ((e = launch_status(ev, inject)) == hipErrorNotReady && now_us() - t0 < limit) cpu_relax();
    } else {
        e = hipEventSynchronize(ev);
        if (e == hipSuccess && inject) e = hipErrorLaunchFailure;
    }
    pthread_mutex_lock(&b->mu);
    /* the same launch still in flight? (the progress thread may have retired
     * it, and the slot may even be in flight again with other work: then
     * `watch` belongs to that launch and is left alone) */
    if (sl->state != SLOT_INFLIGHT || sl->gen != gen) return;
    if (e == hipErrorNotReady) {
        sl->watch = WATCH_GAVE_UP;              /* nobody spins on it again */
        return;
    }
    slot_complete(b, sl, e);
    if (b->open >= 0) slot_try_launch(b, &b->s[b->open]);
    pthread_cond_broadcast(&b->work_cv);
}

/* Block until ticket t is complete (mu held on entry and exit); its error.
 * An open slot holding t is hastened: launched at once while nothing is in
 * flight (no linger), else by the usual policy (md5_batch_wait's rule; a
 * synchronous submission's too, so that callers arriving while the device is
 * busy coalesce into one launch instead of one launch each). */
static int wait_ticket(md5hip_batcher *b, uint64_t t)
{
    int err = 0;
    while (!tk_done(b, t, &err)) {
        struct slot *in = NULL, *open = NULL;
        for (uint32_t k = 0; k < b->nslots; k++) {
            struct slot *sl = &b->s[k];
            if (sl->state == SLOT_FREE || !seg_has(sl, t)) continue;
            if (sl->state == SLOT_OPEN) {
                if (b->inflight == 0) sl->flush = 1;
                slot_try_launch(b, sl);
            }
            if (sl->state == SLOT_INFLIGHT && !in) in = sl;
            else if (sl->state == SLOT_OPEN && !open) open = sl;
        }
        if (tk_done(b, t, &err)) break;
        if (in && in->watch == WATCH_NONE) {
            watch_launch(b, in);
            continue;
        }
        struct slot *sl = in ? in : open;
        if (!sl) {                  /* not held by any slot yet (cannot happen for a
                                       returned ticket): re-check shortly */
            wait_cv_us(b, &b->done_cv, 1000);
            continue;
        }
        sl->nwait++;
        if (!b->poll_fast) pthread_cond_broadcast(&b->work_cv);   /* it may need to now */
        pthread_cond_wait(&sl->cv, &b->mu);
        sl->nwait--;
    }
    return err;
}

/* ------------------------------------------------------------------------
 * Create / destroy / settings
 * ------------------------------------------------------------------------ */
static void batcher_free(md5hip_batcher *b)
{
    for (uint32_t k = 0; b->s && k < b->nslots; k++) {
        struct slot *sl = &b->s[k];
        if (sl->state == SLOT_INFLIGHT) hipEventSynchronize(sl->done);
        if (sl->stream) hipStreamDestroy(sl->stream);
        if (sl->done) hipEventDestroy(sl->done);
        if (sl->kdone) hipEventDestroy(sl->kdone);
        hipHostFree(sl->h_data); hipHostFree(sl->h_off); hipHostFree(sl->h_len);
        hipHostFree(sl->h_ord); hipHostFree(sl->h_dig);
        hipFree(sl->d_data); hipFree(sl->d_off); hipFree(sl->d_len);
        hipFree(sl->d_ord); hipFree(sl->d_dig);
        hipHostFree(sl->h_seg); hipFree(sl->d_seg);
        hipHostFree(sl->h_dsc); hipFree(sl->d_dsc);
        free(sl->b_dst); free(sl->b_src); free(sl->b_len); free(sl->b_reg);
        free(sl->segs);
        free(sl->hh);
        hipHostFree(sl->h_bkt); hipFree(sl->d_bkt);
        if (sl->d_sort) hipFree(sl->d_sort);
        pthread_cond_destroy(&sl->cv);
    }
    free(b->s);
    if (b->after_ev) hipEventDestroy(b->after_ev);
    tk_ring_free(&b->tk);
    pthread_mutex_destroy(&b->mu);
    pthread_cond_destroy(&b->done_cv);
    pthread_cond_destroy(&b->work_cv);
    free(b);
}

void md5hip_batcher_destroy(md5hip_batcher *b)
{
    if (!b) return;
    struct dev_guard g;
    if (dev_enter(&g, b->device)) g.ok = 0;
    if (b->progress_started) {
        pthread_mutex_lock(&b->mu);
        /* launch what is still open so every ticket completes, then drain */
        if (b->open >= 0) {
            struct slot *o = &b->s[b->open];
            o->flush = 1;
            slot_try_launch(b, o);
        }
        while (b->inflight) pthread_cond_wait(&b->done_cv, &b->mu);
        b->stop = 1;
        pthread_cond_broadcast(&b->work_cv);
        pthread_mutex_unlock(&b->mu);
        pthread_join(b->progress, NULL);
    }
    batcher_free(b);
    dev_leave(&g);
}

static int batcher_new(int device, uint64_t slice_bytes, uint32_t nslots, uint64_t maxn,
                       md5hip_batcher **out)
{
    int rc = 0;
    if (!out) return -EINVAL;
    *out = NULL;
    if (nslots == 0) nslots = 4;
    if (nslots > 16) return -EINVAL;
    slice_bytes = (slice_bytes + 4095) & ~4095ull;
    if (slice_bytes == 0) slice_bytes = 4096;
    struct dev_guard g;
    if (dev_enter(&g, device)) return -ENODEV;
    md5hip_batcher *b = calloc(1, sizeof *b);
    if (!b) { dev_leave(&g); return -ENOMEM; }
    pthread_mutex_init(&b->mu, NULL);
    pthread_cond_init(&b->done_cv, NULL);
    pthread_cond_init(&b->work_cv, NULL);
    b->device = device;
    b->kind = MD5HIP_DIGEST_MD5;
    b->dsz = 16;
    b->nslots = nslots;
    b->cap = slice_bytes;
    b->maxn = maxn;
    b->segcap = slice_bytes / 1024 < 4096 ? 4096 : slice_bytes / 1024;
    b->gather = MD5HIP_GATHER_AUTO;
    b->target = nslots > 2 ? 2 : 1;
    b->linger_max_us = 5000;
    b->chain = 2;
    b->open = -1;
    {
        const char *w = getenv("MD5HIP_WATCH");      /* spin / tail / block (A/B of the watcher) */
        b->watch_policy = !w ? WATCH_POLICY_TAIL
                        : !strcmp(w, "spin") ? WATCH_POLICY_SPIN
                        : !strcmp(w, "block") ? WATCH_POLICY_BLOCK : WATCH_POLICY_TAIL;
    }
    /* BLOCK's watcher sleeps in hipEventSynchronize: blocking-sync events */
    const unsigned done_flags = hipEventDisableTiming |
                                (b->watch_policy == WATCH_POLICY_BLOCK ? hipEventBlockingSync : 0u);
    b->s = calloc(nslots, sizeof *b->s);
    /* ticket 0 = "nothing": complete at once */
    if (!b->s || tk_ring_init(&b->tk, 1)) { rc = -ENOMEM; goto fail; }
    for (uint32_t k = 0; k < nslots; k++) pthread_cond_init(&b->s[k].cv, NULL);
    CK(hipEventCreateWithFlags(&b->after_ev, hipEventDisableTiming));
    for (uint32_t k = 0; k < nslots; k++) {
        struct slot *sl = &b->s[k];
        CK(hipStreamCreateWithFlags(&sl->stream, hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&sl->done, done_flags));
        CK(hipEventCreateWithFlags(&sl->kdone, hipEventDisableTiming));
        CK(hipHostMalloc((void **)&sl->h_data, b->cap, hipHostMallocDefault));
        /* fine-grained: a small slot's kernel reads them in place (slot_prepare) */
        CK(hipHostMalloc((void **)&sl->h_off, 8 * b->maxn, hipHostMallocCoherent));
        CK(hipHostMalloc((void **)&sl->h_len, 4 * b->maxn, hipHostMallocCoherent));
        CK(hipHostGetDevicePointer((void **)&sl->dh_off, sl->h_off, 0));
        CK(hipHostGetDevicePointer((void **)&sl->dh_len, sl->h_len, 0));
        CK(hipHostMalloc((void **)&sl->h_ord, 4 * b->maxn, hipHostMallocDefault));
        CK(hipHostMalloc((void **)&sl->h_dig, 16 * b->maxn, hipHostMallocDefault));
        CK(hipMalloc((void **)&sl->d_data, b->cap));
        CK(hipMalloc((void **)&sl->d_off, 8 * b->maxn));
        CK(hipMalloc((void **)&sl->d_len, 4 * b->maxn));
        CK(hipMalloc((void **)&sl->d_ord, 4 * b->maxn));
        CK(hipMalloc((void **)&sl->d_dig, 16 * b->maxn));
        CK(hipHostMalloc((void **)&sl->h_seg, sizeof(struct md5hip_seg) * b->segcap, hipHostMallocDefault));
        CK(hipMalloc((void **)&sl->d_seg, sizeof(struct md5hip_seg) * b->segcap));
        CK(hipHostMalloc((void **)&sl->h_dsc, sizeof(struct md5hip_seg) * b->segcap, hipHostMallocDefault));
        CK(hipMalloc((void **)&sl->d_dsc, sizeof(struct md5hip_seg) * b->segcap));
        sl->b_dst = malloc(sizeof(void *) * b->segcap);
        sl->b_src = malloc(sizeof(void *) * b->segcap);
        sl->b_len = malloc(sizeof(size_t) * b->segcap);
        sl->b_reg = malloc(sizeof(long) * b->segcap);
        sl->hh = calloc((size_t)MD5HIP_HIST_KMAX + 2, sizeof(uint32_t));
        CK(hipHostMalloc((void **)&sl->h_bkt, sizeof(uint32_t) * ((size_t)MD5HIP_HIST_KMAX + 2),
                         hipHostMallocDefault));
        CK(hipMalloc((void **)&sl->d_bkt, sizeof(uint32_t) * ((size_t)MD5HIP_HIST_KMAX + 2)));
        /* the stable order's scratch for slots past DESC_DIRECT_MAX chunks
         * (none: those slots keep order_scatter) */
        sl->sort_bytes = b->maxn > DESC_DIRECT_MAX ? md5hip_order_stable_scratch(b->maxn, 0) : 0;
        if (sl->sort_bytes && hipMalloc(&sl->d_sort, sl->sort_bytes) != hipSuccess) {
            (void)hipGetLastError();
            sl->d_sort = NULL;
        }
        if (!sl->b_dst || !sl->b_src || !sl->b_len || !sl->b_reg || !sl->hh) { rc = -ENOMEM; goto fail; }
    }
    if (pthread_create(&b->progress, NULL, progress_main, b) != 0) { rc = -EAGAIN; goto fail; }
    b->progress_started = 1;
    *out = b;
    dev_leave(&g);
    return 0;
fail:
    (void)hipGetLastError();          /* a failed allocation is returned as rc, not left sticky */
    batcher_free(b);
    dev_leave(&g);
    return rc;
}

int md5hip_batcher_create(int device, uint64_t slice_bytes, uint32_t nslots, md5hip_batcher **out)
{
    /* defaults sized for MD5's serial chains: a slice of B-byte chunks keeps
     * slice/B lanes busy for B/110 MB/s (one chain), so the bytes in flight
     * must cover PCIe rate x chain time -- 4 x 128 MiB reaches the H2D rate
     * for 256 KiB blocks where 3 x 64 MiB stalls at ~34 GB/s */
    if (slice_bytes == 0) slice_bytes = 128ull << 20;
    uint64_t maxn = slice_bytes / 64 < 4096 ? 4096 : slice_bytes / 64;
    if (maxn > (1u << 20)) maxn = 1u << 20;      /* descriptors: 32 B per chunk */
    return batcher_new(device, slice_bytes, nslots, maxn, out);
}

int md5hip_queue_create(int device, uint64_t max_chunks, uint32_t nslots, md5hip_batcher **out)
{
    if (max_chunks == 0) max_chunks = 1u << 20;
    if (max_chunks > (1ull << 26)) return -EINVAL;
    /* a small staging slice keeps host-memory submissions possible */
    return batcher_new(device, 16ull << 20, nslots, max_chunks, out);
}

/* Wait until nothing is open or in flight (mu held). */
static void drain(md5hip_batcher *b)
{
    for (;;) {
        if (b->open >= 0) {
            struct slot *o = &b->s[b->open];
            o->flush = 1;
            slot_try_launch(b, o);
        }
        int busy = 0;
        for (uint32_t k = 0; k < b->nslots; k++) busy |= b->s[k].state != SLOT_FREE;
        if (!busy) return;
        pthread_cond_wait(&b->done_cv, &b->mu);
    }
}

int md5hip_batcher_set_digest(md5hip_batcher *b, int kind, uint32_t fastcrc)
{
    if (!b) return -EINVAL;
    uint32_t dsz;
    if (kind == MD5HIP_DIGEST_MD5) {
        if (fastcrc) return -EINVAL;
        dsz = 16;
    } else if (kind == MD5HIP_DIGEST_CRC32) {
        if (fastcrc & 3u) return -EINVAL;       /* cfs_apix.c:2222-2236 */
        dsz = 4;
    } else {
        return -EINVAL;
    }
    struct dev_guard g;
    if (dev_enter(&g, b->device)) return -ENODEV;  /* drain may launch the open slot */
    pthread_mutex_lock(&b->mu);
    drain(b);                                    /* never change kind under queued work */
    b->kind = kind;
    b->fastcrc = fastcrc;
    b->dsz = dsz;
    pthread_mutex_unlock(&b->mu);
    dev_leave(&g);
    return 0;
}

int md5hip_batcher_get_digest(const md5hip_batcher *b, int *kind, uint32_t *fastcrc)
{
    if (!b || !kind || !fastcrc) return -EINVAL;
    pthread_mutex_lock((pthread_mutex_t *)&b->mu);
    *kind = b->kind;
    *fastcrc = b->fastcrc;
    pthread_mutex_unlock((pthread_mutex_t *)&b->mu);
    return 0;
}

int md5hip_batcher_set_gather(md5hip_batcher *b, int mode)
{
    if (!b || mode < MD5HIP_GATHER_HOST || mode > MD5HIP_GATHER_AUTO) return -EINVAL;
    pthread_mutex_lock(&b->mu);
    __atomic_store_n(&b->gather, mode, __ATOMIC_RELAXED);
    pthread_mutex_unlock(&b->mu);
    return 0;
}

int md5hip_batcher_set_inflight(md5hip_batcher *b, uint32_t target)
{
    if (!b || target == 0 || target > b->nslots) return -EINVAL;
    struct dev_guard g;
    if (dev_enter(&g, b->device)) return -ENODEV;
    pthread_mutex_lock(&b->mu);
    b->target = target;
    if (b->open >= 0) slot_try_launch(b, &b->s[b->open]);
    pthread_mutex_unlock(&b->mu);
    dev_leave(&g);
    return 0;
}

int md5hip_batcher_set_linger(md5hip_batcher *b, uint32_t max_us)
{
    if (!b) return -EINVAL;
    pthread_mutex_lock(&b->mu);
    b->linger_max_us = max_us;
    pthread_cond_broadcast(&b->work_cv);
    pthread_mutex_unlock(&b->mu);
    return 0;
}

int md5hip_batcher_set_chain(md5hip_batcher *b, int mode)
{
    if (!b || mode < 0 || mode > 2) return -EINVAL;
    pthread_mutex_lock(&b->mu);
    b->chain = mode;
    pthread_mutex_unlock(&b->mu);
    return 0;
}

int md5hip_batcher_health(const md5hip_batcher *b)
{
    if (!b) return -EINVAL;
    return __atomic_load_n(&b->failed, __ATOMIC_ACQUIRE);
}

int md5hip_batcher_inject_fault(md5hip_batcher *b, uint64_t after)
{
    if (!b) return -EINVAL;
    pthread_mutex_lock(&b->mu);
    int rc = b->failed;
    if (!rc) b->inject_at = after ? b->st.launches + after : 0;
    pthread_mutex_unlock(&b->mu);
    return rc;
}

int md5hip_batcher_get_stats(md5hip_batcher *b, struct md5hip_batcher_stats *out)
{
    if (!b || !out) return -EINVAL;
    pthread_mutex_lock(&b->mu);
    *out = b->st;
    out->inflight_target = b->target;
    out->nslots = b->nslots;
    out->max_chunks_per_slot = b->maxn;
    pthread_mutex_unlock(&b->mu);
    return 0;
}

/* ------------------------------------------------------------------------
 * Chunk sources
 * ------------------------------------------------------------------------ */
/* a flat (ptr, len) list, an iovec list with per-chunk segment ranges, or
 * device addresses (no bytes to move) */
struct chunk_src {
    const void *const *ptrs;
    const uint32_t *lens;
    const struct md5hip_iov *segs;
    const uint64_t *seg_first;
    const uint64_t *dptrs;
};

static uint64_t src_len(const struct chunk_src *s, uint64_t i)
{
    if (s->ptrs || s->dptrs) return s->lens[i];
    uint64_t L = 0;
    for (uint64_t j = s->seg_first[i]; j < s->seg_first[i + 1]; j++) L += s->segs[j].len;
    return L;
}

static uint64_t src_nseg(const struct chunk_src *s, uint64_t i)
{
    return s->ptrs ? 1 : s->seg_first[i + 1] - s->seg_first[i];
}

static void src_seg(const struct chunk_src *s, uint64_t i, uint64_t k, const void **base,
                    uint32_t *len)
{
    if (s->ptrs) { *base = s->ptrs[i]; *len = s->lens[i]; return; }
    *base = s->segs[s->seg_first[i] + k].base;
    *len = s->segs[s->seg_first[i] + k].len;
}

/* Every non-empty segment of the call in registered memory? */
static int src_registered(const struct chunk_src *s, uint64_t n)
{
    int ok = 1;
    pthread_rwlock_rdlock(&g_reg_lock);
    for (uint64_t i = 0; i < n && ok; i++)
        for (uint64_t k = 0; k < src_nseg(s, i) && ok; k++) {
            const void *p;
            uint32_t L;
            src_seg(s, i, k, &p, &L);
            if (L && reg_find((uintptr_t)p, L) < 0) ok = 0;
        }
    pthread_rwlock_unlock(&g_reg_lock);
    return ok;
}

static void src_copy(const struct chunk_src *s, uint64_t i, unsigned char *dst)
{
    if (s->ptrs) {
        if (s->lens[i]) memcpy(dst, s->ptrs[i], s->lens[i]);
        return;
    }
    for (uint64_t j = s->seg_first[i]; j < s->seg_first[i + 1]; j++) {
        if (s->segs[j].len) memcpy(dst, s->segs[j].base, s->segs[j].len);
        dst += s->segs[j].len;
    }
}

/* Bytes [a, a + len) of chunk i to dst. */
static void src_copy_range(const struct chunk_src *s, uint64_t i, uint64_t a, uint64_t len, unsigned char *dst)
{
    if (!len) return;
    if (s->ptrs) {
        memcpy(dst, (const unsigned char *)s->ptrs[i] + a, len);
        return;
    }
    for (uint64_t j = s->seg_first[i]; j < s->seg_first[i + 1] && len; j++) {
        const uint64_t sl = s->segs[j].len;
        if (a >= sl) {
            a -= sl;
            continue;
        }
        const uint64_t take = sl - a < len ? sl - a : len;
        memcpy(dst, (const unsigned char *)s->segs[j].base + a, take);
        dst += take;
        len -= take;
        a = 0;
    }
}

/* What a digest reads of an L-byte chunk: netcache's CRC-32 with a fastcrc
 * window F < L reads only the first and the last F bytes (blk_io.c:408-424),
 * so for L > 2F only those 2F bytes are staged and sent, as ONE 2F-byte
 * chunk whose own fastcrc digest is the same crc(head) ^ crc(tail) (a 16 KiB
 * block with F = 128: 256 B over PCIe instead of 16 KiB).  Up to 2F, and
 * for F = 0 (MD5 too), the whole chunk: never more than L bytes, so a chunk
 * that passes submit()'s size check always fits an empty slot. */
static inline uint64_t staged_len(uint32_t F, uint64_t L) { return F && L > 2ull * F ? 2ull * F : L; }

/* Table entries a zero-copy chunk of `ns` segments may take: one per
 * segment, one more when it is sent as two windows (one segment may hold
 * both), plus two spare.  submit() sends a chunk zero-copy only if this fits
 * an empty slot (win = 1, whatever the digest), so reserve() always places
 * it. */
static inline uint64_t zc_pieces(uint64_t ns, int win) { return ns + (win ? 1 : 0) + 2; }

/* chunk i as staged: whole, or its head and tail windows */
static void src_copy_staged(const struct chunk_src *s, uint64_t i, uint32_t F, unsigned char *dst)
{
    const uint64_t L = F ? src_len(s, i) : 0;
    if (staged_len(F, L) == L) {
        src_copy(s, i, dst);
        return;
    }
    src_copy_range(s, i, 0, F, dst);
    src_copy_range(s, i, L - F, F, dst + F);
}

/* Host gather of chunks [first, first + m) to dst + off[j].  One thread's
 * memcpy from pageable memory into pinned staging runs ~15 GB/s (DESIGN.md
 * §5), well below PCIe, so a large range is cut by bytes into parts copied
 * by MD5HIP_GATHER_THREADS threads (default 4; the calling thread copies the
 * first part). */
struct gather_part {
    const struct chunk_src *src;
    uint64_t first, jlo, jhi;
    const uint64_t *off;
    unsigned char *dst;
    uint32_t win;                         /* fastcrc window of a CRC-32 slot (staged_len), else 0 */
};

static void *gather_run(void *arg)
{
    const struct gather_part *p = arg;
    for (uint64_t j = p->jlo; j < p->jhi; j++) src_copy_staged(p->src, p->first + j, p->win, p->dst + p->off[j]);
    return NULL;
}

static pthread_once_t g_gather_once = PTHREAD_ONCE_INIT;
static int g_gather_threads = 4;

static void gather_threads_init(void)
{
    const char *e = getenv("MD5HIP_GATHER_THREADS");
    if (e && *e) {
        const int t = atoi(e);
        g_gather_threads = t < 1 ? 1 : t > 32 ? 32 : t;
    }
}

#define GATHER_SPLIT_MIN (8ull << 20)   /* bytes per range before it is split */
#define GATHER_PART_MIN (2ull << 20)    /* and at least this many bytes per part */

static void gather_range(const struct chunk_src *src, uint64_t first, uint64_t m,
                         const uint64_t *off, unsigned char *dst, uint64_t lo, uint64_t used, uint32_t win)
{
    pthread_once(&g_gather_once, gather_threads_init);
    const uint64_t bytes = used - lo;
    uint64_t T = (uint64_t)g_gather_threads;
    if (bytes < GATHER_SPLIT_MIN) T = 1;
    if (T > bytes / GATHER_PART_MIN) T = bytes / GATHER_PART_MIN ? bytes / GATHER_PART_MIN : 1;
    if (T > m) T = m ? m : 1;
    T = T < 1 ? 1 : T > 32 ? 32 : T;                /* the arrays below */
    struct gather_part part[32];
    pthread_t tid[32];
    int started[32] = {0};
    uint64_t j = 0;
    for (uint64_t t = 0; t < T; t++) {      /* part t: chunks whose offset < lo + (t+1) * bytes / T */
        const uint64_t lim = t + 1 == T ? UINT64_MAX : lo + (t + 1) * bytes / T;
        part[t] = (struct gather_part){src, first, j, j, off, dst, win};
        while (j < m && off[j] < lim) j++;
        part[t].jhi = j;
    }
    for (uint64_t t = 1; t < T; t++)
        started[t] = pthread_create(&tid[t], NULL, gather_run, &part[t]) == 0;
    gather_run(&part[0]);
    for (uint64_t t = 1; t < T; t++) {
        if (started[t]) pthread_join(tid[t], NULL);
        else gather_run(&part[t]);           /* no thread: copy it here */
    }
}

/* ------------------------------------------------------------------------
 * Submission
 * ------------------------------------------------------------------------ */
/* Device-resident chunks [i, i + m) into slot `sl` (mu held, m fits): the
 * descriptors, payload and key histogram in one pass with the running
 * values in registers -- no bytes to stage.  While a burst of C3 vectors is
 * submitted to an idle queue this pass is the device's idle time (bench.py
 * --config c3q `drained`): ~97 us of a 79 K-chunk vector's submission on
 * the box's host, the rest of the call ~3 us of HIP calls (rocprofv3
 * --hip-trace, profiles/r04k/).  Neither threads (slower at every count,
 * profiles/r04f/) nor non-temporal stores (2.4x in isolation,
 * profiles/r04i/, no change in the submission, profiles/r04j/) shortened
 * it, so it stays one plain pass on the calling thread. */
static void reserve_device(md5hip_batcher *b, struct slot *sl, const struct chunk_src *src, uint64_t i,
                           uint64_t m)
{
    uint64_t *ho = sl->h_off + sl->n;
    uint32_t *hl = sl->h_len + sl->n;
    uint32_t *hh = sl->hh;
    const uint64_t *dp = src->dptrs + i;
    const uint32_t *ln = src->lens + i;
    const uint64_t dbase = (uint64_t)(uintptr_t)sl->d_data;
    uint64_t pay = 0, unl = 0;
    uint32_t last = sl->last_key, kmax = sl->hkmax;
    int unsorted = sl->unsorted, hovf = sl->hovf;
    for (uint64_t k = 0; k < m; k++) {
        const uint64_t p = dp[k];
        const uint32_t L = ln[k];
        ho[k] = p - dbase;
        hl[k] = L;
        pay += L;
        unl += ((p & 127u) != 0 && (p & 15u) == 0) ? L : 0;
        const uint32_t key = (L >> 6) + 1;           /* L < 2^32: no overflow */
        unsorted |= key > last;
        last = key;
        if (key > MD5HIP_HIST_KMAX) {
            hovf = 1;
        } else {
            hh[key]++;
            if (key > kmax) kmax = key;
        }
    }
    sl->last_key = last;
    sl->hkmax = kmax;
    sl->unsorted = unsorted;
    sl->hovf = hovf;
    sl->payload += pay;
    sl->unlined += unl;
    sl->load += pay + 64 * m;
    __atomic_store_n(&b->load_bytes, b->load_bytes + pay + 64 * m, __ATOMIC_RELAXED);
    sl->n += m;
}

/* One piece of a zero-copy chunk -- `len` registered bytes at host address
 * p (registration r) -- to staging offset `at` of the slot's gather tables. */
static void zc_piece(struct slot *sl, int dev, const void *p, uint32_t len, long r, uint64_t at)
{
    const uint64_t dsrc = (uint64_t)((uintptr_t)p + g_reg[r].delta[dev]);
    /* device table: contiguous pieces merged up to 64 KiB, so a slice keeps
     * >= ~1000 workgroups of gather work */
    struct md5hip_seg *prev = sl->nseg ? &sl->h_seg[sl->nseg - 1] : NULL;
    if (prev && prev->src + prev->len == dsrc && prev->dst + prev->len == at &&
        (uint64_t)prev->len + len <= (64u << 10)) {
        prev->len += len;
    } else {
        sl->h_seg[sl->nseg++] = (struct md5hip_seg){dsrc, at, len, 0};
    }
    /* DMA list: merged without limit (a copy has a fixed cost), but only
     * within one registered range (one pinned allocation) */
    const uint64_t q1 = sl->ndma;
    if (q1 && sl->b_reg[q1 - 1] == r &&
        (const unsigned char *)sl->b_src[q1 - 1] + sl->b_len[q1 - 1] == (const unsigned char *)p &&
        (unsigned char *)sl->b_dst[q1 - 1] + sl->b_len[q1 - 1] == sl->d_data + at) {
        sl->b_len[q1 - 1] += len;
    } else {
        sl->b_dst[q1] = sl->d_data + at;
        sl->b_src[q1] = (void *)p;
        sl->b_len[q1] = len;
        sl->b_reg[q1] = r;
        sl->ndma++;
    }
}

/* Reserve chunks [i, n) of `src` into the open slot (mu held): descriptors,
 * staging offsets, zero-copy tables.  Returns the number reserved (the slot
 * is marked full when a chunk did not fit) or -errno.  A CRC-32 slot with a
 * fastcrc window stages each longer chunk's two windows only (staged_len). */
static long reserve(md5hip_batcher *b, struct slot *sl, const struct chunk_src *src, uint64_t i,
                    uint64_t n, int zc)
{
    const int dev = b->device;
    const uint32_t F = sl->kind == MD5HIP_DIGEST_CRC32 ? sl->fastcrc : 0;
    uint64_t j = i;
    if (sl->n == 0 && i < n) sl->opened_us = now_us();
    if (src->dptrs) {
        const uint64_t m = n - i < b->maxn - sl->n ? n - i : b->maxn - sl->n;
        reserve_device(b, sl, src, i, m);
        if (i + m < n) sl->full = 1;
        return (long)m;
    }
    if (zc) pthread_rwlock_rdlock(&g_reg_lock);
    while (j < n && sl->n < b->maxn) {
        const uint64_t L = src_len(src, j);
        const uint64_t E = staged_len(F, L);
        {   /* host bytes (device-resident chunks: reserve_device above) */
            /* chunks packed on 128-B lines: the LDS-DMA loaders read 128-B
             * stages, and a stage off the line shares a line with the next
             * one (the nt policy is then off, md5_kernels.h) */
            const uint64_t sz = (E + 127) & ~127ull;
            if (sl->used + sz > b->cap) break;
            if (zc) {
                const uint64_t ns = src_nseg(src, j);
                /* the chunk's byte ranges staged: all of it, or its windows */
                const int win = E != L;
                const uint64_t need = zc_pieces(ns, win);
                if (sl->nseg + need > b->segcap || sl->ndma + need > b->segcap) break;
                const uint64_t ra[2] = {0, win ? L - F : 0}, rl[2] = {win ? F : L, win ? F : 0};
                uint64_t at = sl->used;
                for (int w = 0; w < 2; w++) {
                    uint64_t a = ra[w], left = rl[w];
                    for (uint64_t q = 0; q < ns && left; q++) {
                        const void *p;
                        uint32_t len;
                        src_seg(src, j, q, &p, &len);
                        if (a >= len) {
                            a -= len;
                            continue;
                        }
                        const uint32_t take = (uint32_t)(len - a < left ? len - a : left);
                        const void *pp = (const unsigned char *)p + a;
                        a = 0;
                        left -= take;
                        const long r = reg_find((uintptr_t)pp, take);
                        if (r < 0) {                           /* unregistered under us */
                            pthread_rwlock_unlock(&g_reg_lock);
                            return -EFAULT;
                        }
                        zc_piece(sl, dev, pp, take, r, at);
                        at += take;
                    }
                }
            }
            sl->h_off[sl->n] = sl->used;
            sl->used += sz;
        }
        sl->h_len[sl->n] = (uint32_t)E;
        sl->load += E + 64;
        sl->payload += E;
        __atomic_store_n(&b->load_bytes, b->load_bytes + E + 64, __ATOMIC_RELAXED);
        {
            const uint64_t k = (E >> 6) + 1;
            if (k > sl->last_key) sl->unsorted = 1;
            sl->last_key = k > UINT32_MAX ? UINT32_MAX : (uint32_t)k;
            if (k > MD5HIP_HIST_KMAX) {
                sl->hovf = 1;
            } else {
                sl->hh[k]++;
                if (k > sl->hkmax) sl->hkmax = (uint32_t)k;
            }
        }
        sl->n++;
        j++;
    }
    if (zc) pthread_rwlock_unlock(&g_reg_lock);
    if (j < n) sl->full = 1;
    return (long)(j - i);
}

/* The submission engine.
 *   async   0 = synchronous (returns when the digests are delivered);
 *           1 = asynchronous (*ticket; the slot may linger and coalesce);
 *           2 = asynchronous but launched at once like a synchronous call
 *               (the caller waits on *ticket right away: the pool's
 *               synchronous entries)
 *   kind    < 0: the batcher's current digest kind; else this submission's
 *           own (it never changes the batcher's setting)
 *   after   != NULL: *after is the producer's stream (NULL there = the null
 *           stream) -- every slot taking chunks of this submission waits on
 *           the producer's work enqueued so far before its kernel (an event
 *           recorded on *after, waited on by the slot's stream) */
static int submit(md5hip_batcher *b, const struct chunk_src *src, uint64_t n, unsigned char *digests,
                  int on_device, int async, uint64_t *ticket, int kind, uint32_t fastcrc,
                  const hipStream_t *after)
{
    const int urgent = async != 1;
    for (uint64_t i = 0; !src->dptrs && i < n; i++) {   /* device chunks: uint32 lengths, no staging */
        const uint64_t L = src_len(src, i);
        if (L > 0xffffffffull) return -E2BIG;
        if ((L + 127) / 128 * 128 > b->cap) return -E2BIG;
    }
    struct dev_guard g;
    if (dev_enter(&g, b->device)) return -ENODEV;
    int zc = 0;
    /* gather is read here without mu (set_gather may change it meanwhile):
     * it only decides whether this submission may go zero-copy */
    if (!src->dptrs && __atomic_load_n(&b->gather, __ATOMIC_RELAXED) != MD5HIP_GATHER_HOST &&
        b->device < REG_MAXDEV &&
        src_registered(src, n)) {
        zc = 1;
        for (uint64_t i = 0; i < n; i++)
            if (zc_pieces(src_nseg(src, i), 1) > b->segcap) zc = 0;   /* too fragmented for one table */
    }
    const int mode = src->dptrs ? MODE_NONE : zc ? MODE_ZEROCOPY : MODE_STAGED;
    pthread_mutex_lock(&b->mu);
    int rc = 0;
    uint64_t t = 0;
    if (kind < 0) {
        kind = b->kind;
        fastcrc = b->fastcrc;
    }
    rc = b->failed ? b->failed : tk_new(b, &t);
    if (rc == 0 && after && hipEventRecord(b->after_ev, *after) != hipSuccess) {
        tk_put(b, t, 0);
        rc = -EINVAL;                              /* not a stream of this device */
    }
    if (rc) {
        pthread_mutex_unlock(&b->mu);
        dev_leave(&g);
        return rc;
    }
    b->st.submissions++;
    const uint32_t dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
    uint64_t i = 0;
    while (i < n) {
        struct slot *sl = b->failed ? NULL : slot_open(b, mode, kind, fastcrc);
        if (!sl || b->failed) {              /* the device failed meanwhile (slot_open may wait) */
            if (sl) slot_try_launch(b, sl);  /* an empty slot it opened retires */
            rc = -ENODEV;
            break;
        }
        const uint64_t at = sl->n;
        const uint64_t lo = sl->used;
        const long got = reserve(b, sl, src, i, n, zc);
        if (got < 0) { rc = (int)got; break; }
        if (got == 0) {                      /* nothing fit: close it and take a fresh one */
            sl->full = 1;
            b->open = -1;
            slot_try_launch(b, sl);
            continue;
        }
        const uint64_t m = (uint64_t)got;
        const uint64_t hi = sl->used;
        /* a large device-resident range: its descriptors go over now, on the
         * slot's idle stream, instead of after the burst's last submission
         * (a drained c3q step's 6 vectors: ~0.12 ms of copies that no longer
         * sit between the burst and its kernel); appended descriptors are
         * final, slot_prepare copies only what follows */
        if (src->dptrs && m >= EARLY_COPY_MIN && sl->n > DESC_DIRECT_MAX && sl->n > sl->copied_n) {
            const uint64_t c0 = sl->copied_n, cn = sl->n - c0;
            if (hipMemcpyAsync(sl->d_off + c0, sl->h_off + c0, 8 * cn, hipMemcpyHostToDevice, sl->stream) ||
                hipMemcpyAsync(sl->d_len + c0, sl->h_len + c0, 4 * cn, hipMemcpyHostToDevice, sl->stream)) {
                if (!sl->err) sl->err = -EIO;
            } else {
                sl->copied_n = sl->n;
            }
        }
        /* recorded and waited on under one hold of b->mu (slot_take may have
         * let another producer record the event meanwhile), before this
         * slot's kernel can be enqueued: the kernel runs after the producer's
         * work enqueued up to here */
        if (after && (hipEventRecord(b->after_ev, *after) != hipSuccess ||
                      hipStreamWaitEvent(sl->stream, b->after_ev, 0) != hipSuccess) && !sl->err)
            sl->err = -EIO;
        if ((rc = seg_push(sl, (struct seg){t, at, m, digests + (size_t)dsz * i, on_device}))) {
            sl->err = rc;                    /* its reserved chunks have no segment */
            break;
        }
        tk_ring_ref(&b->tk, t);
        if (mode == MODE_STAGED && hi > lo) {
            /* copy outside the lock: other submitters may reserve behind us */
            sl->writers++;
            pthread_mutex_unlock(&b->mu);
            gather_range(src, i, m, sl->h_off + at, sl->h_data, lo, hi,
                         sl->kind == MD5HIP_DIGEST_CRC32 ? sl->fastcrc : 0);
            pthread_mutex_lock(&b->mu);
            sl->writers--;
        }
        i += m;
        /* the caller waits right away: no linger; the slot goes while fewer
         * than nslots - 1 launches run, else it coalesces in the last slot
         * (slot_try_launch) -- forcing every synchronous call out at once
         * made one launch per vector at ASIO scale (profiles/r04b/), and
         * holding them to `target` launches cost the 8-thread call site a
         * fifth of its throughput (profiles/r04d/asio_threads.json) */
        if (urgent && i >= n) sl->urgent = 1;
        slot_try_launch(b, sl);
    }
    tk_put(b, t, rc);                        /* the submission's own reference */
    if (ticket) *ticket = t;
    if (!async || rc) {
        const int err = wait_ticket(b, t);
        if (!rc) rc = err;
    }
    pthread_mutex_unlock(&b->mu);
    dev_leave(&g);
    return rc;
}

/* A waiter or poller on `ticket` (mu held): if its chunks sit in the open
 * slot and nothing is in flight, launch that slot now (no linger).  While
 * launches are in flight the slot keeps coalescing and goes out as soon as
 * one retires (the inflight target holds; its plan is made meanwhile) --
 * forcing it out beside a running launch only splits the device between
 * them. */
static void hasten(md5hip_batcher *b, uint64_t ticket)
{
    for (uint32_t k = 0; k < b->nslots; k++)
        if (b->s[k].state == SLOT_OPEN && seg_has(&b->s[k], ticket)) {
            if (b->inflight == 0) b->s[k].flush = 1;
            slot_try_launch(b, &b->s[k]);
        }
}

/* Wait, poll and flush may launch the open slot from the caller's thread
 * (slot_enqueue's device-keyed state: the BALANCED counter, CU counts), so
 * they run on the batcher's device like submit -- a pool waits on a ticket
 * of one device from a thread whose current device is another. */
int md5_batch_wait(md5hip_batcher *b, uint64_t ticket)
{
    if (!b) return -EINVAL;
    if (ticket == 0) return 0;               /* "nothing submitted" */
    struct dev_guard g;
    if (dev_enter(&g, b->device)) return -ENODEV;
    pthread_mutex_lock(&b->mu);
    const int rc = ticket >= b->tk.hi ? -EINVAL : wait_ticket(b, ticket);
    pthread_mutex_unlock(&b->mu);
    dev_leave(&g);
    return rc;
}

int md5_batch_poll(md5hip_batcher *b, uint64_t ticket)
{
    if (!b) return -EINVAL;
    if (ticket == 0) return 1;
    struct dev_guard g;
    if (dev_enter(&g, b->device)) return -ENODEV;
    pthread_mutex_lock(&b->mu);
    int rc, err = 0;
    if (ticket >= b->tk.hi) {
        rc = -EINVAL;
    } else if (tk_done(b, ticket, &err)) {
        rc = err ? err : 1;
    } else {
        hasten(b, ticket);                   /* progress without the caller blocking */
        rc = 0;
    }
    pthread_mutex_unlock(&b->mu);
    dev_leave(&g);
    return rc;
}

int md5_batch_flush(md5hip_batcher *b)
{
    if (!b) return -EINVAL;
    struct dev_guard g;
    if (dev_enter(&g, b->device)) return -ENODEV;
    pthread_mutex_lock(&b->mu);
    if (b->open >= 0) {
        struct slot *o = &b->s[b->open];
        o->flush = 1;
        slot_try_launch(b, o);
    }
    pthread_mutex_unlock(&b->mu);
    dev_leave(&g);
    return 0;
}

static int check_ptrs(const void *const *ptrs, const uint32_t *lens, uint64_t n)
{
    if (!ptrs || !lens) return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (!ptrs[i] && lens[i]) return -EINVAL;
    return 0;
}

static int check_iov(const struct md5hip_iov *segs, const uint64_t *seg_first, uint64_t n)
{
    if (!segs || !seg_first || seg_first[0] != 0) return -EINVAL;
    for (uint64_t i = 0; i < n; i++) {
        if (seg_first[i + 1] < seg_first[i]) return -EINVAL;
        for (uint64_t j = seg_first[i]; j < seg_first[i + 1]; j++)
            if (!segs[j].base && segs[j].len) return -EINVAL;
    }
    return 0;
}

int md5_batch_submit(md5hip_batcher *b, const void *const *ptrs, const uint32_t *lens, uint64_t n,
                     unsigned char *digests)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = check_ptrs(ptrs, lens, n);
    if (rc) return rc;
    const struct chunk_src src = {ptrs, lens, NULL, NULL, NULL};
    return submit(b, &src, n, digests, 0, 0, NULL, -1, 0, NULL);
}

int md5_batch_submit_async(md5hip_batcher *b, const void *const *ptrs, const uint32_t *lens,
                           uint64_t n, unsigned char *digests, uint64_t *ticket)
{
    if (!b || !ticket) return -EINVAL;
    *ticket = 0;                           /* an empty batch is complete at once */
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = check_ptrs(ptrs, lens, n);
    if (rc) return rc;
    const struct chunk_src src = {ptrs, lens, NULL, NULL, NULL};
    return submit(b, &src, n, digests, 0, 1, ticket, -1, 0, NULL);
}

int md5_batch_submit_iov(md5hip_batcher *b, const struct md5hip_iov *segs,
                         const uint64_t *seg_first, uint64_t n, unsigned char *digests)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = check_iov(segs, seg_first, n);
    if (rc) return rc;
    const struct chunk_src src = {NULL, NULL, segs, seg_first, NULL};
    return submit(b, &src, n, digests, 0, 0, NULL, -1, 0, NULL);
}

int md5_batch_submit_iov_async(md5hip_batcher *b, const struct md5hip_iov *segs,
                               const uint64_t *seg_first, uint64_t n, unsigned char *digests,
                               uint64_t *ticket)
{
    if (!b || !ticket) return -EINVAL;
    *ticket = 0;
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = check_iov(segs, seg_first, n);
    if (rc) return rc;
    const struct chunk_src src = {NULL, NULL, segs, seg_first, NULL};
    return submit(b, &src, n, digests, 0, 1, ticket, -1, 0, NULL);
}

int md5_batch_submit_device_async(md5hip_batcher *b, const uint64_t *d_ptrs, const uint32_t *lens,
                                  uint64_t n, unsigned char *digests, int digests_on_device,
                                  uint64_t *ticket)
{
    if (!b || !ticket) return -EINVAL;
    *ticket = 0;
    if (n == 0) return 0;
    if (!d_ptrs || !lens || !digests) return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (!d_ptrs[i] && lens[i]) return -EINVAL;
    const struct chunk_src src = {NULL, lens, NULL, NULL, d_ptrs};
    return submit(b, &src, n, digests, digests_on_device != 0, 1, ticket, -1, 0, NULL);
}

int md5_batch_submit_device(md5hip_batcher *b, const uint64_t *d_ptrs, const uint32_t *lens,
                            uint64_t n, unsigned char *digests, int digests_on_device)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!d_ptrs || !lens || !digests) return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (!d_ptrs[i] && lens[i]) return -EINVAL;
    const struct chunk_src src = {NULL, lens, NULL, NULL, d_ptrs};
    return submit(b, &src, n, digests, digests_on_device != 0, 0, NULL, -1, 0, NULL);
}

/* Is the byte at p page-locked host memory known to the runtime? */
static int pinned_at(const void *p)
{
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();                  /* pageable: not an error of ours */
        return 0;
    }
    return a.type == hipMemoryTypeHost;
}

/* Is [p, p + len) page-locked host memory the DMA engine can read in place
 * (hipHostMalloc'd, hipHostRegister'ed, or registered here)?  The whole
 * range, not its first byte: a source that starts in a pinned block and runs
 * on into pageable memory is staged.  Both ends must be pinned, and the
 * runtime's allocation holding the first byte must hold the last too (HIP's
 * RANGE_START/RANGE_SIZE attribute, else hipMemGetAddressRange); a range
 * whose extent the runtime will not tell is staged. */
static int host_pinned(const void *p, uint64_t len)
{
    if (!len) return 0;
    pthread_rwlock_rdlock(&g_reg_lock);
    const int reg = reg_find((uintptr_t)p, len) >= 0;
    pthread_rwlock_unlock(&g_reg_lock);
    if (reg) return 1;
    const uintptr_t lo = (uintptr_t)p, hi = lo + len;      /* [lo, hi) */
    if (!pinned_at(p) || !pinned_at((const void *)(hi - 1))) return 0;
    void *start = NULL;
    size_t size = 0;
    if (hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p) == hipSuccess &&
        hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p) == hipSuccess &&
        start && size)
        return (uintptr_t)start <= lo && hi <= (uintptr_t)start + size;
    (void)hipGetLastError();
    if (hipMemGetAddressRange((hipDeviceptr_t *)&start, &size, (hipDeviceptr_t)p) == hipSuccess && start && size)
        return (uintptr_t)start <= lo && hi <= (uintptr_t)start + size;
    (void)hipGetLastError();
    return 0;
}

/* memcpy of `bytes` on MD5HIP_GATHER_THREADS threads (gather_range's rule:
 * parts of >= 2 MiB once the copy passes 8 MiB; this thread copies the
 * first part) */
struct copy_part {
    unsigned char *dst;
    const unsigned char *src;
    uint64_t len;
};

static void *copy_run(void *arg)
{
    const struct copy_part *c = arg;
    memcpy(c->dst, c->src, c->len);
    return NULL;
}

static void copy_parallel(void *dst, const void *src, uint64_t bytes)
{
    pthread_once(&g_gather_once, gather_threads_init);
    uint64_t T = (uint64_t)g_gather_threads;
    if (bytes < GATHER_SPLIT_MIN) T = 1;
    if (T > bytes / GATHER_PART_MIN) T = bytes / GATHER_PART_MIN ? bytes / GATHER_PART_MIN : 1;
    T = T < 1 ? 1 : T > 32 ? 32 : T;                /* the arrays below */
    struct copy_part part[32];
    pthread_t tid[32];
    int started[32] = {0};
    for (uint64_t t = 0; t < T; t++) {
        const uint64_t a = bytes * t / T, z = bytes * (t + 1) / T;
        part[t] = (struct copy_part){(unsigned char *)dst + a, (const unsigned char *)src + a, z - a};
    }
    for (uint64_t t = 1; t < T; t++) started[t] = pthread_create(&tid[t], NULL, copy_run, &part[t]) == 0;
    copy_run(&part[0]);
    for (uint64_t t = 1; t < T; t++) {
        if (started[t]) pthread_join(tid[t], NULL);
        else copy_run(&part[t]);
    }
}

/* Fixed-length chunks from one contiguous range (MODE_FIXED), one slot per
 * slice of it: host memory (dev_src 0: one H2D copy per slot, no host
 * gather) or device memory (dev_src 1: read in place, no per-chunk
 * descriptor -- md5_batch_submit_device_fixed).  Digests to host memory, or
 * device memory when dig_dev.  after != NULL: the producer's stream, as
 * submit().  ticket NULL = synchronous. */
static int fixed_submit(md5hip_batcher *b, int kind, uint32_t fastcrc, const void *base, int dev_src,
                        uint64_t n, uint32_t len, uint64_t stride, unsigned char *digests, int dig_dev,
                        const hipStream_t *after, uint64_t *ticket)
{
    if (!dev_src && stride > b->cap) return -E2BIG;
    struct dev_guard g;
    if (dev_enter(&g, b->device)) return -ENODEV;
    const unsigned char *src = (const unsigned char *)base;
    uint64_t per = dev_src || !stride ? b->maxn : b->cap / stride;   /* stride 0: empty chunks */
    if (per > b->maxn) per = b->maxn;
    /* a pageable source is copied into the slot's pinned staging by this
     * thread: HIP's own pageable H2D path stalls other threads' HIP calls on
     * the device while it runs (submitters' p90 +2.7 ms beside 128 MiB
     * slices, profiles/r05f/) */
    const int pinned = !dev_src && n && host_pinned(base, (n - 1) * stride + len);
    pthread_mutex_lock(&b->mu);
    if (kind < 0) {
        kind = b->kind;
        fastcrc = b->fastcrc;
    }
    const uint32_t dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
    uint64_t t = 0;
    int rc = b->failed ? b->failed : tk_new(b, &t);
    if (rc == 0 && after && hipEventRecord(b->after_ev, *after) != hipSuccess) {
        tk_put(b, t, 0);
        rc = -EINVAL;                              /* not a stream of this device */
    }
    if (rc) {
        pthread_mutex_unlock(&b->mu);
        dev_leave(&g);
        return rc;
    }
    b->st.submissions++;
    for (uint64_t i = 0; i < n && !rc; i += per) {
        const uint64_t m = n - i < per ? n - i : per;
        /* straight from the caller's buffer: a slot of its own (the open
         * slot keeps coalescing other work) */
        struct slot *sl = b->failed ? NULL : slot_take(b, MODE_FIXED, kind, fastcrc);
        if (!sl || b->failed) {              /* the device failed (slot_take may wait) */
            if (sl) slot_retire(b, sl, -ENODEV);
            rc = -ENODEV;
            break;
        }
        sl->n = m;
        sl->fx_src = src + i * stride;
        sl->fx_dev = dev_src;
        sl->fx_bytes = (m - 1) * stride + len;
        sl->fx_len = len;
        sl->fx_stride = stride;
        sl->full = 1;
        sl->load = m * ((uint64_t)len + 64);
        __atomic_store_n(&b->load_bytes, b->load_bytes + sl->load, __ATOMIC_RELAXED);
        if ((rc = seg_push(sl, (struct seg){t, 0, m, digests + (size_t)dsz * i, dig_dev}))) {
            slot_retire(b, sl, rc);
            break;
        }
        tk_ring_ref(&b->tk, t);
        /* the producer's work before this call, before this slot's kernel
         * (recorded again per slot: slot_take may have let another producer
         * record the event meanwhile) */
        if (after && (hipEventRecord(b->after_ev, *after) != hipSuccess ||
                      hipStreamWaitEvent(sl->stream, b->after_ev, 0) != hipSuccess))
            sl->err = -EIO;
        if (!dev_src) {
            /* the copy outside the lock, the slot held by this writer: a
             * pageable source through the pinned staging (host_pinned), a
             * pinned one by DMA in place; every other submitter and waiter
             * needs b->mu meanwhile.  Nothing else touches a FIXED slot's
             * stream or staging until its writers are done (slot_try_launch
             * waits for writers == 0). */
            sl->writers++;
            pthread_mutex_unlock(&b->mu);
            const void *from = sl->fx_src;
            if (!pinned) {
                copy_parallel(sl->h_data, sl->fx_src, sl->fx_bytes);
                from = sl->h_data;
            }
            const hipError_t ce = hipMemcpyAsync(sl->d_data, from, sl->fx_bytes, hipMemcpyHostToDevice, sl->stream);
            pthread_mutex_lock(&b->mu);
            sl->writers--;
            if (!pinned) b->st.bytes_staged += sl->fx_bytes;
            if (ce != hipSuccess && !sl->err) sl->err = -EIO;
            if (ce != hipSuccess && hip_lost(hipStreamQuery(sl->stream))) batcher_fail(b);
        }
        slot_try_launch(b, sl);
    }
    tk_put(b, t, rc);
    if (ticket) *ticket = t;
    if (!ticket || rc) {
        const int err = wait_ticket(b, t);
        if (!rc) rc = err;
    }
    pthread_mutex_unlock(&b->mu);
    dev_leave(&g);
    return rc;
}

static int host_fixed(md5hip_batcher *b, int kind, uint32_t fastcrc, const void *h_base, uint64_t n,
                      uint32_t len, uint64_t stride, unsigned char *digests, uint64_t *ticket)
{
    return fixed_submit(b, kind, fastcrc, h_base, 0, n, len, stride, digests, 0, NULL, ticket);
}

int md5_batch_submit_device_fixed(md5hip_batcher *b, const void *d_base, uint64_t n, uint32_t len,
                                  uint64_t stride, unsigned char *digests, int digests_on_device,
                                  void *producer_stream, int order, uint64_t *ticket)
{
    if (ticket) *ticket = 0;
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!d_base || !digests || len > stride) return -EINVAL;
    const hipStream_t after = (hipStream_t)producer_stream;
    return fixed_submit(b, -1, 0, d_base, 1, n, len, stride, digests, digests_on_device != 0,
                        order ? &after : NULL, ticket);
}

int md5_batch_submit_device_after(md5hip_batcher *b, const uint64_t *d_ptrs, const uint32_t *lens,
                                  uint64_t n, unsigned char *digests, int digests_on_device,
                                  void *producer_stream, int order, uint64_t *ticket)
{
    if (ticket) *ticket = 0;
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!d_ptrs || !lens || !digests) return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (!d_ptrs[i] && lens[i]) return -EINVAL;
    const struct chunk_src src = {NULL, lens, NULL, NULL, d_ptrs};
    const hipStream_t after = (hipStream_t)producer_stream;
    return submit(b, &src, n, digests, digests_on_device != 0, ticket != NULL, ticket, -1, 0,
                  order ? &after : NULL);
}

int md5_batch_submit_device_on(md5hip_batcher *b, const uint64_t *d_ptrs, const uint32_t *lens,
                               uint64_t n, unsigned char *digests, int digests_on_device,
                               void *producer_stream, uint64_t *ticket)
{
    return md5_batch_submit_device_after(b, d_ptrs, lens, n, digests, digests_on_device,
                                         producer_stream, producer_stream != NULL, ticket);
}

int md5hip_batch_host_fixed(md5hip_batcher *b, const void *h_base, uint64_t n, uint32_t len,
                            uint64_t stride, unsigned char *digests)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!h_base || !digests || len > stride) return -EINVAL;
    return host_fixed(b, -1, 0, h_base, n, len, stride, digests, NULL);
}

/* ------------------------------------------------------------------------
 * Entries for the multi-GPU pool (md5_internal.h)
 * ------------------------------------------------------------------------ */
uint64_t md5hip_batcher_load(const md5hip_batcher *b)
{
    return __atomic_load_n(&b->load_bytes, __ATOMIC_RELAXED);
}

uint64_t md5hip_batcher_slice(const md5hip_batcher *b) { return b->cap; }

int md5hip_submit_as(md5hip_batcher *b, int kind, uint32_t fastcrc, const void *const *ptrs,
                     const uint32_t *lens, const struct md5hip_iov *segs, const uint64_t *seg_first,
                     uint64_t n, unsigned char *digests, uint64_t *ticket, int urgent)
{
    if (ticket) *ticket = 0;
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = ptrs ? check_ptrs(ptrs, lens, n) : check_iov(segs, seg_first, n);
    if (rc) return rc;
    const struct chunk_src src = {ptrs, ptrs ? lens : NULL, ptrs ? NULL : segs, ptrs ? NULL : seg_first,
                                  NULL};
    return submit(b, &src, n, digests, 0, ticket ? (urgent ? 2 : 1) : 0, ticket, kind, fastcrc, NULL);
}

int md5hip_host_fixed_as(md5hip_batcher *b, int kind, uint32_t fastcrc, const void *h_base,
                         uint64_t n, uint32_t len, uint64_t stride, unsigned char *digests,
                         uint64_t *ticket)
{
    if (ticket) *ticket = 0;
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!h_base || !digests || len > stride) return -EINVAL;
    return host_fixed(b, kind, fastcrc, h_base, n, len, stride, digests, ticket);
}

int md5hip_batcher_ticket_state(md5hip_batcher *b, uint64_t ticket, int *err)
{
    *err = 0;
    if (ticket == 0) return 1;
    pthread_mutex_lock(&b->mu);
    int rc = ticket >= b->tk.hi ? -EINVAL : tk_done(b, ticket, err);
    pthread_mutex_unlock(&b->mu);
    return rc;
}

/* Batched verify for the cache-read / write-verify sites (blk_io.c:665-704,
 * bc_mgr.c:1464-1492): ok[i] = digest(chunk i) == expected[i]; returns the
 * number of mismatching chunks (>= 0) or -errno.  A mismatch is what
 * dm_verify_block_crc (diskcache.c:3245-3265) reports per block; the caller
 * applies its own EAGAIN / inode-reset policy per flagged block.
 * md5hip_verify_iov_as: with an explicit digest kind for this call only (the
 * batcher's setting is untouched, so concurrent users are unaffected). */
int md5hip_verify_iov_as(md5hip_batcher *b, int kind, uint32_t fastcrc,
                         const struct md5hip_iov *segs, const uint64_t *seg_first, uint64_t n,
                         const void *expected, unsigned char *ok)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!expected || !ok) return -EINVAL;
    if (kind != MD5HIP_DIGEST_MD5 && kind != MD5HIP_DIGEST_CRC32) return -EINVAL;
    if (kind == MD5HIP_DIGEST_MD5 ? fastcrc != 0 : (fastcrc & 3u) != 0) return -EINVAL;
    int rc = check_iov(segs, seg_first, n);
    if (rc) return rc;
    const uint32_t dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
    unsigned char *got = malloc((size_t)dsz * n);
    if (!got) return -ENOMEM;
    const struct chunk_src src = {NULL, NULL, segs, seg_first, NULL};
    rc = submit(b, &src, n, got, 0, 0, NULL, kind, fastcrc, NULL);
    if (rc == 0) {
        const unsigned char *e = (const unsigned char *)expected;
        for (uint64_t i = 0; i < n; i++) {
            ok[i] = memcmp(got + (size_t)dsz * i, e + (size_t)dsz * i, dsz) == 0;
            rc += !ok[i];
        }
    }
    free(got);
    return rc;
}

int md5hip_batch_verify_iov(md5hip_batcher *b, const struct md5hip_iov *segs,
                            const uint64_t *seg_first, uint64_t n, const void *expected,
                            unsigned char *ok)
{
    if (!b) return -EINVAL;
    int kind;
    uint32_t fastcrc;
    md5hip_batcher_get_digest(b, &kind, &fastcrc);
    return md5hip_verify_iov_as(b, kind, fastcrc, segs, seg_first, n, expected, ok);
}
