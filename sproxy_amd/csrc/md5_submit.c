/*
 * md5_submit.c -- host-memory batched submit (include/md5hip.h).
 *
 * Serves the netcache block-completion checksum site (blk_make_crc,
 * netcache/common/blk_io.c:354-430): chunks live in host memory (cache pages,
 * socket buffers), so the batch is staged H2D, hashed on the device and the
 * 16-byte digests come back D2H.  A batcher owns `nslots` pipeline slots; slot
 * k has its own HIP stream, pinned staging buffer, device buffer, descriptor
 * arrays and completion event, so the host gather of slice k+1, the H2D copy
 * of slice k and the kernel of slice k-1 overlap.
 *
 * Errors: 0 / negative errno (include/md5hip.h conventions); -E2BIG when one
 * chunk alone exceeds the slot's staging capacity.
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <hip/hip_runtime_api.h>

#include "../../include/md5hip.h"
#include "md5_internal.h"

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

int md5hip_host_register(void *base, uint64_t bytes)
{
    if (!base || bytes == 0) return -EINVAL;
    const uintptr_t lo = (uintptr_t)base, hi = lo + bytes;
    int ndev = 0, cur = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= 0) return -ENODEV;
    if (ndev > REG_MAXDEV) ndev = REG_MAXDEV;
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
     * writes (calls are synchronous), and DMA from coarse-grained pages runs
     * 44 vs 34 GB/s; MD5HIP_REGISTER_COARSE=0 turns it off */
    unsigned flags = hipHostRegisterPortable | hipHostRegisterMapped;
    const char *coarse = getenv("MD5HIP_REGISTER_COARSE");
    if (!coarse || atoi(coarse)) flags |= hipExtHostRegisterCoarseGrained;
    if (hipHostRegister(base, bytes, flags) != hipSuccess) {
        rc = -ENODEV;
        goto out;
    }
    struct reg_range r = {lo, hi, {0}};
    (void)hipGetDevice(&cur);
    for (int d = 0; d < ndev; d++) {
        void *dp = NULL;
        if (hipSetDevice(d) == hipSuccess && hipHostGetDevicePointer(&dp, base, 0) == hipSuccess)
            r.delta[d] = (intptr_t)((uintptr_t)dp - lo);
    }
    (void)hipSetDevice(cur);
    memmove(&g_reg[at + 1], &g_reg[at], (g_nreg - at) * sizeof *g_reg);
    g_reg[at] = r;
    g_nreg++;
out:
    pthread_rwlock_unlock(&g_reg_lock);
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

struct slot {
    hipStream_t stream;
    hipEvent_t done;
    unsigned char *h_data, *d_data;   /* staging, `cap` bytes */
    uint64_t *h_off, *d_off;          /* descriptors, `maxn` entries */
    uint32_t *h_len, *d_len;
    uint32_t *h_ord, *d_ord;
    unsigned char *h_dig, *d_dig;     /* 16 * maxn */
    struct md5hip_seg *h_seg, *d_seg; /* zero-copy gather table, `segcap` entries */
    void **b_dst, **b_src;            /* DMA-batch gather arrays (plain host memory) */
    size_t *b_len;
    unsigned char *user_dig;          /* where this slot's digests go (NULL = idle) */
    uint64_t ticket;                  /* submission the in-flight work belongs to */
    uint64_t ndig;
    uint32_t dsz;
    int busy;
};

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
    uint32_t next;     /* slot the next slice goes to (round robin across calls) */
    uint64_t ticket;   /* last submission ticket issued (md5_batch_wait) */
    struct slot *s;
};

#define CK(x) do { if ((x) != hipSuccess) { rc = -ENODEV; goto fail; } } while (0)

static int slot_retire(struct slot *sl)
{
    if (!sl->busy) return 0;
    if (hipEventSynchronize(sl->done) != hipSuccess) return -EIO;
    if (sl->user_dig) memcpy(sl->user_dig, sl->h_dig, (size_t)sl->dsz * sl->ndig);
    sl->busy = 0;
    sl->user_dig = NULL;
    return 0;
}

void md5hip_batcher_destroy(md5hip_batcher *b)
{
    if (!b) return;
    hipSetDevice(b->device);
    for (uint32_t k = 0; b->s && k < b->nslots; k++) {
        struct slot *sl = &b->s[k];
        if (sl->busy) hipEventSynchronize(sl->done);
        if (sl->stream) hipStreamDestroy(sl->stream);
        if (sl->done) hipEventDestroy(sl->done);
        hipHostFree(sl->h_data); hipHostFree(sl->h_off); hipHostFree(sl->h_len);
        hipHostFree(sl->h_ord); hipHostFree(sl->h_dig);
        hipFree(sl->d_data); hipFree(sl->d_off); hipFree(sl->d_len);
        hipFree(sl->d_ord); hipFree(sl->d_dig);
        hipHostFree(sl->h_seg); hipFree(sl->d_seg);
        free(sl->b_dst); free(sl->b_src); free(sl->b_len);
    }
    free(b->s);
    free(b);
}

int md5hip_batcher_create(int device, uint64_t slice_bytes, uint32_t nslots, md5hip_batcher **out)
{
    int rc = 0;
    if (!out) return -EINVAL;
    *out = NULL;
    /* defaults sized for MD5's serial chains: a slice of B-byte chunks keeps
     * slice/B lanes busy for B/110 MB/s (one chain), so the bytes in flight
     * must cover PCIe rate x chain time -- 4 x 128 MiB reaches the H2D rate
     * for 256 KiB blocks where 3 x 64 MiB stalls at ~34 GB/s */
    if (nslots == 0) nslots = 4;
    if (nslots > 16) return -EINVAL;
    if (slice_bytes == 0) slice_bytes = 128ull << 20;
    slice_bytes = (slice_bytes + 4095) & ~4095ull;
    if (hipSetDevice(device) != hipSuccess) return -ENODEV;
    md5hip_batcher *b = calloc(1, sizeof *b);
    if (!b) return -ENOMEM;
    b->device = device;
    b->kind = MD5HIP_DIGEST_MD5;
    b->dsz = 16;
    b->nslots = nslots;
    b->cap = slice_bytes;
    b->maxn = slice_bytes / 64 < 4096 ? 4096 : slice_bytes / 64;
    if (b->maxn > (1u << 20)) b->maxn = 1u << 20;      /* descriptors: 32 B per chunk */
    b->segcap = slice_bytes / 1024 < 4096 ? 4096 : slice_bytes / 1024;
    b->gather = MD5HIP_GATHER_AUTO;
    b->s = calloc(nslots, sizeof *b->s);
    if (!b->s) { free(b); return -ENOMEM; }
    for (uint32_t k = 0; k < nslots; k++) {
        struct slot *sl = &b->s[k];
        CK(hipStreamCreateWithFlags(&sl->stream, hipStreamNonBlocking));
        CK(hipEventCreateWithFlags(&sl->done, hipEventDisableTiming));
        CK(hipHostMalloc((void **)&sl->h_data, b->cap, hipHostMallocDefault));
        CK(hipHostMalloc((void **)&sl->h_off, 8 * b->maxn, hipHostMallocDefault));
        CK(hipHostMalloc((void **)&sl->h_len, 4 * b->maxn, hipHostMallocDefault));
        CK(hipHostMalloc((void **)&sl->h_ord, 4 * b->maxn, hipHostMallocDefault));
        CK(hipHostMalloc((void **)&sl->h_dig, 16 * b->maxn, hipHostMallocDefault));
        CK(hipMalloc((void **)&sl->d_data, b->cap));
        CK(hipMalloc((void **)&sl->d_off, 8 * b->maxn));
        CK(hipMalloc((void **)&sl->d_len, 4 * b->maxn));
        CK(hipMalloc((void **)&sl->d_ord, 4 * b->maxn));
        CK(hipMalloc((void **)&sl->d_dig, 16 * b->maxn));
        CK(hipHostMalloc((void **)&sl->h_seg, sizeof(struct md5hip_seg) * b->segcap, hipHostMallocDefault));
        CK(hipMalloc((void **)&sl->d_seg, sizeof(struct md5hip_seg) * b->segcap));
        sl->b_dst = malloc(sizeof(void *) * b->segcap);
        sl->b_src = malloc(sizeof(void *) * b->segcap);
        sl->b_len = malloc(sizeof(size_t) * b->segcap);
        if (!sl->b_dst || !sl->b_src || !sl->b_len) { rc = -ENOMEM; goto fail; }
    }
    *out = b;
    return 0;
fail:
    md5hip_batcher_destroy(b);
    return rc;
}

int md5hip_batcher_set_digest(md5hip_batcher *b, int kind, uint32_t fastcrc)
{
    if (!b) return -EINVAL;
    if (kind == MD5HIP_DIGEST_MD5) {
        if (fastcrc) return -EINVAL;
        b->dsz = 16;
    } else if (kind == MD5HIP_DIGEST_CRC32) {
        if (fastcrc & 3u) return -EINVAL;       /* cfs_apix.c:2222-2236 */
        b->dsz = 4;
    } else {
        return -EINVAL;
    }
    for (uint32_t k = 0; k < b->nslots; k++) {  /* never change kind under in-flight work */
        int rc = 0;
        struct slot *sl = &b->s[k];
        if (sl->busy && hipEventSynchronize(sl->done) != hipSuccess) rc = -EIO;
        if (rc) return rc;
    }
    b->kind = kind;
    b->fastcrc = fastcrc;
    return 0;
}

int md5hip_batcher_get_digest(const md5hip_batcher *b, int *kind, uint32_t *fastcrc)
{
    if (!b || !kind || !fastcrc) return -EINVAL;
    *kind = b->kind;
    *fastcrc = b->fastcrc;
    return 0;
}

int md5hip_batcher_set_gather(md5hip_batcher *b, int mode)
{
    if (!b || mode < MD5HIP_GATHER_HOST || mode > MD5HIP_GATHER_AUTO) return -EINVAL;
    b->gather = mode;
    return 0;
}

/* Enqueue slot `sl` holding `n` chunks, `bytes` packed bytes.  nseg == 0: the
 * bytes are in the pinned staging buffer (one H2D copy); nseg > 0: they are
 * pulled from registered host memory by the gather table (zero-copy modes). */
static int slot_launch(const md5hip_batcher *b, struct slot *sl, uint64_t n, uint64_t bytes,
                       uint64_t nseg, uint64_t ndma, unsigned char *user_dig)
{
    sl->ticket = b->ticket;
    int rc;
    const int dvar = md5hip_plan_desc(sl->h_len, n, sl->h_ord);
    if (dvar < 0) return -EINVAL;
    if (hipMemcpyAsync(sl->d_off, sl->h_off, 8 * n, hipMemcpyHostToDevice, sl->stream) ||
        hipMemcpyAsync(sl->d_len, sl->h_len, 4 * n, hipMemcpyHostToDevice, sl->stream) ||
        hipMemcpyAsync(sl->d_ord, sl->h_ord, 4 * n, hipMemcpyHostToDevice, sl->stream))
        return -EIO;
    int mode = b->gather;
    if (mode == MD5HIP_GATHER_AUTO)
        /* measured: per-copy DMA beats the PCIe-reading gather
         * kernel (~32 GB/s) once copies average more than ~192 KiB */
        mode = ndma * (256u << 10) <= bytes ? MD5HIP_GATHER_DMA : MD5HIP_GATHER_DEVICE;
    if (nseg == 0) {
        if (hipMemcpyAsync(sl->d_data, sl->h_data, bytes, hipMemcpyHostToDevice, sl->stream))
            return -EIO;
    } else if (mode == MD5HIP_GATHER_DEVICE) {
        if (hipMemcpyAsync(sl->d_seg, sl->h_seg, sizeof(struct md5hip_seg) * nseg,
                           hipMemcpyHostToDevice, sl->stream))
            return -EIO;
        if ((rc = md5hip_gather_launch(sl->d_seg, nseg, sl->d_data, sl->stream))) return rc;
    } else {
        /* one async copy per segment (hipMemcpyBatchAsync is newer than the
         * HIP runtime torch ships, which this library shares) */
        for (uint64_t q = 0; q < ndma; q++)
            if (hipMemcpyAsync(sl->b_dst[q], sl->b_src[q], sl->b_len[q], hipMemcpyHostToDevice,
                               sl->stream) != hipSuccess)
                return -EIO;
    }
    if (b->kind == MD5HIP_DIGEST_CRC32)
        rc = crc32hip_desc(sl->d_data, sl->d_off, sl->d_len, sl->d_ord, n, b->fastcrc,
                           (uint32_t *)sl->d_dig, sl->stream);
    else
        rc = md5hip_digest_desc_variant(sl->d_data, sl->d_off, sl->d_len, sl->d_ord, n, sl->d_dig,
                                        sl->stream, dvar);
    if (rc) return rc;
    if (hipMemcpyAsync(sl->h_dig, sl->d_dig, (size_t)b->dsz * n, hipMemcpyDeviceToHost, sl->stream) ||
        hipEventRecord(sl->done, sl->stream))
        return -EIO;
    sl->busy = 1;
    sl->user_dig = user_dig;
    sl->ndig = n;
    sl->dsz = b->dsz;
    return 0;
}

/* Chunk sources for the generic gather loop: a flat (ptr, len) list or an
 * iovec list with per-chunk segment ranges. */
struct chunk_src {
    const void *const *ptrs;
    const uint32_t *lens;
    const struct md5hip_iov *segs;
    const uint64_t *seg_first;
};

static uint64_t src_len(const struct chunk_src *s, uint64_t i)
{
    if (s->ptrs) return s->lens[i];
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

/* Host gather of one slice: chunks [first, first + m) into the pinned
 * staging at sl->h_off[].  One thread's memcpy from pageable memory into
 * pinned staging runs ~15 GB/s (zero-copy table), well below
 * the PCIe H2D rate, so a large slice is cut by bytes into parts copied by
 * MD5HIP_GATHER_THREADS threads (default 4; the calling thread copies the
 * first part).  Threads are started per slice: a slice worth splitting
 * (>= 8 MiB) takes milliseconds to copy, a pthread_create microseconds. */
struct gather_part {
    const struct chunk_src *src;
    uint64_t first, jlo, jhi;
    const uint64_t *off;
    unsigned char *dst;
};

static void *gather_run(void *arg)
{
    const struct gather_part *p = arg;
    for (uint64_t j = p->jlo; j < p->jhi; j++) src_copy(p->src, p->first + j, p->dst + p->off[j]);
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

#define GATHER_SPLIT_MIN (8ull << 20)   /* bytes per slice before it is split */
#define GATHER_PART_MIN (2ull << 20)    /* and at least this many bytes per part */

static void gather_slice(const struct chunk_src *src, uint64_t first, uint64_t m,
                         const uint64_t *off, unsigned char *dst, uint64_t used)
{
    pthread_once(&g_gather_once, gather_threads_init);
    uint64_t T = (uint64_t)g_gather_threads;
    if (used < GATHER_SPLIT_MIN) T = 1;
    if (T > used / GATHER_PART_MIN) T = used / GATHER_PART_MIN ? used / GATHER_PART_MIN : 1;
    if (T > m) T = m ? m : 1;
    struct gather_part part[32];
    pthread_t tid[32];
    int started[32] = {0};
    uint64_t j = 0;
    for (uint64_t t = 0; t < T; t++) {      /* part t: chunks whose offset < (t+1) * used / T */
        const uint64_t lim = t + 1 == T ? UINT64_MAX : (t + 1) * used / T;
        part[t] = (struct gather_part){src, first, j, j, off, dst};
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

/* async == 0: returns once every digest is in `digests`.  async != 0:
 * returns once the host gather is done (the caller's buffers are free again,
 * except in the zero-copy modes); *ticket names the submission for
 * md5_batch_wait / md5_batch_poll, which deliver its digests. */
static int submit_gather(md5hip_batcher *b, const struct chunk_src *src, uint64_t n,
                         unsigned char *digests, int async, uint64_t *ticket)
{
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t L = src_len(src, i);
        if (L > 0xffffffffull) return -E2BIG;
        if ((L + 15) / 16 * 16 > b->cap) return -E2BIG;
    }
    if (hipSetDevice(b->device) != hipSuccess) return -ENODEV;
    int zc = b->gather != MD5HIP_GATHER_HOST && src_registered(src, n);
    if (zc)
        for (uint64_t i = 0; i < n; i++)
            if (src_nseg(src, i) > b->segcap) zc = 0;   /* a chunk too fragmented for one table */
    const int dev = b->device < REG_MAXDEV ? b->device : 0;
    int rc = 0;
    uint32_t k = b->next;
    uint64_t i = 0;
    const uint64_t t = ++b->ticket;
    if (ticket) *ticket = t;
    while (i < n) {
        struct slot *sl = &b->s[k];
        if ((rc = slot_retire(sl))) return rc;
        uint64_t used = 0, m = 0, first = i, nseg = 0, ndma = 0;
        if (zc) pthread_rwlock_rdlock(&g_reg_lock);
        while (i < n && m < b->maxn) {
            const uint64_t L = src_len(src, i);
            const uint64_t sz = (L + 15) & ~15ull;   /* 16-B aligned packing */
            if (used + sz > b->cap) break;
            if (zc) {
                const uint64_t ns = src_nseg(src, i);
                if (nseg + ns > b->segcap) break;
                uint64_t at = used;
                for (uint64_t q = 0; q < ns; q++) {
                    const void *p;
                    uint32_t len;
                    src_seg(src, i, q, &p, &len);
                    if (!len) continue;
                    const long r = reg_find((uintptr_t)p, len);
                    const uint64_t dsrc = (uint64_t)((uintptr_t)p + g_reg[r].delta[dev]);
                    /* device table: contiguous pieces merged up to 64 KiB, so
                     * a slice keeps >= ~1000 workgroups of gather work */
                    struct md5hip_seg *prev = nseg ? &sl->h_seg[nseg - 1] : NULL;
                    if (prev && prev->src + prev->len == dsrc && prev->dst + prev->len == at &&
                        (uint64_t)prev->len + len <= (64u << 10)) {
                        prev->len += len;
                    } else {
                        sl->h_seg[nseg++] = (struct md5hip_seg){dsrc, at, len, 0};
                    }
                    /* DMA list: merged without limit (a copy has a fixed cost) */
                    if (ndma && (const unsigned char *)sl->b_src[ndma - 1] + sl->b_len[ndma - 1] ==
                                    (const unsigned char *)p &&
                        sl->b_dst[ndma - 1] == sl->d_data + at - sl->b_len[ndma - 1]) {
                        sl->b_len[ndma - 1] += len;
                    } else {
                        sl->b_dst[ndma] = sl->d_data + at;
                        sl->b_src[ndma] = (void *)p;
                        sl->b_len[ndma] = len;
                        ndma++;
                    }
                    at += len;
                }
            }
            sl->h_off[m] = used;
            sl->h_len[m] = (uint32_t)L;
            used += sz;
            m++;
            i++;
        }
        if (zc) pthread_rwlock_unlock(&g_reg_lock);
        else gather_slice(src, first, m, sl->h_off, sl->h_data, used);
        if ((rc = slot_launch(b, sl, m, used ? used : 16, zc ? nseg : 0, ndma,
                              digests + (size_t)b->dsz * first)))
            return rc;
        k = (k + 1) % b->nslots;
        b->next = k;
    }
    return async ? 0 : md5_batch_wait(b, t);
}

int md5_batch_wait(md5hip_batcher *b, uint64_t ticket)
{
    if (!b) return -EINVAL;
    int rc = 0;
    for (uint32_t j = 0; j < b->nslots; j++) {
        struct slot *sl = &b->s[j];
        if (sl->busy && sl->ticket <= ticket) {
            const int r = slot_retire(sl);
            if (r && !rc) rc = r;
        }
    }
    return rc;
}

int md5_batch_poll(md5hip_batcher *b, uint64_t ticket)
{
    if (!b) return -EINVAL;
    for (uint32_t j = 0; j < b->nslots; j++) {
        const struct slot *sl = &b->s[j];
        if (!sl->busy || sl->ticket > ticket) continue;
        const hipError_t e = hipEventQuery(sl->done);
        if (e == hipErrorNotReady) return 0;
        if (e != hipSuccess) return -EIO;
    }
    const int rc = md5_batch_wait(b, ticket);    /* all complete: deliver, no blocking */
    return rc ? rc : 1;
}

int md5_batch_submit(md5hip_batcher *b, const void *const *ptrs, const uint32_t *lens, uint64_t n,
                     unsigned char *digests)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!ptrs || !lens || !digests) return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (!ptrs[i] && lens[i]) return -EINVAL;
    const struct chunk_src src = {ptrs, lens, NULL, NULL};
    return submit_gather(b, &src, n, digests, 0, NULL);
}

int md5_batch_submit_async(md5hip_batcher *b, const void *const *ptrs, const uint32_t *lens,
                           uint64_t n, unsigned char *digests, uint64_t *ticket)
{
    if (!b || !ticket) return -EINVAL;
    *ticket = b->ticket;                   /* an empty batch is complete at once */
    if (n == 0) return 0;
    if (!ptrs || !lens || !digests) return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (!ptrs[i] && lens[i]) return -EINVAL;
    const struct chunk_src src = {ptrs, lens, NULL, NULL};
    return submit_gather(b, &src, n, digests, 1, ticket);
}

int md5_batch_submit_iov(md5hip_batcher *b, const struct md5hip_iov *segs,
                         const uint64_t *seg_first, uint64_t n, unsigned char *digests)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!segs || !seg_first || !digests || seg_first[0] != 0) return -EINVAL;
    for (uint64_t i = 0; i < n; i++) {
        if (seg_first[i + 1] < seg_first[i]) return -EINVAL;
        for (uint64_t j = seg_first[i]; j < seg_first[i + 1]; j++)
            if (!segs[j].base && segs[j].len) return -EINVAL;
    }
    const struct chunk_src src = {NULL, NULL, segs, seg_first};
    return submit_gather(b, &src, n, digests, 0, NULL);
}

int md5_batch_submit_iov_async(md5hip_batcher *b, const struct md5hip_iov *segs,
                               const uint64_t *seg_first, uint64_t n, unsigned char *digests,
                               uint64_t *ticket)
{
    if (!b || !ticket) return -EINVAL;
    *ticket = b->ticket;
    if (n == 0) return 0;
    if (!segs || !seg_first || !digests || seg_first[0] != 0) return -EINVAL;
    for (uint64_t i = 0; i < n; i++) {
        if (seg_first[i + 1] < seg_first[i]) return -EINVAL;
        for (uint64_t j = seg_first[i]; j < seg_first[i + 1]; j++)
            if (!segs[j].base && segs[j].len) return -EINVAL;
    }
    const struct chunk_src src = {NULL, NULL, segs, seg_first};
    return submit_gather(b, &src, n, digests, 1, ticket);
}

int md5hip_batch_host_fixed(md5hip_batcher *b, const void *h_base, uint64_t n, uint32_t len,
                            uint64_t stride, unsigned char *digests)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!h_base || !digests || len > stride) return -EINVAL;
    if (stride > b->cap) return -E2BIG;
    if (hipSetDevice(b->device) != hipSuccess) return -ENODEV;
    const unsigned char *src = (const unsigned char *)h_base;
    uint64_t per = b->cap / stride;
    if (per > b->maxn) per = b->maxn;
    int rc = 0;
    uint32_t k = b->next;
    const uint64_t t = ++b->ticket;
    for (uint64_t i = 0; i < n; i += per) {
        const uint64_t m = n - i < per ? n - i : per;
        struct slot *sl = &b->s[k];
        if ((rc = slot_retire(sl))) return rc;
        const uint64_t bytes = (m - 1) * stride + len;
        /* straight from the caller's (ideally pinned) buffer: no host gather */
        if (hipMemcpyAsync(sl->d_data, src + i * stride, bytes, hipMemcpyHostToDevice, sl->stream))
            return -EIO;
        if (b->kind == MD5HIP_DIGEST_CRC32)
            rc = crc32hip_fixed(sl->d_data, m, len, stride, b->fastcrc, (uint32_t *)sl->d_dig,
                                sl->stream);
        else
            rc = md5hip_digest_fixed(sl->d_data, m, len, stride, sl->d_dig, sl->stream);
        if (rc) return rc;
        if (hipMemcpyAsync(sl->h_dig, sl->d_dig, (size_t)b->dsz * m, hipMemcpyDeviceToHost, sl->stream) ||
            hipEventRecord(sl->done, sl->stream))
            return -EIO;
        sl->busy = 1;
        sl->user_dig = digests + (size_t)b->dsz * i;
        sl->ticket = t;
        sl->ndig = m;
        sl->dsz = b->dsz;
        k = (k + 1) % b->nslots;
        b->next = k;
    }
    return md5_batch_wait(b, t);
}

/* Batched verify for the cache-read / write-verify sites (blk_io.c:665-704,
 * bc_mgr.c:1464-1492): ok[i] = digest(chunk i) == expected[i]; returns the
 * number of mismatching chunks (>= 0) or -errno.  A mismatch is what
 * dm_verify_block_crc (diskcache.c:3245-3265) reports per block; the caller
 * applies its own EAGAIN / inode-reset policy per flagged block. */
int md5hip_batch_verify_iov(md5hip_batcher *b, const struct md5hip_iov *segs,
                            const uint64_t *seg_first, uint64_t n, const void *expected,
                            unsigned char *ok)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!expected || !ok) return -EINVAL;
    unsigned char *got = malloc((size_t)b->dsz * n);
    if (!got) return -ENOMEM;
    int rc = md5_batch_submit_iov(b, segs, seg_first, n, got);
    if (rc == 0) {
        const unsigned char *e = (const unsigned char *)expected;
        for (uint64_t i = 0; i < n; i++) {
            ok[i] = memcmp(got + (size_t)b->dsz * i, e + (size_t)b->dsz * i, b->dsz) == 0;
            rc += !ok[i];
        }
    }
    free(got);
    return rc;
}
