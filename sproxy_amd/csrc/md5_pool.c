/*
 * md5_pool.c -- multi-GPU host pool (include/md5hip.h).
 *
 * Chunks are independent, so a batch shards with no collective: the pool cuts
 * it into contiguous chunk ranges, one per device, and a host thread per
 * device drives that device's batcher (md5_submit.c), which writes its
 * digests straight into its own slice of the caller's digest array.  Ranges
 * are balanced by bytes (md5hip_pool_plan) because a netcache batch mixes
 * block sizes (chunk_size 4 KiB-1 MiB, httpd.c:7968) and last-block tails
 * (blk_io.c:377); fixed-length batches reduce to [g*n/G, (g+1)*n/G).
 *
 * A pool serializes its callers with a mutex, so the ASIO pool threads that
 * call blk_make_crc concurrently (asio_mgr.c:1054-1057) may share one.
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/md5hip.h"

#define POOL_MAX_DEV 64

struct md5hip_pool {
    uint32_t ndev;
    uint32_t dsz;                        /* digest bytes per chunk */
    md5hip_batcher *b[POOL_MAX_DEV];
    pthread_mutex_t lock;
};

/* Per-chunk weight for the byte balance: payload plus a fixed cost per chunk
 * (one descriptor and one padding block), so empty chunks still spread. */
static inline uint64_t chunk_weight(uint64_t len) { return len + 64; }

int md5hip_pool_plan(const uint32_t *lens, uint64_t n, uint32_t nparts, uint64_t *first)
{
    if (!first || nparts == 0) return -EINVAL;
    if (n && !lens) {                                   /* equal counts */
        for (uint32_t g = 0; g <= nparts; g++) first[g] = n * g / nparts;
        return 0;
    }
    uint64_t total = 0;
    for (uint64_t i = 0; i < n; i++) total += chunk_weight(lens[i]);
    /* part g starts at the first chunk whose prefix weight reaches g*total/G */
    first[0] = 0;
    uint64_t i = 0, acc = 0;
    for (uint32_t g = 1; g < nparts; g++) {
        const unsigned __int128 target = (unsigned __int128)total * g / nparts;
        while (i < n && acc + chunk_weight(lens[i]) / 2 < target) acc += chunk_weight(lens[i++]);
        first[g] = i;
    }
    first[nparts] = n;
    return 0;
}

void md5hip_pool_destroy(md5hip_pool *p)
{
    if (!p) return;
    for (uint32_t g = 0; g < p->ndev; g++) md5hip_batcher_destroy(p->b[g]);
    pthread_mutex_destroy(&p->lock);
    free(p);
}

int md5hip_pool_create(const int *devices, uint32_t ndev, uint64_t slice_bytes, uint32_t nslots,
                       md5hip_pool **out)
{
    if (!out) return -EINVAL;
    *out = NULL;
    if (!devices || ndev == 0 || ndev > POOL_MAX_DEV) return -EINVAL;
    md5hip_pool *p = calloc(1, sizeof *p);
    if (!p) return -ENOMEM;
    pthread_mutex_init(&p->lock, NULL);
    p->dsz = 16;
    for (uint32_t g = 0; g < ndev; g++) {
        int rc = md5hip_batcher_create(devices[g], slice_bytes, nslots, &p->b[g]);
        if (rc) {
            p->ndev = g;
            md5hip_pool_destroy(p);
            return rc;
        }
        p->ndev = g + 1;
    }
    *out = p;
    return 0;
}

int md5hip_pool_ndev(const md5hip_pool *p) { return p ? (int)p->ndev : -EINVAL; }

int md5hip_pool_set_digest(md5hip_pool *p, int kind, uint32_t fastcrc)
{
    if (!p) return -EINVAL;
    pthread_mutex_lock(&p->lock);
    int rc = 0;
    for (uint32_t g = 0; g < p->ndev && rc == 0; g++)
        rc = md5hip_batcher_set_digest(p->b[g], kind, fastcrc);
    if (rc == 0) p->dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
    pthread_mutex_unlock(&p->lock);
    return rc;
}

int md5hip_pool_set_gather(md5hip_pool *p, int mode)
{
    if (!p) return -EINVAL;
    pthread_mutex_lock(&p->lock);
    int rc = 0;
    for (uint32_t g = 0; g < p->ndev && rc == 0; g++) rc = md5hip_batcher_set_gather(p->b[g], mode);
    pthread_mutex_unlock(&p->lock);
    return rc;
}

/* One device's share of a call. */
enum job_kind { JOB_PTRS, JOB_IOV, JOB_FIXED };
struct job {
    enum job_kind kind;
    md5hip_batcher *b;
    uint64_t lo, hi;                     /* chunk range */
    const void *const *ptrs;             /* JOB_PTRS */
    const uint32_t *lens;
    const struct md5hip_iov *segs;       /* JOB_IOV */
    const uint64_t *seg_first;
    uint64_t *rebased;                   /* JOB_IOV: seg_first[lo..hi] - seg_first[lo] */
    const unsigned char *h_base;         /* JOB_FIXED */
    uint32_t len;
    uint64_t stride;
    unsigned char *digests;              /* already offset to chunk lo */
    int rc;
};

static void *job_run(void *arg)
{
    struct job *j = arg;
    const uint64_t m = j->hi - j->lo;
    if (m == 0) { j->rc = 0; return NULL; }
    switch (j->kind) {
    case JOB_PTRS:
        j->rc = md5_batch_submit(j->b, j->ptrs + j->lo, j->lens + j->lo, m, j->digests);
        break;
    case JOB_IOV:
        j->rc = md5_batch_submit_iov(j->b, j->segs + j->seg_first[j->lo], j->rebased, m, j->digests);
        break;
    case JOB_FIXED:
        j->rc = md5hip_batch_host_fixed(j->b, j->h_base + j->lo * j->stride, m, j->len, j->stride,
                                        j->digests);
        break;
    }
    return NULL;
}

/* Run jobs[0..G) -- job 0 on the calling thread, the rest on their own. */
static int run_jobs(struct job *jobs, uint32_t G)
{
    pthread_t th[POOL_MAX_DEV];
    int started[POOL_MAX_DEV] = {0};
    for (uint32_t g = 1; g < G; g++) {
        if (jobs[g].hi == jobs[g].lo) { jobs[g].rc = 0; continue; }
        if (pthread_create(&th[g], NULL, job_run, &jobs[g]) == 0) started[g] = 1;
        else job_run(&jobs[g]);          /* no thread: run it inline */
    }
    job_run(&jobs[0]);
    int rc = 0;
    for (uint32_t g = 0; g < G; g++) {
        if (g && started[g]) pthread_join(th[g], NULL);
        if (rc == 0 && jobs[g].rc) rc = jobs[g].rc;
    }
    return rc;
}

static void jobs_init(md5hip_pool *p, struct job *jobs, enum job_kind kind, const uint64_t *first,
                      unsigned char *digests)
{
    for (uint32_t g = 0; g < p->ndev; g++) {
        memset(&jobs[g], 0, sizeof jobs[g]);
        jobs[g].kind = kind;
        jobs[g].b = p->b[g];
        jobs[g].lo = first[g];
        jobs[g].hi = first[g + 1];
        jobs[g].digests = digests + (size_t)p->dsz * first[g];
    }
}

int md5hip_pool_submit(md5hip_pool *p, const void *const *ptrs, const uint32_t *lens, uint64_t n,
                       unsigned char *digests)
{
    if (!p) return -EINVAL;
    if (n == 0) return 0;
    if (!ptrs || !lens || !digests) return -EINVAL;
    for (uint64_t i = 0; i < n; i++)
        if (!ptrs[i] && lens[i]) return -EINVAL;
    uint64_t first[POOL_MAX_DEV + 1];
    struct job jobs[POOL_MAX_DEV];
    pthread_mutex_lock(&p->lock);
    md5hip_pool_plan(lens, n, p->ndev, first);
    jobs_init(p, jobs, JOB_PTRS, first, digests);
    for (uint32_t g = 0; g < p->ndev; g++) { jobs[g].ptrs = ptrs; jobs[g].lens = lens; }
    int rc = run_jobs(jobs, p->ndev);
    pthread_mutex_unlock(&p->lock);
    return rc;
}

/* (p->lock held) */
static int pool_submit_iov_locked(md5hip_pool *p, const struct md5hip_iov *segs,
                                  const uint64_t *seg_first, uint64_t n, unsigned char *digests)
{
    uint32_t *lens = malloc(4 * n);
    uint64_t *rebased = malloc(8 * (n + p->ndev));
    if (!lens || !rebased) { free(lens); free(rebased); return -ENOMEM; }
    int rc = 0;
    for (uint64_t i = 0; i < n && rc == 0; i++) {
        if (seg_first[i + 1] < seg_first[i]) { rc = -EINVAL; break; }
        uint64_t L = 0;
        for (uint64_t s = seg_first[i]; s < seg_first[i + 1]; s++) {
            if (!segs[s].base && segs[s].len) { rc = -EINVAL; break; }
            L += segs[s].len;
        }
        lens[i] = L > 0xffffffffull ? 0xffffffffu : (uint32_t)L;   /* batcher rejects it */
    }
    if (rc == 0) {
        uint64_t first[POOL_MAX_DEV + 1];
        struct job jobs[POOL_MAX_DEV];
        md5hip_pool_plan(lens, n, p->ndev, first);
        jobs_init(p, jobs, JOB_IOV, first, digests);
        /* each device sees its own seg_first[] re-based to 0 (n+G entries total) */
        uint64_t at = 0;
        for (uint32_t g = 0; g < p->ndev; g++) {
            jobs[g].segs = segs;
            jobs[g].seg_first = seg_first;
            jobs[g].rebased = rebased + at;
            for (uint64_t i = first[g]; i <= first[g + 1]; i++)
                rebased[at++] = seg_first[i] - seg_first[first[g]];
        }
        rc = run_jobs(jobs, p->ndev);
    }
    free(lens);
    free(rebased);
    return rc;
}

int md5hip_pool_submit_iov(md5hip_pool *p, const struct md5hip_iov *segs, const uint64_t *seg_first,
                           uint64_t n, unsigned char *digests)
{
    if (!p) return -EINVAL;
    if (n == 0) return 0;
    if (!segs || !seg_first || !digests || seg_first[0] != 0) return -EINVAL;
    pthread_mutex_lock(&p->lock);
    const int rc = pool_submit_iov_locked(p, segs, seg_first, n, digests);
    pthread_mutex_unlock(&p->lock);
    return rc;
}

int md5hip_pool_host_fixed(md5hip_pool *p, const void *h_base, uint64_t n, uint32_t len,
                           uint64_t stride, unsigned char *digests)
{
    if (!p) return -EINVAL;
    if (n == 0) return 0;
    if (!h_base || !digests || len > stride) return -EINVAL;
    uint64_t first[POOL_MAX_DEV + 1];
    struct job jobs[POOL_MAX_DEV];
    pthread_mutex_lock(&p->lock);
    md5hip_pool_plan(NULL, n, p->ndev, first);
    jobs_init(p, jobs, JOB_FIXED, first, digests);
    for (uint32_t g = 0; g < p->ndev; g++) {
        jobs[g].h_base = h_base;
        jobs[g].len = len;
        jobs[g].stride = stride;
    }
    int rc = run_jobs(jobs, p->ndev);
    pthread_mutex_unlock(&p->lock);
    return rc;
}

int md5hip_pool_verify_iov(md5hip_pool *p, const struct md5hip_iov *segs, const uint64_t *seg_first,
                           uint64_t n, const void *expected, unsigned char *ok)
{
    if (!p) return -EINVAL;
    if (n == 0) return 0;
    if (!expected || !ok || !segs || !seg_first || seg_first[0] != 0) return -EINVAL;
    /* the digest size is read and used under one hold of the pool lock, so a
     * concurrent md5hip_pool_set_digest cannot change it in between */
    pthread_mutex_lock(&p->lock);
    const uint32_t dsz = p->dsz;
    unsigned char *got = malloc((size_t)dsz * n);
    int rc = got ? pool_submit_iov_locked(p, segs, seg_first, n, got) : -ENOMEM;
    pthread_mutex_unlock(&p->lock);
    if (rc == 0) {
        const unsigned char *e = expected;
        for (uint64_t i = 0; i < n; i++) {
            ok[i] = memcmp(got + (size_t)dsz * i, e + (size_t)dsz * i, dsz) == 0;
            rc += !ok[i];
        }
    }
    free(got);
    return rc;
}
