/*
 * md5_pool.c -- multi-GPU host pool (include/md5hip.h): a
 * router over one coalescing batcher (md5_submit.c) per listed device.
 *
 * The reference calls its chunk checksum (blk_make_crc, blk_io.c:354) from
 * every ASIO pool thread at once, without a lock (asio_mgr.c:205,
 * :1050-1057), one vector of 64-1,024 blocks at a time, and completes the
 * vector as a unit (asio_read_vector_done_LOCK, asio_mgr.c:1414).  So the
 * pool keeps a vector whole: a submission goes to the device whose batcher
 * has the least outstanding weight, where it coalesces with the other
 * threads' vectors into that device's next launch.  Cutting a 64-block
 * vector eight ways would make eight launches, each bound by one 16 KiB
 * chunk's serial chain.  Only a submission heavier than the split threshold
 * (one batcher slice by default) is cut into contiguous byte-balanced ranges
 * (md5hip_pool_plan) over the least-loaded devices.
 *
 * Concurrency: routing reads each batcher's load lock-free and reserves the
 * submission's weight on the chosen device (`claim`) until the batcher has
 * taken the chunks, so concurrent callers spread instead of piling onto the
 * same idle device.  p->mu guards only the pool's own fields (digest kind,
 * counters, the multi-part ticket table) and is never held across a batcher
 * call that waits for the device.  No thread is created per call.
 *
 * Failed devices (md5hip_batcher_health): never routed to.  A part that
 * finds its device failed before the device took it (-ENODEV) goes to
 * another; a synchronous submission or part whose launch failed with its
 * device is resubmitted on a healthy one from the caller's buffers (still
 * valid: the call has not returned); an asynchronous ticket keeps its -EIO
 * (or -ENODEV if it was still coalescing).
 *
 * Tickets: a submission routed whole is (batcher ticket << 6) | device; a
 * split one is bit 63 | id, its parts kept in `mt` (ascending ids) until all
 * of them have completed, then dropped (an error is kept in `failed`).
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/md5hip.h"
#include "md5_internal.h"

#define POOL_MAX_DEV 64
#define MT_BIT (1ull << 63)
#define FAILED_MAX (1u << 16)

struct mt_part {
    uint32_t dev;
    uint64_t t;
};

struct mt_entry {                      /* one split submission */
    uint64_t id;
    uint32_t nparts;
    struct mt_part part[];
};

struct md5hip_pool {
    uint32_t ndev;
    md5hip_batcher *b[POOL_MAX_DEV];
    uint64_t claim[POOL_MAX_DEV];     /* weight routed to a device, not yet taken by its batcher */
    pthread_mutex_t mu;
    int kind;
    uint32_t fastcrc;
    uint64_t split_bytes;             /* 0 = one batcher slice */
    uint32_t rr;                      /* rotating start for ties */
    struct md5hip_pool_stats st;
    uint64_t st_failovers;            /* md5hip_pool_health.failovers */
    /* split tickets still running, ascending ids; [mt_lo, mt_lo + mt_n) of a ring */
    struct mt_entry **mt;
    uint64_t mt_cap, mt_lo, mt_n, mt_next;
    /* split tickets that completed with an error: (id, err), ascending */
    uint64_t *failed_id;
    int *failed_err;
    uint64_t nfailed, capfailed;
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
    for (uint64_t k = 0; k < p->mt_n; k++) free(p->mt[(p->mt_lo + k) % p->mt_cap]);
    free(p->mt);
    free(p->failed_id);
    free(p->failed_err);
    pthread_mutex_destroy(&p->mu);
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
    pthread_mutex_init(&p->mu, NULL);
    p->kind = MD5HIP_DIGEST_MD5;
    p->mt_next = 1;
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
    if (kind == MD5HIP_DIGEST_MD5 ? fastcrc != 0
        : kind == MD5HIP_DIGEST_CRC32 ? (fastcrc & 3u) != 0 : 1)   /* cfs_apix.c:2222-2236 */
        return -EINVAL;
    pthread_mutex_lock(&p->mu);
    p->kind = kind;
    p->fastcrc = fastcrc;
    pthread_mutex_unlock(&p->mu);
    return 0;
}

int md5hip_pool_set_gather(md5hip_pool *p, int mode)
{
    if (!p) return -EINVAL;
    int rc = 0;
    for (uint32_t g = 0; g < p->ndev && rc == 0; g++) rc = md5hip_batcher_set_gather(p->b[g], mode);
    return rc;
}

int md5hip_pool_set_split(md5hip_pool *p, uint64_t bytes)
{
    if (!p) return -EINVAL;
    pthread_mutex_lock(&p->mu);
    p->split_bytes = bytes;
    pthread_mutex_unlock(&p->mu);
    return 0;
}

int md5hip_pool_get_stats(md5hip_pool *p, struct md5hip_pool_stats *out)
{
    if (!p || !out) return -EINVAL;
    pthread_mutex_lock(&p->mu);
    *out = p->st;
    pthread_mutex_unlock(&p->mu);
    return 0;
}

int md5hip_pool_device_stats(md5hip_pool *p, uint32_t g, struct md5hip_batcher_stats *out)
{
    if (!p || !out || g >= p->ndev) return -EINVAL;
    return md5hip_batcher_get_stats(p->b[g], out);
}

int md5hip_pool_device_health(md5hip_pool *p, uint32_t g)
{
    if (!p || g >= p->ndev) return -EINVAL;
    return md5hip_batcher_health(p->b[g]);
}

int md5hip_pool_get_health(md5hip_pool *p, struct md5hip_pool_health *out)
{
    if (!p || !out) return -EINVAL;
    memset(out, 0, sizeof *out);
    out->ndev = p->ndev;
    for (uint32_t g = 0; g < p->ndev; g++)
        if (md5hip_batcher_health(p->b[g])) {
            out->nfailed++;
            if (g < 64) out->failed_mask |= 1ull << g;
        }
    pthread_mutex_lock(&p->mu);
    out->failovers = p->st_failovers;
    pthread_mutex_unlock(&p->mu);
    return 0;
}

int md5hip_pool_inject_fault(md5hip_pool *p, uint32_t g, uint64_t after)
{
    if (!p || g >= p->ndev) return -EINVAL;
    return md5hip_batcher_inject_fault(p->b[g], after);
}

/* ------------------------------------------------------------------------
 * Routing
 * ------------------------------------------------------------------------ */
static uint64_t dev_load(md5hip_pool *p, uint32_t g)
{
    return md5hip_batcher_load(p->b[g]) + __atomic_load_n(&p->claim[g], __ATOMIC_RELAXED);
}

static int dev_ok(md5hip_pool *p, uint32_t g) { return md5hip_batcher_health(p->b[g]) == 0; }

/* The k least-loaded healthy devices (ties from a rotating start), their
 * weight w claimed on each; into sel[0..k).  Returns how many were chosen:
 * fewer than k when fewer devices are healthy (0: every device failed). */
static uint32_t route(md5hip_pool *p, uint32_t k, const uint64_t *w, uint32_t *sel)
{
    const uint32_t G = p->ndev;
    const uint32_t r0 = __atomic_fetch_add(&p->rr, 1, __ATOMIC_RELAXED);
    uint64_t load[POOL_MAX_DEV];
    int used[POOL_MAX_DEV];
    for (uint32_t g = 0; g < G; g++) {
        used[g] = !dev_ok(p, g);                      /* a failed device is never picked */
        load[g] = dev_load(p, g);
    }
    for (uint32_t j = 0; j < k; j++) {
        uint32_t best = G;
        for (uint32_t q = 0; q < G; q++) {
            const uint32_t g = (r0 + q) % G;
            if (!used[g] && (best == G || load[g] < load[best])) best = g;
        }
        if (best == G) return j;
        used[best] = 1;
        sel[j] = best;
        __atomic_fetch_add(&p->claim[best], w[j], __ATOMIC_RELAXED);
    }
    return k;
}

static void unclaim(md5hip_pool *p, uint32_t g, uint64_t w)
{
    __atomic_fetch_sub(&p->claim[g], w, __ATOMIC_RELAXED);
}

/* ------------------------------------------------------------------------
 * Split-ticket table (p->mu held)
 * ------------------------------------------------------------------------ */
static void failed_add(md5hip_pool *p, uint64_t id, int err)
{
    if (p->nfailed == p->capfailed) {
        if (p->capfailed >= FAILED_MAX) {                 /* keep the newest half */
            const uint64_t keep = p->nfailed / 2;
            memmove(p->failed_id, p->failed_id + p->nfailed - keep, keep * sizeof *p->failed_id);
            memmove(p->failed_err, p->failed_err + p->nfailed - keep, keep * sizeof *p->failed_err);
            p->nfailed = keep;
        } else {
            const uint64_t nc = p->capfailed ? 2 * p->capfailed : 64;
            uint64_t *fi = realloc(p->failed_id, nc * sizeof *fi);
            if (fi) p->failed_id = fi;
            int *fe = realloc(p->failed_err, nc * sizeof *fe);
            if (fe) p->failed_err = fe;
            if (!fi || !fe) return;
            p->capfailed = nc;
        }
    }
    p->failed_id[p->nfailed] = id;
    p->failed_err[p->nfailed] = err;
    p->nfailed++;
}

static int failed_find(const md5hip_pool *p, uint64_t id)
{
    uint64_t a = 0, z = p->nfailed;
    while (a < z) {
        const uint64_t mid = (a + z) / 2;
        if (p->failed_id[mid] < id) a = mid + 1;
        else z = mid;
    }
    return a < p->nfailed && p->failed_id[a] == id ? p->failed_err[a] : 0;
}

/* 1 = every part done (*err = the first part error), 0 = running */
static int mt_state(md5hip_pool *p, const struct mt_entry *e, int *err)
{
    *err = 0;
    for (uint32_t j = 0; j < e->nparts; j++) {
        int pe = 0;
        const int s = md5hip_batcher_ticket_state(p->b[e->part[j].dev], e->part[j].t, &pe);
        if (s < 0) pe = s;
        else if (s == 0) return 0;
        if (pe && !*err) *err = pe;
    }
    return 1;
}

/* Drop completed entries from the low end (they are looked up by failed_find
 * from then on). */
static void mt_reap(md5hip_pool *p)
{
    while (p->mt_n) {
        struct mt_entry *e = p->mt[p->mt_lo % p->mt_cap];
        int err;
        if (!mt_state(p, e, &err)) break;
        if (err) failed_add(p, e->id, err);
        free(e);
        p->mt_lo++;
        p->mt_n--;
    }
}

static int mt_push(md5hip_pool *p, struct mt_entry *e)
{
    if (p->mt_n == p->mt_cap) {
        const uint64_t nc = p->mt_cap ? 2 * p->mt_cap : 64;
        struct mt_entry **m = malloc(nc * sizeof *m);
        if (!m) return -ENOMEM;
        for (uint64_t k = 0; k < p->mt_n; k++) m[k] = p->mt[(p->mt_lo + k) % p->mt_cap];
        free(p->mt);
        p->mt = m;
        p->mt_cap = nc;
        p->mt_lo = 0;
    }
    p->mt[(p->mt_lo + p->mt_n) % p->mt_cap] = e;
    p->mt_n++;
    return 0;
}

/* the live entry with this id, or NULL (completed and dropped, or unknown) */
static struct mt_entry *mt_find(md5hip_pool *p, uint64_t id)
{
    uint64_t a = 0, z = p->mt_n;
    while (a < z) {
        const uint64_t mid = (a + z) / 2;
        if (p->mt[(p->mt_lo + mid) % p->mt_cap]->id < id) a = mid + 1;
        else z = mid;
    }
    if (a < p->mt_n) {
        struct mt_entry *e = p->mt[(p->mt_lo + a) % p->mt_cap];
        if (e->id == id) return e;
    }
    return NULL;
}

/* ------------------------------------------------------------------------
 * Submission
 * ------------------------------------------------------------------------ */
enum src_kind { SRC_PTRS, SRC_IOV, SRC_FIXED };
struct pool_src {
    enum src_kind kind;
    const void *const *ptrs;             /* SRC_PTRS */
    const uint32_t *lens;
    const struct md5hip_iov *segs;       /* SRC_IOV */
    const uint64_t *seg_first;
    const unsigned char *h_base;         /* SRC_FIXED */
    uint32_t len;
    uint64_t stride;
};

/* chunks [lo, hi) of `s` to device g's batcher, asynchronously; urgent =
 * the caller waits right away (launch at once, as a synchronous call) */
static int part_submit(md5hip_pool *p, uint32_t g, int kind, uint32_t fastcrc,
                       const struct pool_src *s, uint64_t lo, uint64_t hi, unsigned char *digests,
                       uint64_t *ticket, int urgent)
{
    const uint64_t m = hi - lo;
    switch (s->kind) {
    case SRC_PTRS:
        return md5hip_submit_as(p->b[g], kind, fastcrc, s->ptrs + lo, s->lens + lo, NULL, NULL, m,
                                digests, ticket, urgent);
    case SRC_IOV: {
        /* the batcher reads seg_first[0..m] re-based to 0; it has taken the
         * chunks when the call returns, so a temporary copy will do */
        uint64_t local[65];
        uint64_t *sf = m + 1 <= 65 ? local : malloc(8 * (m + 1));
        if (!sf) return -ENOMEM;
        for (uint64_t i = 0; i <= m; i++) sf[i] = s->seg_first[lo + i] - s->seg_first[lo];
        const int rc = md5hip_submit_as(p->b[g], kind, fastcrc, NULL, NULL, s->segs + s->seg_first[lo],
                                        sf, m, digests, ticket, urgent);
        if (sf != local) free(sf);
        return rc;
    }
    case SRC_FIXED:
        return md5hip_host_fixed_as(p->b[g], kind, fastcrc, s->h_base + lo * s->stride, m, s->len,
                                    s->stride, digests, ticket);
    }
    return -EINVAL;
}

static uint64_t src_weight(const struct pool_src *s, uint64_t i)
{
    if (s->kind == SRC_PTRS) return chunk_weight(s->lens[i]);
    if (s->kind == SRC_FIXED) return chunk_weight(s->len);
    uint64_t L = 0;
    for (uint64_t j = s->seg_first[i]; j < s->seg_first[i + 1]; j++) L += s->segs[j].len;
    return chunk_weight(L);
}

static void count_failover(md5hip_pool *p)
{
    pthread_mutex_lock(&p->mu);
    p->st_failovers++;
    pthread_mutex_unlock(&p->mu);
}

/* Chunks [lo, hi) whole to one healthy device (weight w): *g, *t its device
 * and ticket.  sync: waited here, and resubmitted elsewhere while the launch
 * failed because its device did (the caller's buffers are still valid).
 * Either way a device that failed before taking the chunks (-ENODEV) is
 * left for another.  -ENODEV once no device is healthy. */
static int submit_range(md5hip_pool *p, int kind, uint32_t fastcrc, const struct pool_src *s,
                        uint64_t lo, uint64_t hi, uint64_t w, unsigned char *digests, int sync,
                        uint32_t *g_out, uint64_t *t_out)
{
    for (;;) {
        uint32_t g;
        if (!route(p, 1, &w, &g)) return -ENODEV;     /* every device failed */
        /* asynchronous even for a synchronous caller, so the claim ends as
         * soon as the batcher holds the chunks (its own load counts them) */
        uint64_t t = 0;
        int rc = part_submit(p, g, kind, fastcrc, s, lo, hi, digests, &t, sync);
        unclaim(p, g, w);
        if (rc == 0 && sync) rc = md5_batch_wait(p->b[g], t);
        if ((rc == -ENODEV || (sync && rc == -EIO)) && !dev_ok(p, g)) {
            count_failover(p);                        /* moved off the failed device */
            continue;
        }
        *g_out = g;
        *t_out = t;
        return rc;
    }
}

/* ticket NULL = synchronous; kind < 0 = the pool's current digest kind */
static int pool_submit(md5hip_pool *p, const struct pool_src *s, uint64_t n, unsigned char *digests,
                       uint64_t *ticket, int kind, uint32_t fastcrc)
{
    if (ticket) *ticket = 0;
    if (n == 0) return 0;
    pthread_mutex_lock(&p->mu);
    if (kind < 0) {
        kind = p->kind;
        fastcrc = p->fastcrc;
    }
    uint64_t split = p->split_bytes;
    p->st.submissions++;
    pthread_mutex_unlock(&p->mu);
    if (split == 0) split = md5hip_batcher_slice(p->b[0]);
    const uint32_t dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
    const int sync = ticket == NULL;
    uint64_t total = 0;
    if (s->kind == SRC_FIXED) {
        total = n * chunk_weight(s->len);
    } else {
        for (uint64_t i = 0; i < n; i++) total += src_weight(s, i);
    }
    uint32_t healthy = 0;
    for (uint32_t g = 0; g < p->ndev; g++) healthy += dev_ok(p, g);
    if (healthy == 0) return -ENODEV;
    uint32_t k = 1;
    if (total > split && healthy > 1) {
        const uint64_t want = (total + split - 1) / split;
        k = want < healthy ? (uint32_t)want : healthy;
        if (k > n) k = (uint32_t)n;
    }
    if (k == 1) {                                     /* the common case: whole */
        uint32_t g = 0;
        uint64_t t = 0;
        const int rc = submit_range(p, kind, fastcrc, s, 0, n, total, digests, sync, &g, &t);
        pthread_mutex_lock(&p->mu);
        p->st.routed_whole++;
        p->st.parts++;
        pthread_mutex_unlock(&p->mu);
        if (ticket && rc == 0 && t) *ticket = (t << 6) | g;
        return rc;
    }
    /* split: contiguous byte-balanced ranges over the k least-loaded devices */
    uint64_t first[POOL_MAX_DEV + 1], w[POOL_MAX_DEV];
    if (s->kind == SRC_FIXED) {
        md5hip_pool_plan(NULL, n, k, first);
    } else {
        uint32_t *lens = malloc(4 * n);
        if (!lens) return -ENOMEM;
        for (uint64_t i = 0; i < n; i++) {
            const uint64_t L = src_weight(s, i) - 64;
            lens[i] = L > 0xffffffffull ? 0xffffffffu : (uint32_t)L;   /* the batcher rejects it */
        }
        md5hip_pool_plan(lens, n, k, first);
        free(lens);
    }
    for (uint32_t j = 0; j < k; j++) {
        w[j] = 0;
        if (s->kind == SRC_FIXED) w[j] = (first[j + 1] - first[j]) * chunk_weight(s->len);
        else for (uint64_t i = first[j]; i < first[j + 1]; i++) w[j] += src_weight(s, i);
    }
    uint32_t sel[POOL_MAX_DEV];
    const uint32_t got = route(p, k, w, sel);         /* < k: a device failed since the count */
    struct mt_entry *e = malloc(sizeof *e + k * sizeof(struct mt_part));
    int rc = e ? 0 : -ENOMEM;
    uint32_t np = 0;
    uint32_t pj[POOL_MAX_DEV];                        /* part index of each submitted part */
    for (uint32_t j = 0; j < k; j++) {
        if (rc == 0 && first[j + 1] > first[j]) {
            uint64_t t = 0;
            uint32_t g = j < got ? sel[j] : 0;
            int r = j < got ? part_submit(p, g, kind, fastcrc, s, first[j], first[j + 1],
                                          digests + (size_t)dsz * first[j], &t, sync)
                            : -ENODEV;
            if (r == -ENODEV && (j >= got || !dev_ok(p, g))) {
                if (j < got) count_failover(p);
                /* its device failed before taking the part: any healthy one
                 * (submitted asynchronously like the others; waited below) */
                r = submit_range(p, kind, fastcrc, s, first[j], first[j + 1], w[j],
                                 digests + (size_t)dsz * first[j], 0, &g, &t);
            }
            rc = r;
            if (rc == 0 && t) {
                pj[np] = j;
                e->part[np++] = (struct mt_part){g, t};
            }
        }
        if (j < got) unclaim(p, sel[j], w[j]);
    }
    pthread_mutex_lock(&p->mu);
    p->st.split++;
    p->st.parts += np;
    pthread_mutex_unlock(&p->mu);
    if (!e) return rc;
    e->nparts = np;
    if (rc || sync) {
        /* synchronous, or a part failed: the submitted parts finish before
         * the caller may reuse its buffers.  Synchronously, a part whose
         * launch failed with its device goes again on a healthy one. */
        for (uint32_t q = 0; q < np; q++) {
            int r = md5_batch_wait(p->b[e->part[q].dev], e->part[q].t);
            if (sync && rc == 0 && (r == -EIO || r == -ENODEV) && !dev_ok(p, e->part[q].dev)) {
                const uint32_t j = pj[q];
                uint32_t g;
                uint64_t t;
                count_failover(p);
                r = submit_range(p, kind, fastcrc, s, first[j], first[j + 1], w[j],
                                 digests + (size_t)dsz * first[j], 1, &g, &t);
            }
            if (r && !rc) rc = r;
        }
        free(e);
        return rc;
    }
    pthread_mutex_lock(&p->mu);
    mt_reap(p);
    e->id = p->mt_next++;
    rc = mt_push(p, e);
    if (rc == 0) *ticket = MT_BIT | e->id;
    pthread_mutex_unlock(&p->mu);
    if (rc) {                                         /* no table space: finish it here */
        for (uint32_t j = 0; j < np; j++) (void)md5_batch_wait(p->b[e->part[j].dev], e->part[j].t);
        free(e);
    }
    return rc;
}

/* wait (block = 1) or poll (block = 0) on a pool ticket: 1 done / 0 running
 * and *err its error, or -EINVAL */
static int pool_ticket(md5hip_pool *p, uint64_t ticket, int block, int *err)
{
    *err = 0;
    if (ticket == 0) return 1;
    if (!(ticket & MT_BIT)) {
        const uint32_t g = (uint32_t)(ticket & 63u);
        if (g >= p->ndev) return -EINVAL;
        const int r = block ? md5_batch_wait(p->b[g], ticket >> 6) : md5_batch_poll(p->b[g], ticket >> 6);
        if (r == -EINVAL) return -EINVAL;
        if (block) { *err = r; return 1; }
        if (r < 0) { *err = r; return 1; }
        return r;                                     /* 1 done, 0 running */
    }
    const uint64_t id = ticket & ~MT_BIT;
    pthread_mutex_lock(&p->mu);
    if (id == 0 || id >= p->mt_next) {
        pthread_mutex_unlock(&p->mu);
        return -EINVAL;
    }
    struct mt_entry *e = mt_find(p, id);
    if (!e) {                                         /* completed and dropped */
        *err = failed_find(p, id);
        pthread_mutex_unlock(&p->mu);
        return 1;
    }
    struct mt_part parts[POOL_MAX_DEV];
    const uint32_t np = e->nparts;
    memcpy(parts, e->part, np * sizeof *parts);
    pthread_mutex_unlock(&p->mu);
    /* the batcher calls below may block: p->mu is not held */
    int done = 1;
    for (uint32_t j = 0; j < np; j++) {
        const int r = block ? md5_batch_wait(p->b[parts[j].dev], parts[j].t)
                            : md5_batch_poll(p->b[parts[j].dev], parts[j].t);
        if (block) {
            if (r && !*err) *err = r;
        } else if (r < 0) {
            if (!*err) *err = r;
        } else if (r == 0) {
            done = 0;                                 /* keep polling: every part is hastened */
        }
    }
    if (done) {
        pthread_mutex_lock(&p->mu);
        mt_reap(p);
        pthread_mutex_unlock(&p->mu);
    }
    return done;
}

int md5hip_pool_wait(md5hip_pool *p, uint64_t ticket)
{
    if (!p) return -EINVAL;
    int err;
    const int r = pool_ticket(p, ticket, 1, &err);
    return r < 0 ? r : err;
}

int md5hip_pool_poll(md5hip_pool *p, uint64_t ticket)
{
    if (!p) return -EINVAL;
    int err;
    const int r = pool_ticket(p, ticket, 0, &err);
    if (r < 0) return r;
    return r == 1 && err ? err : r;
}

/* ------------------------------------------------------------------------
 * Entries
 * ------------------------------------------------------------------------ */
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

int md5hip_pool_submit_async(md5hip_pool *p, const void *const *ptrs, const uint32_t *lens,
                             uint64_t n, unsigned char *digests, uint64_t *ticket)
{
    if (!p || !ticket) return -EINVAL;
    *ticket = 0;
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = check_ptrs(ptrs, lens, n);
    if (rc) return rc;
    const struct pool_src s = {SRC_PTRS, ptrs, lens, NULL, NULL, NULL, 0, 0};
    return pool_submit(p, &s, n, digests, ticket, -1, 0);
}

int md5hip_pool_submit_iov_async(md5hip_pool *p, const struct md5hip_iov *segs,
                                 const uint64_t *seg_first, uint64_t n, unsigned char *digests,
                                 uint64_t *ticket)
{
    if (!p || !ticket) return -EINVAL;
    *ticket = 0;
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = check_iov(segs, seg_first, n);
    if (rc) return rc;
    const struct pool_src s = {SRC_IOV, NULL, NULL, segs, seg_first, NULL, 0, 0};
    return pool_submit(p, &s, n, digests, ticket, -1, 0);
}

int md5hip_pool_submit(md5hip_pool *p, const void *const *ptrs, const uint32_t *lens, uint64_t n,
                       unsigned char *digests)
{
    if (!p) return -EINVAL;
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = check_ptrs(ptrs, lens, n);
    if (rc) return rc;
    const struct pool_src s = {SRC_PTRS, ptrs, lens, NULL, NULL, NULL, 0, 0};
    return pool_submit(p, &s, n, digests, NULL, -1, 0);
}

int md5hip_pool_submit_iov(md5hip_pool *p, const struct md5hip_iov *segs, const uint64_t *seg_first,
                           uint64_t n, unsigned char *digests)
{
    if (!p) return -EINVAL;
    if (n == 0) return 0;
    if (!digests) return -EINVAL;
    int rc = check_iov(segs, seg_first, n);
    if (rc) return rc;
    const struct pool_src s = {SRC_IOV, NULL, NULL, segs, seg_first, NULL, 0, 0};
    return pool_submit(p, &s, n, digests, NULL, -1, 0);
}

int md5hip_pool_host_fixed(md5hip_pool *p, const void *h_base, uint64_t n, uint32_t len,
                           uint64_t stride, unsigned char *digests)
{
    if (!p) return -EINVAL;
    if (n == 0) return 0;
    if (!h_base || !digests || len > stride) return -EINVAL;
    const struct pool_src s = {SRC_FIXED, NULL, NULL, NULL, NULL, h_base, len, stride};
    return pool_submit(p, &s, n, digests, NULL, -1, 0);
}

int md5hip_pool_verify_iov(md5hip_pool *p, const struct md5hip_iov *segs, const uint64_t *seg_first,
                           uint64_t n, const void *expected, unsigned char *ok)
{
    if (!p) return -EINVAL;
    if (n == 0) return 0;
    if (!expected || !ok) return -EINVAL;
    int rc = check_iov(segs, seg_first, n);
    if (rc) return rc;
    /* one snapshot of the kind for the digest size and the submission */
    pthread_mutex_lock(&p->mu);
    const int kind = p->kind;
    const uint32_t fastcrc = p->fastcrc;
    pthread_mutex_unlock(&p->mu);
    const uint32_t dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
    unsigned char *got = malloc((size_t)dsz * n);
    if (!got) return -ENOMEM;
    const struct pool_src s = {SRC_IOV, NULL, NULL, segs, seg_first, NULL, 0, 0};
    rc = pool_submit(p, &s, n, got, NULL, kind, fastcrc);
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
