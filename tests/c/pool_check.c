/*
 * pool_check.c -- the multi-GPU pool's host logic (sproxy_amd/csrc/md5_pool.c:
 * routing, claims, whole and split submissions, split-ticket table, error
 * bookkeeping, stats) driven on the host with NO device: the batcher entries
 * the pool calls are replaced by a fake defined here, which hashes on the CPU
 * with the library's own host MD5 (md5_stream.c) / CRC-32 (nc_digest.c) and
 * completes a ticket only after a few polls, failing every 9th submission
 * with -EIO when asked to, and losing a device on request
 * (md5hip_batcher_inject_fault: that submission completes with -EIO and
 * garbage digests, the batcher reports -ENODEV from then on and refuses
 * every submission with it).  Built with ASan+UBSan and with TSan by
 * tests/test_pool_host.py.  Exits 0 when every check holds, else prints the
 * failing check.
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "md5.h"
#include "md5hip.h"
#include "nc_digest.h"
#include "../../sproxy_amd/csrc/md5_internal.h"

#define CHECK(c, ...)                                                        \
    do {                                                                     \
        if (!(c)) {                                                          \
            printf("FAIL line %d: %s: ", __LINE__, #c);                      \
            printf(__VA_ARGS__);                                             \
            printf("\n");                                                    \
            exit(1);                                                         \
        }                                                                    \
    } while (0)

/* ------------------------------------------------------------------ fake batcher */
struct fake_ticket {
    int polls_left, err;
};

struct md5hip_batcher {
    pthread_mutex_t mu;
    struct fake_ticket *tk;
    uint64_t ntk, captk;
    uint64_t load;                 /* weight of tickets not yet completed */
    uint64_t *tk_weight;
    uint64_t submissions, launches;
    int device;
    int lost;                      /* -ENODEV once "lost" (read lock-free: atomic) */
    uint64_t lose_in;              /* the lose_in-th submission from now fails and loses the device */
};

int md5hip_batcher_health(const md5hip_batcher *b) { return __atomic_load_n(&b->lost, __ATOMIC_ACQUIRE); }

int md5hip_batcher_inject_fault(md5hip_batcher *b, uint64_t after)
{
    pthread_mutex_lock(&b->mu);
    const int rc = b->lost;
    if (!rc) b->lose_in = after;
    pthread_mutex_unlock(&b->mu);
    return rc;
}

static int g_fail_every = 0;       /* every n-th submission (process-wide) fails */
static uint64_t g_submit_count = 0;
static pthread_mutex_t g_count_mu = PTHREAD_MUTEX_INITIALIZER;

int md5hip_batcher_create(int device, uint64_t slice_bytes, uint32_t nslots, md5hip_batcher **out)
{
    (void)slice_bytes;
    (void)nslots;
    md5hip_batcher *b = calloc(1, sizeof *b);
    if (!b) return -ENOMEM;
    pthread_mutex_init(&b->mu, NULL);
    b->device = device;
    *out = b;
    return 0;
}

void md5hip_batcher_destroy(md5hip_batcher *b)
{
    if (!b) return;
    free(b->tk);
    free(b->tk_weight);
    pthread_mutex_destroy(&b->mu);
    free(b);
}

int md5hip_batcher_set_gather(md5hip_batcher *b, int mode) { return b && mode >= 0 && mode <= 3 ? 0 : -EINVAL; }

int md5hip_batcher_get_stats(md5hip_batcher *b, struct md5hip_batcher_stats *out)
{
    pthread_mutex_lock(&b->mu);
    memset(out, 0, sizeof *out);
    out->submissions = b->submissions;
    out->launches = b->launches;
    pthread_mutex_unlock(&b->mu);
    return 0;
}

uint64_t md5hip_batcher_load(const md5hip_batcher *b) { return __atomic_load_n(&b->load, __ATOMIC_RELAXED); }
uint64_t md5hip_batcher_slice(const md5hip_batcher *b) { (void)b; return 1u << 20; }

static void digest_one(int kind, const struct md5hip_iov *segs, uint64_t nseg, unsigned char *out)
{
    if (kind == MD5HIP_DIGEST_CRC32) {
        uint64_t L = 0;
        for (uint64_t k = 0; k < nseg; k++) L += segs[k].len;
        unsigned char *tmp = malloc(L ? L : 1);
        uint64_t at = 0;
        for (uint64_t k = 0; k < nseg; k++) {
            if (segs[k].len) memcpy(tmp + at, segs[k].base, segs[k].len);
            at += segs[k].len;
        }
        const uint32_t c = nc_crc32(tmp, L);
        memcpy(out, &c, 4);
        free(tmp);
        return;
    }
    struct MD5Context ctx;
    MD5Init(&ctx);
    for (uint64_t k = 0; k < nseg; k++) MD5Update(&ctx, segs[k].base, segs[k].len);
    MD5Final(out, &ctx);
}

/* a new fake ticket: digests are written now, the ticket completes later */
static int fake_submit(md5hip_batcher *b, int kind, uint64_t weight, uint64_t *ticket, int *failed)
{
    pthread_mutex_lock(&g_count_mu);
    const uint64_t c = ++g_submit_count;
    pthread_mutex_unlock(&g_count_mu);
    *failed = g_fail_every && c % (uint64_t)g_fail_every == 0;
    (void)kind;
    pthread_mutex_lock(&b->mu);
    if (b->lose_in && --b->lose_in == 0) {          /* this launch faults: the device is gone */
        *failed = 1;
        __atomic_store_n(&b->lost, -ENODEV, __ATOMIC_RELEASE);
    }
    if (b->ntk == b->captk) {
        b->captk = b->captk ? 2 * b->captk : 64;
        b->tk = realloc(b->tk, b->captk * sizeof *b->tk);
        b->tk_weight = realloc(b->tk_weight, b->captk * sizeof *b->tk_weight);
    }
    const uint64_t id = ++b->ntk;                       /* ids from 1 */
    b->tk[id - 1] = (struct fake_ticket){1 + (int)(id % 3), *failed ? -EIO : 0};
    b->tk_weight[id - 1] = weight;
    __atomic_fetch_add(&b->load, weight, __ATOMIC_RELAXED);
    b->submissions++;
    b->launches++;
    pthread_mutex_unlock(&b->mu);
    *ticket = id;
    return 0;
}

static int fake_state(md5hip_batcher *b, uint64_t t, int advance, int *err)
{
    pthread_mutex_lock(&b->mu);
    if (t == 0 || t > b->ntk) {
        pthread_mutex_unlock(&b->mu);
        return -EINVAL;
    }
    struct fake_ticket *k = &b->tk[t - 1];
    if (advance && k->polls_left > 0 && --k->polls_left == 0)
        __atomic_fetch_sub(&b->load, b->tk_weight[t - 1], __ATOMIC_RELAXED);
    const int done = k->polls_left == 0;
    *err = done ? k->err : 0;
    pthread_mutex_unlock(&b->mu);
    return done;
}

int md5hip_submit_as(md5hip_batcher *b, int kind, uint32_t fastcrc, const void *const *ptrs,
                     const uint32_t *lens, const struct md5hip_iov *segs, const uint64_t *seg_first,
                     uint64_t n, unsigned char *digests, uint64_t *ticket, int urgent)
{
    (void)fastcrc;
    (void)urgent;
    if (ticket) *ticket = 0;
    if (n == 0) return 0;
    if (md5hip_batcher_health(b)) return -ENODEV;
    const uint32_t dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
    uint64_t weight = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (ptrs) {
            const struct md5hip_iov one = {ptrs[i], lens[i]};
            digest_one(kind, &one, 1, digests + (size_t)dsz * i);
            weight += (uint64_t)lens[i] + 64;
        } else {
            digest_one(kind, segs + seg_first[i], seg_first[i + 1] - seg_first[i], digests + (size_t)dsz * i);
            for (uint64_t k = seg_first[i]; k < seg_first[i + 1]; k++) weight += segs[k].len;
            weight += 64;
        }
    }
    uint64_t t;
    int failed;
    fake_submit(b, kind, weight, &t, &failed);
    if (failed) memset(digests, 0xAA, (size_t)dsz * n);  /* what a failed launch leaves */
    if (!ticket) {                                      /* synchronous */
        int err = 0;
        while (!fake_state(b, t, 1, &err)) {}
        return err;
    }
    *ticket = t;
    return 0;
}

int md5hip_host_fixed_as(md5hip_batcher *b, int kind, uint32_t fastcrc, const void *h_base, uint64_t n,
                         uint32_t len, uint64_t stride, unsigned char *digests, uint64_t *ticket)
{
    (void)fastcrc;
    if (ticket) *ticket = 0;
    if (md5hip_batcher_health(b)) return -ENODEV;
    const uint32_t dsz = kind == MD5HIP_DIGEST_CRC32 ? 4 : 16;
    for (uint64_t i = 0; i < n; i++) {
        const struct md5hip_iov one = {(const unsigned char *)h_base + i * stride, len};
        digest_one(kind, &one, 1, digests + (size_t)dsz * i);
    }
    uint64_t t;
    int failed;
    fake_submit(b, kind, n * ((uint64_t)len + 64), &t, &failed);
    if (failed) memset(digests, 0xAA, (size_t)dsz * n);
    if (!ticket) {
        int err = 0;
        while (!fake_state(b, t, 1, &err)) {}
        return err;
    }
    *ticket = t;
    return 0;
}

int md5hip_batcher_ticket_state(md5hip_batcher *b, uint64_t ticket, int *err)
{
    *err = 0;
    if (ticket == 0) return 1;
    return fake_state(b, ticket, 0, err);
}

int md5_batch_wait(md5hip_batcher *b, uint64_t ticket)
{
    if (ticket == 0) return 0;
    int err = 0, r;
    while ((r = fake_state(b, ticket, 1, &err)) == 0) {}
    return r < 0 ? r : err;
}

int md5_batch_poll(md5hip_batcher *b, uint64_t ticket)
{
    if (ticket == 0) return 1;
    int err = 0;
    const int r = fake_state(b, ticket, 1, &err);
    if (r < 0) return r;
    return r == 1 && err ? err : r;
}

/* ------------------------------------------------------------------ checks */
static unsigned char *g_blob;
static uint32_t g_lens[2000];
static uint64_t g_offs[2000];
static unsigned char g_want[2000][16];
static uint32_t g_want_crc[2000];

static void make_data(void)
{
    uint64_t total = 0;
    uint64_t s = 0x1234567;
    for (int i = 0; i < 2000; i++) {
        s ^= s << 13; s ^= s >> 7; s ^= s << 17;
        g_lens[i] = (uint32_t)(s % 20000u);
        if (i % 50 == 0) g_lens[i] = 0;
        g_offs[i] = total;
        total += g_lens[i];
    }
    g_blob = malloc(total + 1);
    for (uint64_t k = 0; k < total; k++) g_blob[k] = (unsigned char)(k * 2654435761u >> 24);
    for (int i = 0; i < 2000; i++) {
        struct MD5Context ctx;
        MD5Init(&ctx);
        MD5Update(&ctx, g_blob + g_offs[i], g_lens[i]);
        MD5Final(g_want[i], &ctx);
        g_want_crc[i] = nc_crc32(g_blob + g_offs[i], g_lens[i]);
    }
}

struct job {
    md5hip_pool *p;
    int t, reps, bad, rc_bad;
};

static void *thread_main(void *arg)
{
    struct job *j = arg;
    const void *ptrs[400];
    unsigned char dig[6][400][16];
    uint64_t tk[6];
    int lo[6], cnt[6];
    for (int r = 0; r < j->reps; r++) {
        for (int v = 0; v < 6; v++) {
            lo[v] = (j->t * 97 + r * 31 + v * 211) % 1600;
            cnt[v] = 1 + (j->t * 7 + r * 13 + v * 29) % 399;
            for (int i = 0; i < cnt[v]; i++) ptrs[i] = g_blob + g_offs[lo[v] + i];
            if (md5hip_pool_submit_async(j->p, ptrs, g_lens + lo[v], (uint64_t)cnt[v], &dig[v][0][0], &tk[v]))
                j->rc_bad++;
        }
        for (int v = 5; v >= 0; v--) {
            if (v % 2) {
                int pr;
                while ((pr = md5hip_pool_poll(j->p, tk[v])) == 0) {}
                if (pr != 1) j->rc_bad++;
            }
            if (md5hip_pool_wait(j->p, tk[v]) != 0) j->rc_bad++;
            for (int i = 0; i < cnt[v]; i++) j->bad += memcmp(dig[v][i], g_want[lo[v] + i], 16) != 0;
        }
    }
    return NULL;
}

int main(void)
{
    make_data();
    const int devs[4] = {0, 1, 2, 3};
    md5hip_pool *p = NULL;
    CHECK(md5hip_pool_create(devs, 4, 0, 0, &p) == 0 && p, "create");
    CHECK(md5hip_pool_ndev(p) == 4, "ndev");
    const void *ptrs[2000];
    for (int i = 0; i < 2000; i++) ptrs[i] = g_blob + g_offs[i];
    static unsigned char dig[2000][16];

    /* whole: a small vector goes to one device; synchronous result exact */
    CHECK(md5hip_pool_submit(p, ptrs, g_lens, 20, &dig[0][0]) == 0, "submit small");
    for (int i = 0; i < 20; i++) CHECK(memcmp(dig[i], g_want[i], 16) == 0, "small %d", i);
    struct md5hip_pool_stats st;
    md5hip_pool_get_stats(p, &st);
    CHECK(st.routed_whole == 1 && st.split == 0 && st.parts == 1, "stats whole %llu", (unsigned long long)st.routed_whole);

    /* split: 2000 chunks (~20 MB) over 4 devices at a 1 MiB slice; digests in place */
    memset(dig, 0, sizeof dig);
    uint64_t t;
    CHECK(md5hip_pool_submit_async(p, ptrs, g_lens, 2000, &dig[0][0], &t) == 0, "split async");
    CHECK(t >> 63, "split ticket has bit 63");
    int pr;
    while ((pr = md5hip_pool_poll(p, t)) == 0) {}
    CHECK(pr == 1, "split poll = %d", pr);
    CHECK(md5hip_pool_wait(p, t) == 0, "split wait");
    CHECK(md5hip_pool_wait(p, t) == 0, "split wait twice");
    for (int i = 0; i < 2000; i++) CHECK(memcmp(dig[i], g_want[i], 16) == 0, "split %d", i);
    md5hip_pool_get_stats(p, &st);
    CHECK(st.split == 1 && st.parts == 5, "stats split %llu parts %llu", (unsigned long long)st.split,
          (unsigned long long)st.parts);
    for (uint32_t g = 0; g < 4; g++) {
        struct md5hip_batcher_stats bs;
        CHECK(md5hip_pool_device_stats(p, g, &bs) == 0 && bs.submissions >= 1, "device %u took a part", g);
    }

    /* iov and CRC-32 through the pool, split */
    static struct md5hip_iov segs[4000];
    static uint64_t first[2001];
    uint64_t ns = 0;
    for (int i = 0; i < 2000; i++) {
        first[i] = ns;
        const uint32_t h = g_lens[i] / 2;
        segs[ns++] = (struct md5hip_iov){g_blob + g_offs[i], h};
        segs[ns++] = (struct md5hip_iov){g_blob + g_offs[i] + h, g_lens[i] - h};
    }
    first[2000] = ns;
    CHECK(md5hip_pool_set_digest(p, MD5HIP_DIGEST_CRC32, 0) == 0, "set crc");
    static uint32_t crc[2000];
    CHECK(md5hip_pool_submit_iov(p, segs, first, 2000, (unsigned char *)crc) == 0, "iov crc");
    for (int i = 0; i < 2000; i++) CHECK(crc[i] == g_want_crc[i], "crc %d", i);
    CHECK(md5hip_pool_set_digest(p, MD5HIP_DIGEST_MD5, 0) == 0, "set md5");
    CHECK(md5hip_pool_set_digest(p, MD5HIP_DIGEST_MD5, 4) == -EINVAL, "md5 takes no window");
    CHECK(md5hip_pool_set_digest(p, MD5HIP_DIGEST_CRC32, 6) == -EINVAL, "window multiple of 4");
    unsigned char ok[2000];
    memcpy(dig, g_want, sizeof dig);
    dig[1234][3] ^= 1;
    CHECK(md5hip_pool_verify_iov(p, segs, first, 2000, dig, ok) == 1 && !ok[1234] && ok[1233], "verify");

    /* unknown tickets */
    CHECK(md5hip_pool_wait(p, (99999ull << 6) | 1) == -EINVAL, "unknown whole ticket");
    CHECK(md5hip_pool_wait(p, (5ull << 6) | 9) == -EINVAL, "no device 9");
    CHECK(md5hip_pool_poll(p, (1ull << 63) | 999) == -EINVAL, "unknown split ticket");
    CHECK(md5hip_pool_wait(p, 0) == 0 && md5hip_pool_poll(p, 0) == 1, "ticket 0");

    /* failures: every 9th device submission fails; a split ticket reports its
     * own (first) part error, whole tickets theirs, and the others stay 0 */
    g_fail_every = 9;
    int fails = 0, oks = 0;
    for (int r = 0; r < 60; r++) {
        uint64_t tt;
        const int n = r % 2 ? 2000 : 30;
        const int rc = md5hip_pool_submit_async(p, ptrs, g_lens, (uint64_t)n, &dig[0][0], &tt);
        CHECK(rc == 0, "submit with failures %d", rc);
        const int w = md5hip_pool_wait(p, tt);
        CHECK(w == 0 || w == -EIO, "wait %d", w);
        CHECK(md5hip_pool_wait(p, tt) == w, "the same result twice");
        if (w) fails++;
        else oks++;
    }
    CHECK(fails > 0 && oks > 0, "failures %d, successes %d", fails, oks);
    g_fail_every = 0;

    /* a lost device (md5_pool.c failover): a synchronous split part on it is
     * moved to a healthy device and the call returns 0 with every digest;
     * the device is never routed to again */
    md5hip_pool_set_split(p, 1u << 20);
    CHECK(md5hip_pool_inject_fault(p, 2, 1) == 0, "inject 2");
    memset(dig, 0, sizeof dig);
    CHECK(md5hip_pool_submit(p, ptrs, g_lens, 2000, &dig[0][0]) == 0, "sync split with a device lost");
    for (int i = 0; i < 2000; i++) CHECK(memcmp(dig[i], g_want[i], 16) == 0, "failover digest %d", i);
    struct md5hip_pool_health h;
    CHECK(md5hip_pool_get_health(p, &h) == 0 && h.ndev == 4 && h.nfailed == 1 && h.failed_mask == 4 &&
          h.failovers == 1, "health: nfailed %u mask %llx failovers %llu", h.nfailed,
          (unsigned long long)h.failed_mask, (unsigned long long)h.failovers);
    CHECK(md5hip_pool_device_health(p, 2) == -ENODEV && md5hip_pool_device_health(p, 1) == 0 &&
          md5hip_pool_device_health(p, 4) == -EINVAL && md5hip_pool_inject_fault(p, 2, 1) == -ENODEV,
          "device health");
    struct md5hip_batcher_stats d2a, d2b;
    md5hip_pool_device_stats(p, 2, &d2a);
    for (int r = 0; r < 30; r++) {
        const int n = r % 2 ? 2000 : 1 + r * 7;
        memset(dig, 0, sizeof dig);
        if (r % 3 == 0) {
            uint64_t tt;
            CHECK(md5hip_pool_submit_async(p, ptrs, g_lens, (uint64_t)n, &dig[0][0], &tt) == 0, "async after loss");
            CHECK(md5hip_pool_wait(p, tt) == 0, "async wait after loss");
        } else {
            CHECK(md5hip_pool_submit(p, ptrs, g_lens, (uint64_t)n, &dig[0][0]) == 0, "sync after loss");
        }
        for (int i = 0; i < n; i++) CHECK(memcmp(dig[i], g_want[i], 16) == 0, "after loss %d/%d", r, i);
    }
    md5hip_pool_device_stats(p, 2, &d2b);
    CHECK(d2b.submissions == d2a.submissions, "the failed device took %llu more",
          (unsigned long long)(d2b.submissions - d2a.submissions));
    /* an asynchronous split ticket whose part's device is lost keeps -EIO */
    CHECK(md5hip_pool_inject_fault(p, 1, 1) == 0, "inject 1");
    memset(dig, 0, sizeof dig);
    CHECK(md5hip_pool_submit_async(p, ptrs, g_lens, 2000, &dig[0][0], &t) == 0, "async split, device 1 lost");
    CHECK(md5hip_pool_wait(p, t) == -EIO, "async ticket -EIO");
    CHECK(md5hip_pool_wait(p, t) == -EIO, "kept");
    CHECK(md5hip_pool_get_health(p, &h) == 0 && h.nfailed == 2 && h.failed_mask == 6 && h.failovers == 1,
          "two lost: mask %llx failovers %llu", (unsigned long long)h.failed_mask, (unsigned long long)h.failovers);
    /* host_fixed while the last two devices are lost on the way: moved from
     * one to the other, then -ENODEV with nothing left */
    CHECK(md5hip_pool_inject_fault(p, 0, 1) == 0 && md5hip_pool_inject_fault(p, 3, 1) == 0, "inject 0, 3");
    static unsigned char fx[64][16];
    CHECK(md5hip_pool_host_fixed(p, g_blob, 64, 1000, 1000, &fx[0][0]) == -ENODEV, "fixed, last two lost");
    CHECK(md5hip_pool_get_health(p, &h) == 0 && h.nfailed == 4 && h.failed_mask == 15 && h.failovers == 3,
          "all lost: %u failovers %llu", h.nfailed, (unsigned long long)h.failovers);
    t = 5;
    CHECK(md5hip_pool_submit(p, ptrs, g_lens, 10, &dig[0][0]) == -ENODEV, "sync, all lost");
    CHECK(md5hip_pool_submit_async(p, ptrs, g_lens, 10, &dig[0][0], &t) == -ENODEV && t == 0, "async, all lost");
    CHECK(md5hip_pool_host_fixed(p, g_blob, 4, 1000, 1000, &fx[0][0]) == -ENODEV, "fixed, all lost");
    md5hip_pool_destroy(p);
    CHECK(md5hip_pool_create(devs, 4, 0, 0, &p) == 0 && p, "create again");

    /* eight threads at once, tickets waited in reverse, half polled first */
    md5hip_pool_set_split(p, 4u << 20);
    struct job jobs[8];
    pthread_t th[8];
    for (int k = 0; k < 8; k++) {
        jobs[k] = (struct job){p, k, 6, 0, 0};
        CHECK(pthread_create(&th[k], NULL, thread_main, &jobs[k]) == 0, "thread");
    }
    for (int k = 0; k < 8; k++) {
        pthread_join(th[k], NULL);
        CHECK(jobs[k].bad == 0 && jobs[k].rc_bad == 0, "thread %d: bad %d rc %d", k, jobs[k].bad, jobs[k].rc_bad);
    }
    md5hip_pool_destroy(p);
    free(g_blob);
    printf("pool ok\n");
    return 0;
}
