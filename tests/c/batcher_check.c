/*
 * batcher_check.c -- the batcher, the device queue and the pool
 * (md5_submit.c, md5_pool.c) run whole on the host against the fake HIP
 * runtime of fake_hip.c, from 10 threads at once for a few seconds, under
 * ASan+UBSan or TSan (tests/test_batcher_host.py).  Every thread picks
 * random operations -- synchronous / asynchronous submits of pointer lists
 * and page lists, verify with a flipped digest, host_fixed, device-resident
 * fixed-length runs (md5_batch_submit_device_fixed), device-resident
 * submits with host or device digests (also ordered after a producer
 * stream), pool submits whole and split, CRC-32 on its own batcher, fastcrc
 * on page lists split across its windows (only the windows staged), netcache
 * header verification, flush -- from pageable or registered memory, and
 * checks every digest against the library's host MD5 computed up front; one
 * more thread keeps changing the batchers' knobs (inflight target, linger,
 * gather mode, pool split) and another registers, uses and unregisters a
 * private page range.  The pool spans devices 0, 1 and 2, and every copy
 * or kernel must be enqueued from a thread whose current device is its
 * stream's (fake_hip_wrong_device stays 0): waits and polls on another
 * device's ticket included.
 *
 * Before that, the blocked-caller phase: 64 threads wait on tickets that all
 * sit in ONE open slot behind a held launch; when the launch is released the
 * slot goes in flight, one of them watches it, and (every other round) that
 * watcher's spin ends on NotReady just as the kernel finishes and the
 * progress thread retires the launch (fake_hip_slow_query) -- every waiter
 * must return with correct digests within the round's deadline (the lost
 * wake-up of round 3 hung here).  Then large_device(): large
 * device-resident vectors, coalesced, with their device digests scattered
 * in pieces.  Then device_lost(): the failure policy (md5_submit.c header,
 * md5_pool.c) -- a device lost after launch K, as its completion event
 * reporting the fault and as the launch itself failing: the failing ticket
 * gets -EIO, tickets coalescing behind it and every later call -ENODEV,
 * nothing is enqueued on the device again, no caller hangs; a 2-device pool
 * moves a synchronous submission off the failed device and never routes to
 * it again; 8 threads at once while a device dies under them.  Then
 * fragmented(): chunks of ~4,096 one-byte registered segments, at the edge of
 * a slot's zero-copy table, MD5 and fastcrc.
 * Exits 0 when every check holds.
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>
#include <unistd.h>

#include "md5.h"
#include "md5hip.h"
#include "nc_digest.h"

#define NCH 3000
#define MAXV 200

static unsigned char *g_heap, *g_pageable;
static uint32_t g_lens[NCH];
static uint64_t g_offs[NCH];
static unsigned char g_md5[NCH][16];
static uint32_t g_crc[NCH];
static md5hip_batcher *g_b, *g_q, *g_crcb, *g_fcrc;
static md5hip_pool *g_pool;
extern uint32_t fake_hip_fail_len;
extern unsigned long fake_hip_wrong_device;
extern int fake_hip_hold, fake_hip_slow_query;
void fake_hip_mark_thread(void);
void fake_hip_lose_device(int dev, int after_kernels, int how);
int fake_hip_device_faulted(int dev);
void fake_hip_pin(const void *p, size_t len);
void fake_hip_unpin(const void *p);
void fake_hip_watch(const void *p, size_t len);
extern unsigned long fake_hip_pageable_dma, fake_hip_watched_h2d;
extern int fake_hip_no_range;
extern unsigned long fake_hip_sort_refused;
static int g_stop;
#define STOPPED() __atomic_load_n(&g_stop, __ATOMIC_RELAXED)
#define STOP() __atomic_store_n(&g_stop, 1, __ATOMIC_RELAXED)
static int g_fail;
static pthread_mutex_t g_fail_mu = PTHREAD_MUTEX_INITIALIZER;

static void fail(const char *what, int t, int rc)
{
    pthread_mutex_lock(&g_fail_mu);
    if (!g_fail) printf("FAIL thread %d: %s (rc %d)\n", t, what, rc);
    g_fail = 1;
    STOP();
    pthread_mutex_unlock(&g_fail_mu);
}

static uint64_t rnd(uint64_t *s)
{
    *s ^= *s << 13; *s ^= *s >> 7; *s ^= *s << 17;
    return *s;
}

static double now(void)
{
    struct timespec ts;
    clock_gettime(CLOCK_MONOTONIC, &ts);
    return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct held {
    uint64_t t;
    int kind;                      /* 0 batcher, 1 queue, 2 pool */
    int n, idx[MAXV];
    unsigned char dig[MAXV][16];
};

static int check_md5(unsigned char (*dig)[16], const int *idx, int n)
{
    for (int i = 0; i < n; i++)
        if (memcmp(dig[i], g_md5[idx[i]], 16)) return 0;
    return 1;
}

static void *worker(void *arg)
{
    const int t = (int)(intptr_t)arg;
    uint64_t s = 0x9E3779B97F4A7C15ull ^ (uint64_t)(t + 1) * 7919u;
    struct held *held[4];
    int nheld = 0;
    const void *ptrs[MAXV];
    uint32_t lens[MAXV];
    uint64_t dptrs[MAXV];
    struct md5hip_iov segs[2 * MAXV];
    uint64_t first[MAXV + 1];
    unsigned char dig[MAXV][16];
    int idx[MAXV];
    while (!STOPPED()) {
        const int n = 1 + (int)(rnd(&s) % MAXV);
        const unsigned char *src = rnd(&s) % 3 ? g_heap : g_pageable;
        for (int i = 0; i < n; i++) {
            idx[i] = (int)(rnd(&s) % NCH);
            ptrs[i] = src + g_offs[idx[i]];
            lens[i] = g_lens[idx[i]];
            dptrs[i] = (uint64_t)(uintptr_t)(g_heap + g_offs[idx[i]]);
        }
        const int op = (int)(rnd(&s) % 14);
        int rc = 0;
        memset(dig, 0, sizeof dig);
        switch (op) {
        case 0:
            rc = md5_batch_submit(g_b, ptrs, lens, (uint64_t)n, &dig[0][0]);
            if (rc || !check_md5(dig, idx, n)) fail("submit", t, rc);
            break;
        case 1: case 2: {
            if (nheld == 4) break;
            struct held *h = held[nheld] = malloc(sizeof *h);
            h->n = n;
            memcpy(h->idx, idx, sizeof(int) * n);
            h->kind = op == 1 ? 0 : 2;
            rc = op == 1 ? md5_batch_submit_async(g_b, ptrs, lens, (uint64_t)n, &h->dig[0][0], &h->t)
                         : md5hip_pool_submit_async(g_pool, ptrs, lens, (uint64_t)n, &h->dig[0][0], &h->t);
            if (rc) fail("submit_async", t, rc);
            else nheld++;
            if (rc) free(h);
            break;
        }
        case 3: {
            uint64_t ns = 0;
            for (int i = 0; i < n; i++) {
                first[i] = ns;
                const uint32_t a = lens[i] / 3;
                segs[ns++] = (struct md5hip_iov){ptrs[i], a};
                segs[ns++] = (struct md5hip_iov){(const unsigned char *)ptrs[i] + a, lens[i] - a};
            }
            first[n] = ns;
            rc = rnd(&s) & 1 ? md5_batch_submit_iov(g_b, segs, first, (uint64_t)n, &dig[0][0])
                             : md5hip_pool_submit_iov(g_pool, segs, first, (uint64_t)n, &dig[0][0]);
            if (rc || !check_md5(dig, idx, n)) fail("submit_iov", t, rc);
            break;
        }
        case 4: {
            uint64_t ns = 0;
            for (int i = 0; i < n; i++) {
                first[i] = ns;
                segs[ns++] = (struct md5hip_iov){ptrs[i], lens[i]};
                memcpy(dig[i], g_md5[idx[i]], 16);
            }
            first[n] = ns;
            const int j = (int)(rnd(&s) % (uint64_t)n);
            dig[j][5] ^= 0x10;
            unsigned char ok[MAXV];
            rc = md5hip_batch_verify_iov(g_b, segs, first, (uint64_t)n, &dig[0][0], ok);
            if (rc != 1 || ok[j]) fail("verify", t, rc);
            break;
        }
        case 5: {
            rc = md5_batch_submit_device(g_q, dptrs, lens, (uint64_t)n, &dig[0][0], 0);
            if (rc || !check_md5(dig, idx, n)) fail("submit_device", t, rc);
            break;
        }
        case 6: {
            /* device digests (16-B aligned in place, or odd: scattered) */
            unsigned char *raw = malloc(16 * (size_t)n + 20);
            unsigned char *d = raw + (rnd(&s) & 1 ? 0 : 4);
            const uint64_t how = rnd(&s) % 3;      /* no ordering / a producer stream / the null stream */
            rc = how == 2 ? md5_batch_submit_device_after(g_q, dptrs, lens, (uint64_t)n, d, 1, NULL, 1, NULL)
                          : md5_batch_submit_device_on(g_q, dptrs, lens, (uint64_t)n, d, 1,
                                                       how ? (void *)g_q : NULL, NULL);
            if (rc || !check_md5((unsigned char (*)[16])d, idx, n)) fail("submit_device_on", t, rc);
            free(raw);
            break;
        }
        case 7: {
            if (nheld == 4) break;
            struct held *h = held[nheld] = malloc(sizeof *h);
            h->n = n;
            memcpy(h->idx, idx, sizeof(int) * n);
            h->kind = 1;
            rc = md5_batch_submit_device_async(g_q, dptrs, lens, (uint64_t)n, &h->dig[0][0], 0, &h->t);
            if (rc) fail("submit_device_async", t, rc), free(h);
            else nheld++;
            break;
        }
        case 8: {
            uint32_t crc[MAXV];
            rc = md5_batch_submit(g_crcb, ptrs, lens, (uint64_t)n, (unsigned char *)crc);
            for (int i = 0; i < n && !rc; i++)
                if (crc[i] != g_crc[idx[i]]) rc = -1000 - i;
            if (rc) fail("crc", t, rc);
            break;
        }
        case 9: {
            /* netcache headers on the MD5 batcher (a CRC-32 call that must
             * leave the shared batcher's kind alone); every 4th a header_size
             * of 0..19 (dm_verify_header's partial fixed part), every 3rd
             * of the others broken */
            enum { NH = 24 };
            unsigned char hb[NH][256];
            const void *hp[NH];
            unsigned char ok[NH], want[NH];
            int bad = 0;
            for (int i = 0; i < NH; i++) {
                const uint32_t hs = i % 4 == 3 ? (uint32_t)(rnd(&s) % 20) : 20 + (uint32_t)(rnd(&s) % 236),
                               magic = NC_MAGIC_V30;
                for (int k = 0; k < 256; k++) hb[i][k] = (unsigned char)rnd(&s);
                memcpy(hb[i] + NC_HDR_OFF_MAGIC, &magic, 4);
                memcpy(hb[i] + NC_HDR_OFF_HEADER_SIZE, &hs, 4);
                if (nc_header_seal(hb[i])) { rc = -1; break; }
                want[i] = 1;
                if (i % 3 == 2 && hs >= 20) hb[i][hs - 1] ^= 0x40, bad++, want[i] = 0;
                hp[i] = hb[i];
            }
            if (!rc) rc = md5hip_batch_verify_headers(g_b, hp, NH, ok);
            for (int i = 0; i < NH && rc == bad; i++)
                if (ok[i] != want[i] || nc_header_verify(hb[i]) != want[i]) rc = -3000 - i;
            if (rc != bad) fail("verify_headers", t, rc);
            rc = 0;
            break;
        }
        case 10: {
            /* asynchronous submit, then an explicit flush, then wait */
            uint64_t tk;
            rc = md5_batch_submit_async(g_b, ptrs, lens, (uint64_t)n, &dig[0][0], &tk);
            if (!rc) rc = md5_batch_flush(g_b);
            if (!rc) rc = md5_batch_wait(g_b, tk);
            if (rc || !check_md5(dig, idx, n)) fail("flush", t, rc);
            int kind;
            uint32_t fc;
            if ((rc = md5hip_batcher_get_digest(g_crcb, &kind, &fc)) || kind != MD5HIP_DIGEST_CRC32 || fc)
                fail("get_digest", t, rc);
            break;
        }
        case 12: {
            /* fastcrc 100 (blk_io.c:408-424) on page lists split at random
             * points: the batcher stages (or maps) only each chunk's head and
             * tail windows, which may straddle segments */
            enum { FW = 100 };
            uint64_t ns = 0;
            for (int i = 0; i < n; i++) {
                first[i] = ns;
                const uint32_t a = lens[i] ? (uint32_t)(rnd(&s) % (lens[i] + 1)) : 0;
                segs[ns++] = (struct md5hip_iov){ptrs[i], a};
                segs[ns++] = (struct md5hip_iov){(const unsigned char *)ptrs[i] + a, lens[i] - a};
            }
            first[n] = ns;
            uint32_t crc[MAXV];
            rc = md5_batch_submit_iov(g_fcrc, segs, first, (uint64_t)n, (unsigned char *)crc);
            for (int i = 0; i < n && !rc; i++) {
                const unsigned char *p = ptrs[i];
                const uint32_t L = lens[i];
                const uint32_t want = L <= FW ? nc_crc32(p, L) : nc_crc32(p, FW) ^ nc_crc32(p + L - FW, FW);
                if (crc[i] != want) rc = -3500 - i;
            }
            if (rc) fail("fastcrc windows", t, rc);
            break;
        }
        case 11: {
            /* device-resident fixed-length chunks on the queue, host or device
             * digests (the latter odd-aligned half the time: scattered) */
            const uint32_t L = 4096;
            const uint64_t k = rnd(&s) % 300;
            const int m = 1 + (int)(rnd(&s) % 60);
            const unsigned char *base = g_heap + k * L;
            unsigned char *raw = malloc(16 * (size_t)m + 20);
            unsigned char *d = rnd(&s) & 1 ? raw + (rnd(&s) & 1 ? 0 : 4) : &dig[0][0];
            const int on_dev = d != &dig[0][0];
            uint64_t tk = 0;
            const int async = (int)(rnd(&s) & 1);
            rc = md5_batch_submit_device_fixed(g_q, base, (uint64_t)m, L, L, d, on_dev, NULL, 0, async ? &tk : NULL);
            if (!rc && async) rc = md5_batch_wait(g_q, tk);
            for (int i = 0; i < m && !rc; i++) {
                unsigned char w[16];
                struct MD5Context c;
                MD5Init(&c);
                MD5Update(&c, base + (uint64_t)i * L, L);
                MD5Final(w, &c);
                if (memcmp(w, d + 16 * i, 16)) rc = -2500 - i;
            }
            free(raw);
            if (rc) fail("device_fixed", t, rc);
            break;
        }
        default: {
            /* 4 KiB pages; or ragged lengths at a larger stride; or empty
             * chunks at stride 0 */
            const uint32_t shape = (uint32_t)(rnd(&s) % 8);
            const uint32_t L = shape < 5 ? 4096 : shape < 7 ? (uint32_t)(rnd(&s) % 4096) : 0;
            const uint64_t S = shape < 5 ? 4096 : shape < 7 ? 4096 + 16 * (rnd(&s) % 8) : 0;
            const uint64_t k = rnd(&s) % 300;
            const int m = 1 + (int)(rnd(&s) % 60);
            const unsigned char *base = g_heap + k * 4096;
            rc = rnd(&s) & 1 ? md5hip_batch_host_fixed(g_b, base, (uint64_t)m, L, S, &dig[0][0])
                             : md5hip_pool_host_fixed(g_pool, base, (uint64_t)m, L, S, &dig[0][0]);
            for (int i = 0; i < m && !rc; i++) {
                unsigned char w[16];
                struct MD5Context c;
                MD5Init(&c);
                MD5Update(&c, base + (uint64_t)i * S, L);
                MD5Final(w, &c);
                if (memcmp(w, dig[i], 16)) rc = -2000 - i;
            }
            if (rc) fail("host_fixed", t, rc);
        }
        }
        /* collect a held ticket now and then, in any order */
        if (nheld && (nheld == 4 || rnd(&s) % 3 == 0)) {
            const int j = (int)(rnd(&s) % (uint64_t)nheld);
            struct held *h = held[j];
            if (rnd(&s) & 1) {                       /* poll a few times first */
                for (int k = 0; k < 3; k++) {
                    const int p = h->kind == 2 ? md5hip_pool_poll(g_pool, h->t)
                                               : md5_batch_poll(h->kind ? g_q : g_b, h->t);
                    if (p < 0) fail("poll", t, p);
                    if (p) break;
                }
            }
            rc = h->kind == 2 ? md5hip_pool_wait(g_pool, h->t) : md5_batch_wait(h->kind ? g_q : g_b, h->t);
            if (rc || !check_md5(h->dig, h->idx, h->n)) fail("wait", t, rc);
            free(h);
            held[j] = held[--nheld];
        }
    }
    for (int j = 0; j < nheld; j++) {
        struct held *h = held[j];
        const int rc = h->kind == 2 ? md5hip_pool_wait(g_pool, h->t) : md5_batch_wait(h->kind ? g_q : g_b, h->t);
        if (rc || !check_md5(h->dig, h->idx, h->n)) fail("final wait", t, rc);
        free(h);
    }
    return NULL;
}

static void *knobs(void *arg)
{
    (void)arg;
    uint64_t s = 42;
    while (!STOPPED()) {
        md5hip_batcher_set_inflight(g_b, 1 + (uint32_t)(rnd(&s) % 3));
        md5hip_batcher_set_linger(g_q, (uint32_t)(rnd(&s) % 400));
        md5hip_batcher_set_chain(g_b, (int)(rnd(&s) % 3));
        md5hip_batcher_set_gather(g_b, (int)(rnd(&s) % 4));
        md5hip_pool_set_gather(g_pool, (int)(rnd(&s) % 4));
        md5hip_pool_set_split(g_pool, (rnd(&s) % 2) ? 0 : 256u << 10);
        struct timespec ts = {0, 2000000};
        nanosleep(&ts, NULL);
    }
    return NULL;
}

/* registrations come and go beside the workers' lookups: each round
 * registers a private copy of a heap slice, hashes chunks from it through the
 * batcher and the pool (zero-copy while registered), unregisters it */
static void *registrar(void *arg)
{
    (void)arg;
    uint64_t s = 7;
    const uint64_t span = g_offs[200];
    unsigned char *copy = malloc(span + 64);
    memcpy(copy, g_heap, span + 64);
    const void *ptrs[200];
    unsigned char dig[200][16];
    int idx[200];
    for (int i = 0; i < 200; i++) ptrs[i] = copy + g_offs[i], idx[i] = i;
    while (!STOPPED()) {
        int rc = md5hip_host_register(copy, span + 64);
        const int n = 1 + (int)(rnd(&s) % 200);
        if (!rc) rc = rnd(&s) & 1 ? md5_batch_submit(g_b, ptrs, g_lens, (uint64_t)n, &dig[0][0])
                                  : md5hip_pool_submit(g_pool, ptrs, g_lens, (uint64_t)n, &dig[0][0]);
        if (rc || !check_md5(dig, idx, n)) fail("registered copy", 99, rc);
        if ((rc = md5hip_host_unregister(copy))) fail("unregister", 99, rc);
    }
    free(copy);
    return NULL;
}

/* ---------------------------------------------------------- blocked callers */
#define WT 64      /* waiters on one slot */
#define WN 8       /* chunks per waiter */
static md5hip_batcher *g_w;
static pthread_barrier_t g_wbar;

struct wjob {
    int t, round, n, rc, bad;
    int idx[WN];
    unsigned char dig[WN][16];
    uint64_t tk;
};

static void *waiter(void *arg)
{
    struct wjob *j = arg;
    uint64_t s = 0xA5A5ull * (uint64_t)(j->t + 1) + (uint64_t)j->round * 131u;
    const void *ptrs[WN];
    uint32_t lens[WN];
    j->n = 1 + (int)(rnd(&s) % WN);
    for (int i = 0; i < j->n; i++) {
        int k;
        do k = (int)(rnd(&s) % NCH); while (g_lens[k] > 3000);
        j->idx[i] = k;
        ptrs[i] = g_heap + g_offs[k];
        lens[i] = g_lens[k];
    }
    j->rc = md5_batch_submit_async(g_w, ptrs, lens, (uint64_t)j->n, &j->dig[0][0], &j->tk);
    pthread_barrier_wait(&g_wbar);          /* every ticket is in the open slot */
    fake_hip_mark_thread();
    if (!j->rc) j->rc = md5_batch_wait(g_w, j->tk);
    j->bad = !check_md5(j->dig, j->idx, j->n);
    return NULL;
}

static int blocked_callers(int rounds)
{
    int rc = md5hip_batcher_create(0, 4u << 20, 2, &g_w);      /* 2 slots: inflight target 1 */
    if (rc) { printf("FAIL waiter batcher %d\n", rc); return 1; }
    /* the held launch outlives every estimate of its end: no chaining (the
     * 64 tickets must stay in the open slot until it is released) */
    if ((rc = md5hip_batcher_set_chain(g_w, 0))) { printf("FAIL set_chain %d\n", rc); return 1; }
    for (int r = 0; r < rounds; r++) {
        struct md5hip_batcher_stats st;
        md5hip_batcher_get_stats(g_w, &st);
        const uint64_t launches0 = st.launches;
        __atomic_store_n(&fake_hip_hold, 1, __ATOMIC_RELAXED);
        /* a held launch in flight, so the waiters' chunks coalesce in the open slot
         * (which may be chained behind it before the release) */
        const void *bp = g_heap;
        uint32_t bl = 100;
        unsigned char bd[16];
        uint64_t bt;
        if ((rc = md5_batch_submit_async(g_w, &bp, &bl, 1, bd, &bt)) || (rc = md5_batch_flush(g_w))) {
            printf("FAIL blocker %d\n", rc);
            return 1;
        }
        pthread_barrier_init(&g_wbar, NULL, WT + 1);
        static struct wjob jobs[WT];
        pthread_t th[WT];
        for (int t = 0; t < WT; t++) {
            jobs[t] = (struct wjob){.t = t, .round = r};
            pthread_create(&th[t], NULL, waiter, &jobs[t]);
        }
        pthread_barrier_wait(&g_wbar);
        struct timespec ts = {0, 20000000};            /* let them all block */
        nanosleep(&ts, NULL);
        __atomic_store_n(&fake_hip_slow_query, r & 1, __ATOMIC_RELAXED);
        __atomic_store_n(&fake_hip_hold, 0, __ATOMIC_RELAXED);
        const double t0 = now();
        for (int t = 0; t < WT; t++) pthread_join(th[t], NULL);
        const double dt = now() - t0;
        __atomic_store_n(&fake_hip_slow_query, 0, __ATOMIC_RELAXED);
        pthread_barrier_destroy(&g_wbar);
        if ((rc = md5_batch_wait(g_w, bt))) { printf("FAIL blocker wait %d\n", rc); return 1; }
        md5hip_batcher_get_stats(g_w, &st);
        for (int t = 0; t < WT; t++)
            if (jobs[t].rc || jobs[t].bad) {
                printf("FAIL waiter %d round %d: rc %d bad %d\n", t, r, jobs[t].rc, jobs[t].bad);
                return 1;
            }
        /* the 64 tickets went out together: the blocker's launch and one more */
        if (st.launches != launches0 + 2 || st.max_tickets_per_launch < WT) {
            printf("FAIL round %d: %llu launches for the waiters, max %llu tickets per launch\n", r,
                   (unsigned long long)(st.launches - launches0), (unsigned long long)st.max_tickets_per_launch);
            return 1;
        }
        if (dt > 5.0) { printf("FAIL round %d took %.1f s\n", r, dt); return 1; }
    }
    md5hip_batcher_destroy(g_w);
    printf("blocked callers: %d rounds x %d waiters on one slot ok\n", rounds, WT);
    return 0;
}

/* ------------------------------------------------- large device submissions */
/* Large device-resident vectors (reserve_device's one-pass descriptors and
 * key histogram) and slots whose device digests go out through a scatter
 * table cut into pieces: 3 coalesced asynchronous
 * vectors of 40,000 chunks (random lengths, unsorted) plus one synchronous
 * vector of 70,000, digests on the host and on the device (16-B aligned and
 * not), every one checked.  The fake planner checks that the histogram
 * counts every chunk. */
static int large_device(void)
{
    enum { NV = 3, NA = 40000, NS = 70000 };
    md5hip_batcher *q;
    int rc = md5hip_queue_create(0, 4 * NA, 2, &q);
    if (rc) { printf("FAIL large queue %d\n", rc); return 1; }
    md5hip_batcher_set_chain(q, 0);
    uint64_t s = 99;
    uint64_t *dp = malloc(sizeof(uint64_t) * NS);
    uint32_t *ln = malloc(sizeof(uint32_t) * NS);
    int *idx = malloc(sizeof(int) * NS);
    unsigned char *raw = malloc(16 * (size_t)NS * (NV + 1) + 32);
    for (int round = 0; round < 2 && !rc; round++) {
        for (int i = 0; i < NS; i++) {
            idx[i] = (int)(rnd(&s) % NCH);
            dp[i] = (uint64_t)(uintptr_t)(g_heap + g_offs[idx[i]]);
            ln[i] = g_lens[idx[i]];
        }
        unsigned char *d = raw + (round ? 4 : 0);       /* device digests: scattered when odd */
        uint64_t tk[NV], bt;
        /* a held launch in flight, so the three vectors coalesce in the open slot */
        __atomic_store_n(&fake_hip_hold, 1, __ATOMIC_RELAXED);
        unsigned char bd[16];
        rc = md5_batch_submit_device_async(q, dp, ln, 1, bd, 0, &bt);
        if (!rc) rc = md5_batch_flush(q);
        for (int v = 0; v < NV && !rc; v++)
            rc = md5_batch_submit_device_async(q, dp + v * 1000, ln + v * 1000, NA, d + (size_t)16 * NA * v,
                                               round, &tk[v]);
        __atomic_store_n(&fake_hip_hold, 0, __ATOMIC_RELAXED);
        if (!rc) rc = md5_batch_wait(q, bt);
        for (int v = 0; v < NV && !rc; v++) rc = md5_batch_wait(q, tk[v]);
        for (int v = 0; v < NV && !rc; v++)
            if (!check_md5((unsigned char (*)[16])(d + (size_t)16 * NA * v), idx + v * 1000, NA)) rc = -4000 - v;
        if (!rc) rc = md5_batch_submit_device(q, dp, ln, NS, d, round);
        if (!rc && !check_md5((unsigned char (*)[16])d, idx, NS)) rc = -4100;
    }
    struct md5hip_batcher_stats st;
    md5hip_batcher_get_stats(q, &st);
    md5hip_batcher_destroy(q);
    free(dp), free(ln), free(idx), free(raw);
    if (rc) { printf("FAIL large device submissions %d\n", rc); return 1; }
    if (st.max_tickets_per_launch < NV) {
        printf("FAIL large device submissions: max %llu tickets per launch\n",
               (unsigned long long)st.max_tickets_per_launch);
        return 1;
    }
    printf("large device submissions ok: %llu launches, max %llu tickets per launch\n",
           (unsigned long long)st.launches, (unsigned long long)st.max_tickets_per_launch);
    return 0;
}

/* ------------------------------------------------------------ device lost */
#define LCHECK(c, ...)                                                      \
    do {                                                                    \
        if (!(c)) {                                                         \
            printf("FAIL device lost line %d: %s: ", __LINE__, #c);         \
            printf(__VA_ARGS__);                                            \
            printf("\n");                                                   \
            return 1;                                                       \
        }                                                                   \
    } while (0)

/* a random vector of small chunks from the registered heap */
static int pick(uint64_t *s, int maxn, const void **ptrs, uint32_t *lens, int *idx)
{
    const int n = 1 + (int)(rnd(s) % (uint64_t)maxn);
    for (int i = 0; i < n; i++) {
        idx[i] = (int)(rnd(s) % NCH);
        ptrs[i] = g_heap + g_offs[idx[i]];
        lens[i] = g_lens[idx[i]];
    }
    return n;
}

/* one batcher: the launch that faults gives -EIO, the rest -ENODEV */
static int lost_single(int dev, int how, int use_inject)
{
    md5hip_batcher *b;
    int rc = md5hip_batcher_create(dev, 1u << 20, 3, &b);
    LCHECK(rc == 0, "create %d", rc);
    md5hip_batcher_set_chain(b, 0);
    md5hip_batcher_set_inflight(b, 1);
    uint64_t s = 77u + (uint64_t)dev;
    const void *ptrs[MAXV];
    uint32_t lens[MAXV];
    int idx[MAXV];
    unsigned char dig[MAXV][16], dig2[MAXV][16];
    int n = pick(&s, 40, ptrs, lens, idx);
    LCHECK((rc = md5_batch_submit(b, ptrs, lens, (uint64_t)n, &dig[0][0])) == 0 && check_md5(dig, idx, n),
           "healthy submit %d", rc);
    LCHECK(md5hip_batcher_health(b) == 0, "healthy");
    /* E goes in flight (held), F coalesces behind it in the open slot */
    __atomic_store_n(&fake_hip_hold, 1, __ATOMIC_RELAXED);
    if (use_inject) LCHECK(md5hip_batcher_inject_fault(b, 1) == 0, "inject");
    else fake_hip_lose_device(dev, 1, how);
    uint64_t te, tf;
    n = pick(&s, 40, ptrs, lens, idx);
    memset(dig, 0x5a, sizeof dig);
    memset(dig2, 0x5a, sizeof dig2);
    rc = md5_batch_submit_async(b, ptrs, lens, (uint64_t)n, &dig[0][0], &te);
    if (how == 1 && !use_inject) {
        /* the launch itself failed at enqueue: E is done, with -EIO */
        LCHECK(rc == 0, "async E %d", rc);
        LCHECK(md5_batch_wait(b, te) == -EIO, "E -EIO");
        __atomic_store_n(&fake_hip_hold, 0, __ATOMIC_RELAXED);
    } else {
        LCHECK(rc == 0, "async E %d", rc);
        LCHECK((rc = md5_batch_flush(b)) == 0, "flush %d", rc);
        LCHECK((rc = md5_batch_submit_async(b, ptrs, lens, (uint64_t)n, &dig2[0][0], &tf)) == 0, "async F %d", rc);
        LCHECK(md5_batch_poll(b, tf) == 0, "F coalescing");
        __atomic_store_n(&fake_hip_hold, 0, __ATOMIC_RELAXED);
        LCHECK((rc = md5_batch_wait(b, te)) == -EIO, "the faulting launch's ticket: %d", rc);
        LCHECK((rc = md5_batch_wait(b, tf)) == -ENODEV, "the ticket behind it: %d", rc);
        LCHECK((rc = md5_batch_wait(b, tf)) == -ENODEV, "kept: %d", rc);
        for (int i = 0; i < n; i++) LCHECK(dig2[i][0] == 0x5a && dig2[i][15] == 0x5a, "F's digests untouched");
    }
    for (int i = 0; i < n; i++) LCHECK(dig[i][0] == 0x5a && dig[i][15] == 0x5a, "no digest of a failed launch");
    LCHECK(md5hip_batcher_health(b) == -ENODEV, "failed: %d", md5hip_batcher_health(b));
    /* every later call: -ENODEV at once, nothing enqueued */
    struct md5hip_batcher_stats st0, st1;
    md5hip_batcher_get_stats(b, &st0);
    uint64_t t = 99;
    LCHECK((rc = md5_batch_submit(b, ptrs, lens, (uint64_t)n, &dig[0][0])) == -ENODEV, "sync %d", rc);
    LCHECK((rc = md5_batch_submit_async(b, ptrs, lens, (uint64_t)n, &dig[0][0], &t)) == -ENODEV && t == 0,
           "async %d", rc);
    LCHECK((rc = md5hip_batch_host_fixed(b, g_heap, 4, 4096, 4096, &dig[0][0])) == -ENODEV, "fixed %d", rc);
    struct md5hip_iov seg = {g_heap, 100};
    uint64_t first[2] = {0, 1};
    unsigned char ok[1];
    LCHECK((rc = md5hip_batch_verify_iov(b, &seg, first, 1, g_md5[0], ok)) == -ENODEV,
           "verify: %d (a device error is not a mismatch count)", rc);
    uint64_t dp = (uint64_t)(uintptr_t)g_heap;
    uint32_t dl = 64;
    LCHECK((rc = md5_batch_submit_device(b, &dp, &dl, 1, &dig[0][0], 0)) == -ENODEV, "device %d", rc);
    md5hip_batcher_get_stats(b, &st1);
    LCHECK(st1.launches == st0.launches, "launched on a failed device");
    LCHECK(md5hip_batcher_inject_fault(b, 1) == -ENODEV, "inject on failed");
    md5hip_batcher_destroy(b);
    return 0;
}

/* a 2-device pool: a synchronous split part is moved off the failed device */
static int lost_pool_split(int d0, int d1)
{
    const int devs[2] = {d0, d1};
    md5hip_pool *p;
    int rc = md5hip_pool_create(devs, 2, 1u << 20, 3, &p);
    LCHECK(rc == 0, "pool %d", rc);
    md5hip_pool_set_split(p, 4096);                  /* every vector over both devices */
    uint64_t s = 5;
    const void *ptrs[MAXV];
    uint32_t lens[MAXV];
    int idx[MAXV];
    unsigned char dig[MAXV][16];
    int n = pick(&s, MAXV, ptrs, lens, idx);
    while (n < 20) n = pick(&s, MAXV, ptrs, lens, idx);
    LCHECK(md5hip_pool_inject_fault(p, 0, 1) == 0, "inject");
    memset(dig, 0, sizeof dig);
    LCHECK((rc = md5hip_pool_submit(p, ptrs, lens, (uint64_t)n, &dig[0][0])) == 0, "sync split %d", rc);
    LCHECK(check_md5(dig, idx, n), "digests after failover");
    struct md5hip_pool_health h;
    LCHECK(md5hip_pool_get_health(p, &h) == 0 && h.ndev == 2 && h.nfailed == 1 && h.failed_mask == 1 &&
           h.failovers == 1, "health nfailed %u mask %llx failovers %llu", h.nfailed,
           (unsigned long long)h.failed_mask, (unsigned long long)h.failovers);
    LCHECK(md5hip_pool_device_health(p, 0) == -ENODEV && md5hip_pool_device_health(p, 1) == 0 &&
           md5hip_pool_device_health(p, 2) == -EINVAL, "device health");
    /* from now on only device 1 works: whole, split, async, host_fixed */
    struct md5hip_batcher_stats b0, b1;
    md5hip_pool_device_stats(p, 0, &b0);
    for (int r = 0; r < 20; r++) {
        n = pick(&s, MAXV, ptrs, lens, idx);
        uint64_t t;
        if (r % 3 == 0) {
            LCHECK((rc = md5hip_pool_submit_async(p, ptrs, lens, (uint64_t)n, &dig[0][0], &t)) == 0, "async %d", rc);
            LCHECK((rc = md5hip_pool_wait(p, t)) == 0, "async wait %d", rc);
        } else if (r % 3 == 1) {
            LCHECK((rc = md5hip_pool_submit(p, ptrs, lens, (uint64_t)n, &dig[0][0])) == 0, "sync %d", rc);
        } else {
            LCHECK((rc = md5hip_pool_host_fixed(p, g_heap, 8, 4096, 4096, &dig[0][0])) == 0, "fixed %d", rc);
            continue;
        }
        LCHECK(check_md5(dig, idx, n), "digests round %d", r);
    }
    md5hip_pool_device_stats(p, 0, &b1);
    LCHECK(b1.submissions == b0.submissions, "routed to the failed device");
    md5hip_pool_destroy(p);
    return 0;
}

/* every device failed: -ENODEV, no hang */
static int lost_pool_all(int d0, int d1)
{
    const int devs[2] = {d0, d1};
    md5hip_pool *p;
    int rc = md5hip_pool_create(devs, 2, 1u << 20, 2, &p);
    LCHECK(rc == 0, "pool %d", rc);
    const void *ptrs[4] = {g_heap, g_heap, g_heap, g_heap};
    uint32_t lens[4] = {10, 20, 30, 40};
    unsigned char dig[4][16];
    LCHECK(md5hip_pool_inject_fault(p, 0, 1) == 0 && md5hip_pool_inject_fault(p, 1, 1) == 0, "inject");
    md5hip_pool_set_split(p, 1);                     /* one part per device */
    LCHECK((rc = md5hip_pool_submit(p, ptrs, lens, 4, &dig[0][0])) == -EIO || rc == -ENODEV, "sync %d", rc);
    struct md5hip_pool_health h;
    md5hip_pool_get_health(p, &h);
    LCHECK(h.nfailed == 2, "both failed: %u", h.nfailed);
    uint64_t t = 7;
    LCHECK((rc = md5hip_pool_submit(p, ptrs, lens, 4, &dig[0][0])) == -ENODEV, "sync after %d", rc);
    LCHECK((rc = md5hip_pool_submit_async(p, ptrs, lens, 4, &dig[0][0], &t)) == -ENODEV && t == 0,
           "async after %d", rc);
    md5hip_pool_destroy(p);
    return 0;
}

/* 8 threads on a pool while one of its devices dies under them: synchronous
 * calls all succeed (moved), asynchronous ones succeed or get -EIO / -ENODEV */
struct lj {
    md5hip_pool *p;
    int t, ops, bad, sync_err, async_eio, other, last_rc;
};

static void *lost_worker(void *arg)
{
    struct lj *j = arg;
    uint64_t s = 0xC0FFEEull * (uint64_t)(j->t + 3);
    const void *ptrs[MAXV];
    uint32_t lens[MAXV];
    int idx[MAXV];
    unsigned char dig[MAXV][16];
    struct md5hip_iov segs[MAXV];
    uint64_t first[MAXV + 1];
    for (int r = 0; r < j->ops; r++) {
        const int n = pick(&s, 80, ptrs, lens, idx);
        const int op = (int)(rnd(&s) % 4);
        int rc;
        memset(dig, 0, sizeof dig);
        if (op == 0) {
            rc = md5hip_pool_submit(j->p, ptrs, lens, (uint64_t)n, &dig[0][0]);
        } else if (op == 1) {
            for (int i = 0; i < n; i++) first[i] = (uint64_t)i, segs[i] = (struct md5hip_iov){ptrs[i], lens[i]};
            first[n] = (uint64_t)n;
            rc = md5hip_pool_submit_iov(j->p, segs, first, (uint64_t)n, &dig[0][0]);
        } else if (op == 2) {
            unsigned char ok[MAXV];
            for (int i = 0; i < n; i++) first[i] = (uint64_t)i, segs[i] = (struct md5hip_iov){ptrs[i], lens[i]};
            first[n] = (uint64_t)n;
            for (int i = 0; i < n; i++) memcpy(dig[i], g_md5[idx[i]], 16);
            rc = md5hip_pool_verify_iov(j->p, segs, first, (uint64_t)n, dig, ok);
            if (rc != 0) j->sync_err++, j->last_rc = rc;   /* 0 mismatches, never a device error */
            continue;
        } else {
            uint64_t t;
            rc = md5hip_pool_submit_async(j->p, ptrs, lens, (uint64_t)n, &dig[0][0], &t);
            if (rc == 0) rc = md5hip_pool_wait(j->p, t);
            /* its launch failed (-EIO), or it was still coalescing when the
             * device failed (-ENODEV): an asynchronous ticket is not moved */
            if (rc == -EIO || rc == -ENODEV) { j->async_eio++; continue; }
        }
        if (rc) j->sync_err++, j->last_rc = rc;
        else if (!check_md5(dig, idx, n)) j->bad++;
    }
    return NULL;
}

static int lost_pool_threads(int d0, int d1)
{
    const int devs[2] = {d0, d1};
    md5hip_pool *p;
    int rc = md5hip_pool_create(devs, 2, 1u << 20, 3, &p);
    LCHECK(rc == 0, "pool %d", rc);
    fake_hip_lose_device(d1, 6, 0);
    enum { LT = 8 };
    struct lj jobs[LT];
    pthread_t th[LT];
    for (int t = 0; t < LT; t++) {
        jobs[t] = (struct lj){p, t, 40, 0, 0, 0, 0, 0};
        pthread_create(&th[t], NULL, lost_worker, &jobs[t]);
    }
    int eio = 0;
    for (int t = 0; t < LT; t++) pthread_join(th[t], NULL);
    for (int t = 0; t < LT; t++) {
        LCHECK(jobs[t].bad == 0 && jobs[t].sync_err == 0, "thread %d: bad %d sync errors %d (last rc %d)", t,
               jobs[t].bad, jobs[t].sync_err, jobs[t].last_rc);
        eio += jobs[t].async_eio;
    }
    struct md5hip_pool_health h;
    md5hip_pool_get_health(p, &h);
    LCHECK(fake_hip_device_faulted(d1) && h.nfailed == 1 && h.failed_mask == 2, "health mask %llx",
           (unsigned long long)h.failed_mask);
    printf("device lost under 8 threads: %llu failovers, %d async tickets failed\n", (unsigned long long)h.failovers, eio);
    md5hip_pool_destroy(p);
    return 0;
}

static int device_lost(void)
{
    /* devices 0-2 belong to the other phases; the fake runtime knows 0-7 */
    if (lost_single(3, 0, 0)) return 1;               /* the completion event reports the fault */
    if (lost_single(4, 1, 0)) return 1;               /* the launch itself fails */
    if (lost_single(5, 0, 1)) return 1;               /* md5hip_batcher_inject_fault */
    if (lost_pool_split(6, 7)) return 1;              /* inject on 6 */
    if (lost_pool_all(3, 4)) return 1;                /* both already failed in the fake */
    if (lost_pool_threads(7, 6)) return 1;            /* 7 still healthy: the fake fault hits 6 again */
    printf("device lost: -EIO / -ENODEV / failover ok\n");
    return 0;
}

/* Chunks of many 1-byte segments of registered memory, around the slot's
 * zero-copy table size (4,096 entries for a 1 MiB slice): a chunk goes
 * zero-copy only if its pieces fit an empty slot, else it is staged; either
 * way it is placed (a chunk one table entry too big once closed slot after
 * empty slot without end); a fastcrc chunk sent as its two windows takes one
 * entry more. */
static int fragmented(void)
{
    static struct md5hip_iov segs[4200];
    static unsigned char flat[4200];
    const uint64_t ns_md5[] = {4094, 4095, 4096, 4097}, ns_crc[] = {150, 4093, 4094, 4097};
    for (int pass = 0; pass < 8; pass++) {
        const int crc = pass >= 4;
        const uint64_t ns = crc ? ns_crc[pass - 4] : ns_md5[pass];
        for (uint64_t k = 0; k < ns; k++) {            /* every other byte: no two pieces merge */
            segs[k] = (struct md5hip_iov){g_heap + 2 * k + pass, 1};
            flat[k] = g_heap[2 * k + pass];
        }
        const uint64_t first[2] = {0, ns};
        unsigned char d[16];
        const int rc = md5_batch_submit_iov(crc ? g_fcrc : g_b, segs, first, 1, d);
        int ok = rc == 0;
        if (ok && crc) {
            uint32_t got;
            memcpy(&got, d, 4);
            ok = got == (nc_crc32(flat, 100) ^ nc_crc32(flat + ns - 100, 100));
        } else if (ok) {
            unsigned char w[16];
            struct MD5Context c;
            MD5Init(&c);
            MD5Update(&c, flat, (unsigned)ns);
            MD5Final(w, &c);
            ok = !memcmp(w, d, 16);
        }
        if (!ok) {
            printf("FAIL fragmented %s chunk of %llu segments: rc %d\n", crc ? "fastcrc" : "md5",
                   (unsigned long long)ns, rc);
            return 1;
        }
    }
    /* a fastcrc window over half the slice: a chunk between F and 2F bytes
     * is staged whole (its two windows would not fit the slot) */
    md5hip_batcher *wb = NULL;
    int rc = md5hip_batcher_create(0, 1u << 20, 2, &wb);
    if (!rc) rc = md5hip_batcher_set_digest(wb, MD5HIP_DIGEST_CRC32, 600u << 10);
    const uint32_t F = 600u << 10, L = 700u << 10;
    const void *p[2] = {g_heap, g_pageable};
    const uint32_t l[2] = {L, L};
    uint32_t crc[2] = {0, 0};
    if (!rc) rc = md5_batch_submit(wb, p, l, 2, (unsigned char *)crc);
    const uint32_t want = nc_crc32(g_heap, F) ^ nc_crc32(g_heap + L - F, F);
    md5hip_batcher_destroy(wb);
    if (rc || crc[0] != want || crc[1] != want) {
        printf("FAIL fastcrc window over half the slice: rc %d\n", rc);
        return 1;
    }
    printf("fragmented chunks: zero-copy or staged, every digest ok\n");
    return 0;
}

/* md5hip_batch_host_fixed's in-place DMA is for a source the runtime pins
 * over its whole range (host_pinned): a buffer whose first half only is
 * page-locked, one made of two adjacent page-locked blocks, and a pinned one
 * whose extent the runtime will not tell are all staged -- no H2D copy reads
 * past a page-locked range (fake_hip_pageable_dma) -- and a wholly pinned
 * one is read in place; every digest right, n not a multiple of the slot's
 * chunk count. */
static int partly_pinned(void)
{
    enum { L = 4096, N = 77, PER = (1u << 18) / L };   /* 64 chunks a slot: one full, one of 13 */
    unsigned char *buf = malloc((size_t)N * L);
    static unsigned char want[N][16], got[N][16];
    uint64_t s = 0xFEED;
    for (size_t k = 0; k < (size_t)N * L; k++) buf[k] = (unsigned char)(rnd(&s) >> 13);
    for (int i = 0; i < N; i++) {
        struct MD5Context c;
        MD5Init(&c);
        MD5Update(&c, buf + (size_t)i * L, L);
        MD5Final(want[i], &c);
    }
    md5hip_batcher *b = NULL;
    int rc = md5hip_batcher_create(0, (uint64_t)PER * L, 2, &b);
    if (rc) { printf("FAIL partly pinned batcher %d\n", rc); free(buf); return 1; }
    fake_hip_watch(buf, (size_t)N * L);
    const char *what[5] = {"first half pinned", "two adjacent pinned blocks", "extent unknown",
                           "wholly pinned", "pageable"};
    int bad = 0;
    for (int c = 0; c < 5 && !bad; c++) {
        const size_t half = (size_t)N * L / 2, all = (size_t)N * L;
        if (c == 0) fake_hip_pin(buf, half);
        if (c == 1) fake_hip_pin(buf + half, all - half);      /* beside case 0's block */
        if (c == 2) {
            fake_hip_unpin(buf);
            fake_hip_unpin(buf + half);
            fake_hip_pin(buf, all);
            __atomic_store_n(&fake_hip_no_range, 1, __ATOMIC_RELAXED);
        }
        if (c == 3) __atomic_store_n(&fake_hip_no_range, 0, __ATOMIC_RELAXED);
        if (c == 4) fake_hip_unpin(buf);
        const unsigned long before = __atomic_load_n(&fake_hip_pageable_dma, __ATOMIC_RELAXED),
                            in0 = __atomic_load_n(&fake_hip_watched_h2d, __ATOMIC_RELAXED);
        memset(got, 0, sizeof got);
        rc = md5hip_batch_host_fixed(b, buf, N, L, L, &got[0][0]);
        const unsigned long dma = __atomic_load_n(&fake_hip_pageable_dma, __ATOMIC_RELAXED) - before,
                            inplace = __atomic_load_n(&fake_hip_watched_h2d, __ATOMIC_RELAXED) - in0;
        /* in place: one H2D per slot (2) straight from buf; staged: none */
        if (rc || memcmp(got, want, sizeof want) || dma || inplace != (c == 3 ? 2u : 0u)) {
            printf("FAIL host_fixed, %s: rc %d, digests %s, %lu H2D copies read past a page-locked range, "
                   "%lu read buf in place\n",
                   what[c], rc, memcmp(got, want, sizeof want) ? "wrong" : "ok", dma, inplace);
            bad = 1;
        }
    }
    fake_hip_watch(NULL, 0);
    md5hip_batcher_destroy(b);
    free(buf);
    if (!bad) printf("host_fixed: partly pinned, split, extent-unknown and pageable sources staged, pinned read in place, digests ok\n");
    return bad;
}

/* a hang is a failure, not a stuck test */
static void *watchdog(void *arg)
{
    const double secs = *(const double *)arg;
    const double t0 = now();
    while (now() - t0 < secs) {
        struct timespec ts = {0, 50000000};
        nanosleep(&ts, NULL);
    }
    printf("FAIL hang: still running after %.0f s\n", secs);
    fflush(stdout);
    _exit(3);
    return NULL;
}

int main(int argc, char **argv)
{
    const double secs = argc > 1 ? atof(argv[1]) : 4.0;
    setvbuf(stdout, NULL, _IOLBF, 0);             /* a crash still shows the phase it was in */
    uint64_t s = 0x1234567ull, total = 0;
    for (int i = 0; i < NCH; i++) {
        const uint64_t r = rnd(&s);
        g_lens[i] = r % 7 == 0 ? 0 : r % 5 == 0 ? (uint32_t)(r % 64)
                  : r % 11 == 0 ? (uint32_t)(r % 40000) : (uint32_t)(r % 3000);
        g_offs[i] = total;
        total += (g_lens[i] + 15) & ~15u;
    }
    g_heap = malloc(total + 64);
    g_pageable = malloc(total + 64);
    for (uint64_t k = 0; k < total + 64; k++) g_heap[k] = (unsigned char)(rnd(&s) >> 11);
    memcpy(g_pageable, g_heap, total + 64);
    for (int i = 0; i < NCH; i++) {
        struct MD5Context c;
        MD5Init(&c);
        MD5Update(&c, g_heap + g_offs[i], g_lens[i]);
        MD5Final(g_md5[i], &c);
        g_crc[i] = nc_crc32(g_heap + g_offs[i], g_lens[i]);
    }
    int rc = md5hip_host_register(g_heap, total + 64);
    if (rc) { printf("FAIL register %d\n", rc); return 1; }
    if ((rc = md5hip_batcher_create(0, 1u << 20, 3, &g_b)) ||
        (rc = md5hip_queue_create(0, 4096, 4, &g_q)) ||
        (rc = md5hip_batcher_create(0, 1u << 20, 2, &g_crcb)) ||
        (rc = md5hip_batcher_create(0, 1u << 20, 2, &g_fcrc))) {
        printf("FAIL create %d\n", rc);
        return 1;
    }
    md5hip_batcher_set_digest(g_crcb, MD5HIP_DIGEST_CRC32, 0);
    md5hip_batcher_set_digest(g_fcrc, MD5HIP_DIGEST_CRC32, 100);
    static double wd_secs;
    wd_secs = secs + 60.0;
    pthread_t wd;
    pthread_create(&wd, NULL, watchdog, &wd_secs);
    pthread_detach(wd);
    if (blocked_callers(12)) return 1;
    if (large_device()) return 1;
    if (device_lost()) return 1;
    /* error paths, one thread: a chunk over the slice, a never-issued
     * ticket, a launch that fails (sync and async; the failure is kept for
     * a second wait and does not touch later submissions) */
    {
        static unsigned char big[(1u << 20) + 1], odd[77777];
        const void *p1[2] = {big, g_pageable};
        uint32_t l1[2] = {sizeof big, 10};
        unsigned char d1[2][16];
        uint64_t tk;
        if ((rc = md5_batch_submit(g_b, p1, l1, 2, &d1[0][0])) != -E2BIG) { printf("FAIL e2big %d\n", rc); return 1; }
        if ((rc = md5_batch_wait(g_b, 1ull << 40)) >= 0) { printf("FAIL bogus ticket %d\n", rc); return 1; }
        fake_hip_fail_len = sizeof odd;
        p1[0] = odd;
        l1[0] = sizeof odd;
        if ((rc = md5_batch_submit(g_b, p1, l1, 2, &d1[0][0])) >= 0) { printf("FAIL launch error %d\n", rc); return 1; }
        if ((rc = md5_batch_submit_async(g_b, p1, l1, 2, &d1[0][0], &tk)) ||
            (rc = md5_batch_wait(g_b, tk)) >= 0 || (rc = md5_batch_wait(g_b, tk)) >= 0) {
            printf("FAIL async launch error %d\n", rc);
            return 1;
        }
        fake_hip_fail_len = 0xffffffffu;
        struct MD5Context c;
        unsigned char w[16];
        MD5Init(&c);
        MD5Update(&c, g_pageable, 10);
        MD5Final(w, &c);
        if ((rc = md5_batch_submit(g_b, p1 + 1, l1 + 1, 1, &d1[0][0])) || memcmp(d1[0], w, 16)) {
            printf("FAIL after error %d\n", rc);
            return 1;
        }
    }
    if (fragmented()) return 1;
    if (partly_pinned()) return 1;
    const int devs[3] = {0, 1, 2};
    if ((rc = md5hip_pool_create(devs, 3, 1u << 20, 2, &g_pool))) { printf("FAIL pool %d\n", rc); return 1; }
    enum { T = 10 };
    pthread_t th[T], kt, rt;
    for (int t = 0; t < T; t++) pthread_create(&th[t], NULL, worker, (void *)(intptr_t)t);
    pthread_create(&kt, NULL, knobs, NULL);
    pthread_create(&rt, NULL, registrar, NULL);
    const double t0 = now();
    while (!STOPPED() && now() - t0 < secs) {
        struct timespec ts = {0, 20000000};
        nanosleep(&ts, NULL);
    }
    STOP();
    for (int t = 0; t < T; t++) pthread_join(th[t], NULL);
    pthread_join(kt, NULL);
    pthread_join(rt, NULL);
    struct md5hip_batcher_stats bs, qs;
    md5hip_batcher_get_stats(g_b, &bs);
    md5hip_batcher_get_stats(g_q, &qs);
    struct md5hip_pool_stats ps;
    md5hip_pool_get_stats(g_pool, &ps);
    md5hip_pool_destroy(g_pool);
    md5hip_batcher_destroy(g_b);
    md5hip_batcher_destroy(g_q);
    md5hip_batcher_destroy(g_crcb);
    md5hip_batcher_destroy(g_fcrc);
    md5hip_host_unregister(g_heap);
    free(g_heap);
    free(g_pageable);
    if (g_fail) return 1;
    if (fake_hip_wrong_device) {
        printf("FAIL %lu copies/kernels enqueued from a thread on another device\n", fake_hip_wrong_device);
        return 1;
    }
    printf("batcher %llu submissions %llu launches %llu coalesced; queue %llu / %llu / %llu; "
           "pool %llu whole %llu split\n",
           (unsigned long long)bs.submissions, (unsigned long long)bs.launches,
           (unsigned long long)bs.coalesced_launches, (unsigned long long)qs.submissions,
           (unsigned long long)qs.launches, (unsigned long long)qs.coalesced_launches,
           (unsigned long long)ps.routed_whole, (unsigned long long)ps.split);
    printf("stable order refused (order_scatter fallback) %lu times\n", fake_hip_sort_refused);
    if (!fake_hip_sort_refused) {
        printf("FAIL the stable order's fallback never ran\n");
        return 1;
    }
    printf("batcher ok\n");
    return 0;
}
