/*
 * md5_tickets.h -- the batcher's ticket table (md5_submit.c), kept apart so
 * the host test (tests/c/tickets_check.c) drives exactly this code.
 *
 * Tickets are ids handed out in increasing order.  Live ids [lo, hi) sit in a
 * power-of-two ring: a count of outstanding references (the submission
 * itself, plus one per slot holding its chunks) and the ticket's first error.
 * When the oldest ids reach zero references the ring's low end advances past
 * them.  A ticket that leaves the ring with an error keeps it in `failed`, a
 * sorted list (ids leave in increasing order, so appending keeps it sorted):
 * a wait or poll on an old ticket reports that ticket's own error, never
 * another ticket's, and 0 for every ticket that completed cleanly.
 *
 * Not thread-safe by itself: the batcher calls these under its mutex.
 */
#ifndef SPROXY_AMD_MD5_TICKETS_H
#define SPROXY_AMD_MD5_TICKETS_H

#include <errno.h>
#include <stdint.h>
#include <stdlib.h>

/* failed tickets kept for lookup; past this many the oldest half is dropped
 * (a caller that waits on a ticket millions of failures old reads 0) */
#define TK_FAILED_MAX (1u << 20)

struct tk_failed {
    uint64_t id;
    int err;
};

struct tk_ring {
    uint64_t lo, hi;          /* live ids [lo, hi) */
    uint64_t cap;             /* ring size, a power of two */
    uint32_t *pending;        /* references per live id */
    int *err;                 /* first error per live id */
    struct tk_failed *failed; /* ids < lo that completed with an error, ascending */
    uint64_t nfailed, capfailed;
};

static inline int tk_ring_grow(struct tk_ring *r)
{
    const uint64_t nc = r->cap ? 2 * r->cap : 1024;
    uint32_t *p = (uint32_t *)malloc(nc * sizeof *p);
    int *e = (int *)malloc(nc * sizeof *e);
    if (!p || !e) { free(p); free(e); return -ENOMEM; }
    for (uint64_t t = r->lo; t < r->hi; t++) {
        p[t & (nc - 1)] = r->pending[t & (r->cap - 1)];
        e[t & (nc - 1)] = r->err[t & (r->cap - 1)];
    }
    free(r->pending);
    free(r->err);
    r->pending = p;
    r->err = e;
    r->cap = nc;
    return 0;
}

/* first id handed out is `first` (ids below it read as complete, no error) */
static inline int tk_ring_init(struct tk_ring *r, uint64_t first)
{
    r->lo = r->hi = first;
    r->cap = 0;
    r->pending = NULL;
    r->err = NULL;
    r->failed = NULL;
    r->nfailed = r->capfailed = 0;
    return tk_ring_grow(r);
}

static inline void tk_ring_free(struct tk_ring *r)
{
    free(r->pending);
    free(r->err);
    free(r->failed);
    r->pending = NULL;
    r->err = NULL;
    r->failed = NULL;
}

/* a new ticket holding one reference (the submission in progress) */
static inline int tk_ring_new(struct tk_ring *r, uint64_t *t)
{
    if (r->hi - r->lo == r->cap) {
        const int rc = tk_ring_grow(r);
        if (rc) return rc;
    }
    const uint64_t id = r->hi++;
    r->pending[id & (r->cap - 1)] = 1;
    r->err[id & (r->cap - 1)] = 0;
    *t = id;
    return 0;
}

/* one more reference on live ticket t (a slot now holds some of its chunks) */
static inline void tk_ring_ref(struct tk_ring *r, uint64_t t)
{
    if (t >= r->lo && t < r->hi) r->pending[t & (r->cap - 1)]++;
}

static inline void tk_ring_remember(struct tk_ring *r, uint64_t id, int err)
{
    if (r->nfailed == r->capfailed) {
        if (r->capfailed >= TK_FAILED_MAX) {          /* drop the oldest half */
            const uint64_t keep = r->nfailed / 2;
            for (uint64_t k = 0; k < keep; k++) r->failed[k] = r->failed[r->nfailed - keep + k];
            r->nfailed = keep;
        } else {
            const uint64_t nc = r->capfailed ? 2 * r->capfailed : 64;
            struct tk_failed *f = (struct tk_failed *)realloc(r->failed, nc * sizeof *f);
            if (!f) return;                           /* no memory: this error reads as 0 later */
            r->failed = f;
            r->capfailed = nc;
        }
    }
    r->failed[r->nfailed].id = id;
    r->failed[r->nfailed].err = err;
    r->nfailed++;
}

/* drop one reference of ticket t, recording err as its error if it is the
 * first; retire the completed ids at the ring's low end */
static inline void tk_ring_put(struct tk_ring *r, uint64_t t, int err)
{
    if (t < r->lo || t >= r->hi) return;
    const uint64_t k = t & (r->cap - 1);
    if (err && !r->err[k]) r->err[k] = err;
    if (r->pending[k]) r->pending[k]--;
    while (r->lo < r->hi && r->pending[r->lo & (r->cap - 1)] == 0) {
        const int e = r->err[r->lo & (r->cap - 1)];
        if (e) tk_ring_remember(r, r->lo, e);
        r->lo++;
    }
}

/* 1 = ticket t is complete (*err = its own error, 0 if none), 0 = pending */
static inline int tk_ring_done(const struct tk_ring *r, uint64_t t, int *err)
{
    if (t < r->lo) {
        uint64_t a = 0, b = r->nfailed;
        while (a < b) {
            const uint64_t mid = (a + b) / 2;
            if (r->failed[mid].id < t) a = mid + 1;
            else b = mid;
        }
        *err = a < r->nfailed && r->failed[a].id == t ? r->failed[a].err : 0;
        return 1;
    }
    *err = r->err[t & (r->cap - 1)];
    return r->pending[t & (r->cap - 1)] == 0;
}

#endif
