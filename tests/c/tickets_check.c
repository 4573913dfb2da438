/*
 * tickets_check.c -- the batcher's ticket table (sproxy_amd/csrc/md5_tickets.h)
 * driven on the host, built with ASan/UBSan by tests/test_tickets.py.
 * Exits 0 when every check holds, else prints the failing line.
 *
 * The case ADVICE r2 raised: once a failing ticket has left the ring, every
 * later ticket must still report its OWN result (0 when it succeeded), and
 * the failed ticket keeps reporting its error, in any order of completion.
 */
#include <stdio.h>

#include "../../sproxy_amd/csrc/md5_tickets.h"

#define CHECK(c)                                                   \
    do {                                                           \
        if (!(c)) {                                                \
            printf("FAIL line %d: %s\n", __LINE__, #c);            \
            return 1;                                              \
        }                                                          \
    } while (0)

static int done(const struct tk_ring *r, uint64_t t, int *err)
{
    *err = 12345;
    return tk_ring_done(r, t, err);
}

int main(void)
{
    struct tk_ring r;
    int err;
    CHECK(tk_ring_init(&r, 1) == 0);
    CHECK(done(&r, 0, &err) == 1 && err == 0);          /* ticket 0: nothing */

    /* a failing submission, then a good synchronous one */
    uint64_t a, b;
    CHECK(tk_ring_new(&r, &a) == 0 && a == 1);
    tk_ring_ref(&r, a);                                  /* one slot holds it */
    tk_ring_put(&r, a, 0);                               /* submission's own ref */
    CHECK(done(&r, a, &err) == 0);                       /* slot still out */
    tk_ring_put(&r, a, -EIO);                            /* the slot fails */
    CHECK(done(&r, a, &err) == 1 && err == -EIO);
    CHECK(r.lo == 2);                                    /* left the ring */
    CHECK(tk_ring_new(&r, &b) == 0 && b == 2);
    tk_ring_ref(&r, b);
    tk_ring_put(&r, b, 0);
    tk_ring_put(&r, b, 0);
    CHECK(done(&r, b, &err) == 1 && err == 0);          /* its own result, not -EIO */
    CHECK(done(&r, a, &err) == 1 && err == -EIO);       /* still its own error */

    /* out-of-order completion over a grown ring, every 7th ticket failing */
    enum { N = 5000 };
    uint64_t id[N];
    for (int i = 0; i < N; i++) {
        CHECK(tk_ring_new(&r, &id[i]) == 0);
        tk_ring_ref(&r, id[i]);
        tk_ring_put(&r, id[i], 0);
    }
    CHECK(r.cap >= N);
    for (int i = N - 1; i >= 0; i -= 2)                  /* odd positions from the top */
        tk_ring_put(&r, id[i], i % 7 == 0 ? -EFAULT : 0);
    for (int i = N - 1; i >= 0; i -= 2) {
        CHECK(done(&r, id[i], &err) == 1);
        CHECK(err == (i % 7 == 0 ? -EFAULT : 0));
    }
    CHECK(done(&r, id[0], &err) == 0);                   /* the ring's low end waits */
    for (int i = 0; i < N; i += 2) tk_ring_put(&r, id[i], i % 7 == 0 ? -ENODEV : 0);
    CHECK(r.lo == r.hi);
    for (int i = 0; i < N; i++) {
        CHECK(done(&r, id[i], &err) == 1);
        const int want = i % 7 ? 0 : (i & 1) ? -EFAULT : -ENODEV;
        CHECK(err == want);
    }
    CHECK(done(&r, a, &err) == 1 && err == -EIO);
    CHECK(done(&r, b, &err) == 1 && err == 0);

    /* only the first error of a ticket is kept */
    uint64_t c;
    CHECK(tk_ring_new(&r, &c) == 0);
    tk_ring_ref(&r, c);
    tk_ring_ref(&r, c);
    tk_ring_put(&r, c, -E2BIG);
    tk_ring_put(&r, c, -EIO);
    tk_ring_put(&r, c, 0);
    CHECK(done(&r, c, &err) == 1 && err == -E2BIG);

    /* the failed list keeps its newest entries past TK_FAILED_MAX */
    uint64_t last = 0;
    for (uint32_t i = 0; i < TK_FAILED_MAX + 10; i++) {
        uint64_t t;
        CHECK(tk_ring_new(&r, &t) == 0);
        tk_ring_put(&r, t, -EIO);
        last = t;
    }
    CHECK(r.nfailed <= TK_FAILED_MAX);
    CHECK(done(&r, last, &err) == 1 && err == -EIO);
    tk_ring_free(&r);
    printf("tickets ok\n");
    return 0;
}
