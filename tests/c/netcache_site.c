/*
 * tests/c/netcache_site.c -- the netcache block-checksum call site of
 * INTEGRATION.md §2 / §2a / §2e / §2g, compiled as plain C against
 * include/md5hip.h and include/md5.h and linked with libmd5hip.so: no Python,
 * no torch, exactly what sproxy's build would see.
 *
 * The netcache types are reduced to what the call site touches:
 *   fc_blk_t   blkno + pages[i]->memory          (netcache/include/block.h:121, :143-146)
 *   fc_inode_t object size, chunk_size, blockcrc  (netcache.h:262, :408-410)
 *   blk_valid_len                                 (blk_io.c:377: last block is short)
 * Pages are 16 KiB slots carved from one 4 KiB-aligned heap (bc_mgr.c:1260-1290)
 * and handed to blocks in a scrambled order, so a block's pages are scattered.
 *
 * Checked against the oracle (oracle/md5_oracle.c, oracle/crc32_oracle.c,
 * linked in as the checker only) over each block's gathered bytes:
 *   1. MD5 per block through md5_batch_submit_iov
 *   2. netcache CRC-32, whole block and fastcrc head^tail (§2a,
 *      blk_io.c:408-424), stored into inode->blockcrc
 *   3. md5hip_batch_verify_iov flags exactly one corrupted block (§2a,
 *      the blk_io.c:693-703 EAGAIN policy input)
 *   4. md5_batch_submit_iov_async + md5_batch_poll / md5_batch_wait (§2g)
 *   5. zero-copy: md5hip_host_register of the heap, gather modes DEVICE,
 *      DMA, AUTO (§2e)
 *   6. md5hip_pool over device 0 listed twice (§2d): one call, then four
 *      threads submitting asynchronously at once, whole and split
 *   7. MD5Init/Update/Final page by page (the per-message drop-in, §1)
 *   8. the device entry: blocks packed into a batch arena (md5hip_arena_alloc),
 *      order and kernel from md5hip_plan_desc, md5hip_digest_desc_variant
 *   9. the same blocks from the arena through the device-input queue
 *      (md5hip_queue_create, md5_batch_submit_device_async, §2h), digests to
 *      host and to device memory, tickets waited in reverse order
 *  10. MD5Init/Update/Final on one device context per block, one update per
 *      16 KiB page (md5hip_*_ctx, §2i)
 *  11. one batcher shared by four "ASIO" threads, each submitting its blocks
 *      asynchronously and collecting its own tickets (§2, §2g)
 *  12. the failure policy (§2j): a device fault injected into the launch of
 *      an origin-read vector -- the call returns -EIO, no checksum of that
 *      vector is stored (memory-only policy: blocks kept off the disk path),
 *      the next vector gets -ENODEV at once and is hashed on the calling
 *      thread with the library's host CRC-32 (host policy), a cache-read
 *      verify on the failed device resets no inode and falls back the same
 *      way; a pool over device 0 listed twice moves a synchronous vector off
 *      its failed half and returns every checksum, and never routes to it
 *      again
 *
 * Exit 0 = all equal; 1 = a mismatch or error; 77 = no usable HIP device
 * (md5hip_batcher_create returned -ENODEV: the batched entries fail loudly,
 * they never fall back to the host).
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <hip/hip_runtime_api.h>

#include "md5.h"
#include "md5hip.h"
#include "nc_digest.h"

/* oracle (checker) */
void oracle_md5(const void *data, uint64_t len, unsigned char digest[16]);
uint32_t oracle_blk_crc(const void *data, uint64_t remained, uint32_t fastcrc);
void oracle_xorshift_fill(void *dst, uint64_t nbytes, uint64_t seed);

#define NC_PAGE_SIZE 16384u
#define CHUNK_SIZE (4u * NC_PAGE_SIZE) /* netcache chunk_size 64 KiB */
#define PAGES_PER_BLOCK (CHUNK_SIZE / NC_PAGE_SIZE)
#define NBLK_MAX 96

typedef struct { void *memory; } nc_page_t;
typedef struct { uint32_t blkno; nc_page_t *pages[PAGES_PER_BLOCK]; } fc_blk_t;
typedef struct {
    uint64_t size;
    uint32_t chunk_size;
    uint32_t blockcrc[NBLK_MAX];
    unsigned char cascade[NBLK_MAX];   /* block goes on to the disk cache (BS_CACHED_DIRTY, blk_io.c:867-871) */
    int resets;                        /* dm_reset_inode_nolock calls (blk_io.c:693-703) */
} fc_inode_t;

static long long blk_valid_len(const fc_inode_t *inode, const fc_blk_t *blk)
{
    long long off = (long long)blk->blkno * inode->chunk_size;
    long long rem = (long long)inode->size - off;
    return rem < (long long)inode->chunk_size ? rem : (long long)inode->chunk_size;
}

static int failures;
#define CHECK(cond, ...)                                                   \
    do {                                                                   \
        if (!(cond)) {                                                     \
            fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__);           \
            fprintf(stderr, __VA_ARGS__);                                  \
            fputc('\n', stderr);                                           \
            failures++;                                                    \
        }                                                                  \
    } while (0)

/* page list of every block -> segments + seg_first */
static uint64_t blk_segments(const fc_inode_t *inode, fc_blk_t *const *blks, int nblk,
                             struct md5hip_iov *segs, uint64_t *first)
{
    uint64_t ns = 0;
    for (int b = 0; b < nblk; b++) {
        long long remained = blk_valid_len(inode, blks[b]);
        first[b] = ns;
        for (int p = 0; remained > 0; p++) {
            uint32_t take = remained < NC_PAGE_SIZE ? (uint32_t)remained : NC_PAGE_SIZE;
            segs[ns].base = blks[b]->pages[p]->memory;
            segs[ns].len = take;
            ns++;
            remained -= take;
        }
    }
    first[nblk] = ns;
    return ns;
}

/* §11: one "ASIO" thread of a pool sharing one batcher */
struct asio_job {
    md5hip_batcher *b;
    const struct md5hip_iov *segs;
    const uint64_t *first;
    int lo, hi, reps;
    unsigned char (*want)[16];
    int bad, rc;
};

static void *asio_thread(void *arg)
{
    struct asio_job *j = arg;
    unsigned char dig[8][NBLK_MAX][16];
    uint64_t tk[8];
    uint64_t rebased[NBLK_MAX + 1];
    for (int b = j->lo; b <= j->hi; b++) rebased[b - j->lo] = j->first[b] - j->first[j->lo];
    for (int r = 0; r < j->reps; r++) {
        const int rc = md5_batch_submit_iov_async(j->b, j->segs + j->first[j->lo], rebased,
                                                  (uint64_t)(j->hi - j->lo), &dig[r][0][0], &tk[r]);
        if (rc && !j->rc) j->rc = rc;
    }
    for (int r = j->reps - 1; r >= 0; r--) {        /* tickets in reverse: out-of-order completion */
        const int rc = md5_batch_wait(j->b, tk[r]);
        if (rc && !j->rc) j->rc = rc;
        for (int b = j->lo; b < j->hi; b++) j->bad += memcmp(dig[r][b - j->lo], j->want[b], 16) != 0;
    }
    return NULL;
}

/* §2d: one "ASIO" thread submitting its vectors into the shared pool */
struct pool_job {
    md5hip_pool *p;
    const struct md5hip_iov *segs;
    const uint64_t *first;
    int lo, hi, reps;
    unsigned char (*want)[16];
    int bad, rc;
};

static void *pool_thread(void *arg)
{
    struct pool_job *j = arg;
    unsigned char dig[8][NBLK_MAX][16];
    uint64_t tk[8];
    uint64_t rebased[NBLK_MAX + 1];
    for (int b = j->lo; b <= j->hi; b++) rebased[b - j->lo] = j->first[b] - j->first[j->lo];
    for (int r = 0; r < j->reps; r++) {
        const int rc = md5hip_pool_submit_iov_async(j->p, j->segs + j->first[j->lo], rebased,
                                                    (uint64_t)(j->hi - j->lo), &dig[r][0][0], &tk[r]);
        if (rc && !j->rc) j->rc = rc;
    }
    for (int r = j->reps - 1; r >= 0; r--) {        /* any order */
        const int rc = md5hip_pool_wait(j->p, tk[r]);
        if (rc && !j->rc) j->rc = rc;
        for (int b = j->lo; b < j->hi; b++) j->bad += memcmp(dig[r][b - j->lo], j->want[b], 16) != 0;
    }
    return NULL;
}

/* ----------------------------------------------------------- §2j bindings */
enum { POLICY_HOST = 0, POLICY_MEMORY_ONLY = 1 };

/* the library's host CRC-32 of one block (product code, not the oracle):
 * what the site computes on the calling thread when the device cannot */
static uint32_t host_blk_crc(const struct md5hip_iov *segs, uint64_t s0, uint64_t s1, uint32_t fastcrc,
                             unsigned char *tmp)
{
    uint64_t L = 0;
    for (uint64_t s = s0; s < s1; s++) {
        memcpy(tmp + L, segs[s].base, segs[s].len);
        L += segs[s].len;
    }
    if (fastcrc == 0 || L <= fastcrc) return nc_crc32(tmp, L);           /* blk_io.c:408-424 */
    return nc_crc32(tmp, fastcrc) ^ nc_crc32(tmp + (L - fastcrc), fastcrc);
}

/* origin read (blk_io.c:851-863) as INTEGRATION.md §2j binds it: a checksum
 * is stored only from a call that returned 0 or from the site's own host
 * code; a device error is never stored as a checksum.  Returns the batched
 * call's rc. */
static int origin_read_vector(md5hip_batcher *b, fc_inode_t *inode, fc_blk_t *const *blks, int lo, int hi,
                              const struct md5hip_iov *segs, const uint64_t *first, int policy,
                              uint32_t *crc_out, unsigned char *tmp)
{
    const int n = hi - lo;
    uint64_t rebased[NBLK_MAX + 1];
    for (int k = 0; k <= n; k++) rebased[k] = first[lo + k] - first[lo];
    const int rc = md5_batch_submit_iov(b, segs + first[lo], rebased, (uint64_t)n, (unsigned char *)crc_out);
    if (rc == 0) {
        for (int k = 0; k < n; k++) {
            inode->blockcrc[blks[lo + k]->blkno] = crc_out[k];      /* dm_update_block_crc_nolock */
            inode->cascade[blks[lo + k]->blkno] = 1;
        }
        return 0;
    }
    for (int k = 0; k < n; k++) {
        if (policy == POLICY_HOST) {
            inode->blockcrc[blks[lo + k]->blkno] = host_blk_crc(segs, first[lo + k], first[lo + k + 1], 0, tmp);
            inode->cascade[blks[lo + k]->blkno] = 1;
        } else {
            inode->cascade[blks[lo + k]->blkno] = 0;                /* BS_CACHED: memory only */
        }
    }
    return rc;
}

/* cache read (blk_io.c:665-704): a mismatch resets the inode; a device error
 * is not a mismatch -- the vector is verified on the calling thread instead.
 * Returns the number of mismatching blocks. */
static int cache_read_verify(md5hip_batcher *b, fc_inode_t *inode, fc_blk_t *const *blks, int nb,
                             const struct md5hip_iov *segs, const uint64_t *first, unsigned char *ok,
                             unsigned char *tmp, int *device_rc)
{
    uint32_t want[NBLK_MAX] = {0};
    for (int k = 0; k < nb; k++) want[k] = inode->blockcrc[blks[k]->blkno];
    int bad = md5hip_batch_verify_iov(b, segs, first, (uint64_t)nb, want, ok);
    *device_rc = bad < 0 ? bad : 0;
    if (bad < 0) {
        bad = 0;
        for (int k = 0; k < nb; k++) {
            ok[k] = host_blk_crc(segs, first[k], first[k + 1], 0, tmp) == want[k];   /* dm_verify_block_crc */
            bad += !ok[k];
        }
    }
    for (int k = 0; k < nb; k++)
        if (!ok[k]) inode->resets++;                                  /* EAGAIN + dm_reset_inode_nolock */
    return bad;
}

static int failure_pass(fc_inode_t *inode, fc_blk_t *const *blks, int nblk, const struct md5hip_iov *segs,
                        const uint64_t *first, const uint32_t *want_crc, const unsigned char (*want_md5)[16],
                        unsigned char *tmp)
{
    const int nf0 = failures;
    md5hip_batcher *b = NULL;
    int rc = md5hip_batcher_create(0, 16u << 20, 3, &b);
    CHECK(rc == 0, "failure batcher = %d", rc);
    if (rc) return 1;
    CHECK(md5hip_batcher_set_digest(b, MD5HIP_DIGEST_CRC32, 0) == 0, "set CRC-32");
    const uint32_t SENT = 0xdeadbeefu;
    for (int k = 0; k < nblk; k++) inode->blockcrc[k] = SENT, inode->cascade[k] = 1;
    uint32_t crc[NBLK_MAX];
    const int half = nblk / 2;

    /* a healthy vector first */
    rc = origin_read_vector(b, inode, blks, 0, 8, segs, first, POLICY_MEMORY_ONLY, crc, tmp);
    CHECK(rc == 0, "healthy vector %d", rc);
    for (int k = 0; k < 8; k++) CHECK(inode->blockcrc[k] == want_crc[k], "healthy crc %d", k);

    /* A: the device faults under this vector's launch */
    CHECK(md5hip_batcher_inject_fault(b, 1) == 0, "inject");
    for (int k = 0; k < NBLK_MAX; k++) crc[k] = SENT;
    rc = origin_read_vector(b, inode, blks, 8, half, segs, first, POLICY_MEMORY_ONLY, crc, tmp);
    CHECK(rc == -EIO, "faulting vector: rc %d, want -EIO", rc);
    for (int k = 8; k < half; k++) {
        CHECK(crc[k - 8] == SENT, "device wrote a checksum for failed block %d", k);
        CHECK(inode->blockcrc[k] == SENT, "a checksum was stored for failed block %d", k);
        CHECK(inode->cascade[k] == 0, "failed block %d still goes to disk", k);
    }
    CHECK(md5hip_batcher_health(b) == -ENODEV, "batcher not failed: %d", md5hip_batcher_health(b));

    /* B: the next vector is refused at once and hashed on the calling thread */
    rc = origin_read_vector(b, inode, blks, half, nblk, segs, first, POLICY_HOST, crc, tmp);
    CHECK(rc == -ENODEV, "next vector: rc %d, want -ENODEV", rc);
    for (int k = half; k < nblk; k++) {
        CHECK(inode->blockcrc[k] == want_crc[k], "host fallback crc %d", k);
        CHECK(inode->cascade[k] == 1, "host-fallback block %d kept off disk", k);
    }

    /* C: cache read on the failed device: no inode reset from the device
     * error; one really corrupted block is still caught (host verify) */
    unsigned char ok[NBLK_MAX];
    int drc = 0;
    const int nb = nblk - half;
    uint64_t rebased[NBLK_MAX + 1];
    for (int k = 0; k <= nb; k++) rebased[k] = first[half + k] - first[half];
    inode->resets = 0;
    int bad = cache_read_verify(b, inode, blks + half, nb, segs + first[half], rebased, ok, tmp, &drc);
    CHECK(drc == -ENODEV && bad == 0 && inode->resets == 0, "verify on a failed device: rc %d bad %d resets %d",
          drc, bad, inode->resets);
    unsigned char *victim = (unsigned char *)blks[half + 3]->pages[1]->memory + 99;
    *victim ^= 0x08;
    bad = cache_read_verify(b, inode, blks + half, nb, segs + first[half], rebased, ok, tmp, &drc);
    *victim ^= 0x08;
    CHECK(bad == 1 && !ok[3] && inode->resets == 1, "host verify: bad %d ok[3] %d resets %d", bad, ok[3],
          inode->resets);
    md5hip_batcher_destroy(b);

    /* D: a pool over device 0 listed twice; its half 0 faults under a
     * synchronous vector split over both halves */
    md5hip_pool *pool = NULL;
    const int devs[2] = {0, 0};
    rc = md5hip_pool_create(devs, 2, 16u << 20, 3, &pool);
    CHECK(rc == 0, "failure pool = %d", rc);
    if (rc) return 1;
    CHECK(md5hip_pool_set_split(pool, 64u << 10) == 0, "split");
    CHECK(md5hip_pool_inject_fault(pool, 0, 1) == 0, "pool inject");
    static unsigned char digest[NBLK_MAX][16];
    memset(digest, 0, sizeof digest);
    rc = md5hip_pool_submit_iov(pool, segs, first, (uint64_t)nblk, &digest[0][0]);
    CHECK(rc == 0, "pool vector with a failed device: %d", rc);
    for (int k = 0; k < nblk; k++) CHECK(memcmp(digest[k], want_md5[k], 16) == 0, "pool failover block %d", k);
    struct md5hip_pool_health h;
    CHECK(md5hip_pool_get_health(pool, &h) == 0 && h.nfailed == 1 && h.failed_mask == 1 && h.failovers == 1,
          "pool health: nfailed %u mask %llx failovers %llu", h.nfailed, (unsigned long long)h.failed_mask,
          (unsigned long long)h.failovers);
    struct md5hip_batcher_stats s0, s1;
    md5hip_pool_device_stats(pool, 0, &s0);
    for (int r = 0; r < 4; r++) {
        memset(digest, 0, sizeof digest);
        rc = md5hip_pool_submit_iov(pool, segs, first, (uint64_t)nblk, &digest[0][0]);
        CHECK(rc == 0, "pool after the fault: %d", rc);
        for (int k = 0; k < nblk; k++) CHECK(memcmp(digest[k], want_md5[k], 16) == 0, "pool after, block %d", k);
    }
    md5hip_pool_device_stats(pool, 0, &s1);
    CHECK(s1.launches == s0.launches && s1.submissions == s0.submissions, "the failed half was used again");
    md5hip_pool_destroy(pool);
    return failures != nf0;
}

/* the block's bytes, gathered on the host for the oracle */
static void gather(const fc_inode_t *inode, const fc_blk_t *blk, unsigned char *dst)
{
    long long remained = blk_valid_len(inode, blk);
    for (int p = 0; remained > 0; p++) {
        uint32_t take = remained < NC_PAGE_SIZE ? (uint32_t)remained : NC_PAGE_SIZE;
        memcpy(dst + (size_t)p * NC_PAGE_SIZE, blk->pages[p]->memory, take);
        remained -= take;
    }
}

int main(void)
{
    /* an object of 83 full 64 KiB blocks plus a 12,345-byte last block */
    const int nblk = 84;
    fc_inode_t inode;
    memset(&inode, 0, sizeof inode);
    inode.chunk_size = CHUNK_SIZE;
    inode.size = (uint64_t)(nblk - 1) * CHUNK_SIZE + 12345u;

    const int npages = nblk * (int)PAGES_PER_BLOCK;
    const size_t heap_bytes = (size_t)npages * NC_PAGE_SIZE;
    unsigned char *heap = NULL;
    if (posix_memalign((void **)&heap, 4096, heap_bytes) != 0) return 1;
    oracle_xorshift_fill(heap, heap_bytes, 0x6e63ull);

    /* scatter: page slot k goes to position (k * 37) mod npages (37 is coprime to npages) */
    static nc_page_t pages[NBLK_MAX * PAGES_PER_BLOCK];
    static fc_blk_t blkstore[NBLK_MAX];
    fc_blk_t *blks[NBLK_MAX];
    for (int k = 0; k < npages; k++)
        pages[k].memory = heap + (size_t)((k * 37) % npages) * NC_PAGE_SIZE;
    for (int b = 0; b < nblk; b++) {
        blkstore[b].blkno = (uint32_t)b;
        for (unsigned p = 0; p < PAGES_PER_BLOCK; p++)
            blkstore[b].pages[p] = &pages[b * PAGES_PER_BLOCK + p];
        blks[b] = &blkstore[b];
    }

    static struct md5hip_iov segs[NBLK_MAX * PAGES_PER_BLOCK];
    uint64_t first[NBLK_MAX + 1];
    blk_segments(&inode, blks, nblk, segs, first);

    /* expected values from the oracle over each block's gathered bytes */
    static unsigned char want_md5[NBLK_MAX][16];
    static uint32_t want_crc[NBLK_MAX], want_fast[NBLK_MAX];
    unsigned char *tmp = malloc(CHUNK_SIZE);
    if (!tmp) return 1;
    for (int b = 0; b < nblk; b++) {
        long long len = blk_valid_len(&inode, blks[b]);
        gather(&inode, blks[b], tmp);
        oracle_md5(tmp, (uint64_t)len, want_md5[b]);
        want_crc[b] = oracle_blk_crc(tmp, (uint64_t)len, 0);
        want_fast[b] = oracle_blk_crc(tmp, (uint64_t)len, 4096);
    }

    md5hip_batcher *t_md5 = NULL;
    int rc = md5hip_batcher_create(0, 64u << 20, 3, &t_md5); /* INTEGRATION §2 */
    if (rc == -ENODEV) {
        printf("netcache_site: no usable HIP device (md5hip_batcher_create = %d)\n", rc);
        return 77;
    }
    CHECK(rc == 0 && t_md5, "md5hip_batcher_create = %d", rc);
    if (rc != 0) return 1;

    /* 1. MD5 per block */
    static unsigned char digest[NBLK_MAX][16];
    memset(digest, 0, sizeof digest);
    rc = md5_batch_submit_iov(t_md5, segs, first, (uint64_t)nblk, &digest[0][0]);
    CHECK(rc == 0, "md5_batch_submit_iov = %d", rc);
    for (int b = 0; b < nblk; b++)
        CHECK(memcmp(digest[b], want_md5[b], 16) == 0, "MD5 block %d", b);

    /* 2. netcache CRC-32, whole block then fastcrc window */
    uint32_t crc[NBLK_MAX];
    rc = md5hip_batcher_set_digest(t_md5, MD5HIP_DIGEST_CRC32, 0);
    CHECK(rc == 0, "set_digest(CRC32, 0) = %d", rc);
    rc = md5_batch_submit_iov(t_md5, segs, first, (uint64_t)nblk, (unsigned char *)crc);
    CHECK(rc == 0, "CRC submit = %d", rc);
    for (int b = 0; b < nblk; b++) {
        CHECK(crc[b] == want_crc[b], "CRC block %d: %08x vs %08x", b, crc[b], want_crc[b]);
        inode.blockcrc[blks[b]->blkno] = crc[b]; /* dm_update_block_crc_nolock */
    }
    rc = md5hip_batcher_set_digest(t_md5, MD5HIP_DIGEST_CRC32, 4096);
    CHECK(rc == 0, "set_digest(CRC32, 4096) = %d", rc);
    rc = md5_batch_submit_iov(t_md5, segs, first, (uint64_t)nblk, (unsigned char *)crc);
    CHECK(rc == 0, "fastcrc submit = %d", rc);
    for (int b = 0; b < nblk; b++)
        CHECK(crc[b] == want_fast[b], "fastcrc block %d: %08x vs %08x", b, crc[b], want_fast[b]);

    /* 3. verify against the stored array with one corrupted block */
    rc = md5hip_batcher_set_digest(t_md5, MD5HIP_DIGEST_CRC32, 0);
    CHECK(rc == 0, "set_digest = %d", rc);
    uint32_t want[NBLK_MAX];
    unsigned char ok[NBLK_MAX];
    for (int b = 0; b < nblk; b++) want[b] = inode.blockcrc[blks[b]->blkno];
    unsigned char *victim = (unsigned char *)blks[5]->pages[2]->memory + 777;
    *victim ^= 0x40;
    rc = md5hip_batch_verify_iov(t_md5, segs, first, (uint64_t)nblk, want, ok);
    CHECK(rc == 1, "verify mismatches = %d, want 1", rc);
    for (int b = 0; b < nblk; b++) CHECK(ok[b] == (b != 5), "verify ok[%d] = %d", b, ok[b]);
    *victim ^= 0x40;
    rc = md5hip_batch_verify_iov(t_md5, segs, first, (uint64_t)nblk, want, ok);
    CHECK(rc == 0, "verify after restore = %d", rc);

    /* 4. asynchronous submit: two block vectors in flight, poll then wait */
    rc = md5hip_batcher_set_digest(t_md5, MD5HIP_DIGEST_MD5, 0);
    CHECK(rc == 0, "set_digest(MD5) = %d", rc);
    static unsigned char da[NBLK_MAX][16], db[NBLK_MAX][16];
    memset(da, 0, sizeof da);
    memset(db, 0, sizeof db);
    const int half = nblk / 2;
    uint64_t t1 = 0, t2 = 0;
    uint64_t first_b[NBLK_MAX + 1];
    for (int b = half; b <= nblk; b++) first_b[b - half] = first[b] - first[half];
    rc = md5_batch_submit_iov_async(t_md5, segs, first, (uint64_t)half, &da[0][0], &t1);
    CHECK(rc == 0, "submit_iov_async(1) = %d", rc);
    rc = md5_batch_submit_iov_async(t_md5, segs + first[half], first_b, (uint64_t)(nblk - half),
                                    &db[0][0], &t2);
    CHECK(rc == 0, "submit_iov_async(2) = %d", rc);
    int polled = 0;
    for (int spin = 0; spin < 200000 && (polled = md5_batch_poll(t_md5, t1)) == 0; spin++)
        usleep(50); /* bounded: ~10 s */
    CHECK(polled == 1, "md5_batch_poll(t1) = %d", polled);
    rc = md5_batch_wait(t_md5, t2);
    CHECK(rc == 0, "md5_batch_wait(t2) = %d", rc);
    for (int b = 0; b < half; b++) CHECK(memcmp(da[b], want_md5[b], 16) == 0, "async A %d", b);
    for (int b = half; b < nblk; b++)
        CHECK(memcmp(db[b - half], want_md5[b], 16) == 0, "async B %d", b);

    /* 5. zero-copy: register the page heap, every gather mode */
    rc = md5hip_host_register(heap, heap_bytes);
    CHECK(rc == 0, "md5hip_host_register = %d", rc);
    const int modes[3] = {MD5HIP_GATHER_DEVICE, MD5HIP_GATHER_DMA, MD5HIP_GATHER_AUTO};
    for (int k = 0; k < 3; k++) {
        rc = md5hip_batcher_set_gather(t_md5, modes[k]);
        CHECK(rc == 0, "set_gather(%d) = %d", modes[k], rc);
        memset(digest, 0, sizeof digest);
        rc = md5_batch_submit_iov(t_md5, segs, first, (uint64_t)nblk, &digest[0][0]);
        CHECK(rc == 0, "zero-copy submit mode %d = %d", modes[k], rc);
        for (int b = 0; b < nblk; b++)
            CHECK(memcmp(digest[b], want_md5[b], 16) == 0, "zero-copy mode %d block %d", modes[k], b);
    }
    md5hip_batcher_destroy(t_md5);
    rc = md5hip_host_unregister(heap);
    CHECK(rc == 0, "md5hip_host_unregister = %d", rc);

    /* 6. pool over device 0 listed twice: each half writes its own slice */
    md5hip_pool *pool = NULL;
    const int devs[2] = {0, 0};
    rc = md5hip_pool_create(devs, 2, 64u << 20, 3, &pool);
    CHECK(rc == 0 && pool, "md5hip_pool_create = %d", rc);
    if (rc == 0) {
        CHECK(md5hip_pool_ndev(pool) == 2, "pool ndev %d", md5hip_pool_ndev(pool));
        memset(digest, 0, sizeof digest);
        rc = md5hip_pool_submit_iov(pool, segs, first, (uint64_t)nblk, &digest[0][0]);
        CHECK(rc == 0, "md5hip_pool_submit_iov = %d", rc);
        for (int b = 0; b < nblk; b++)
            CHECK(memcmp(digest[b], want_md5[b], 16) == 0, "pool block %d", b);
        /* four ASIO threads at once, no lock of their own: each vector goes
         * whole to one batcher; then the same with a split threshold below
         * a vector, so every vector is cut over both */
        for (int split = 0; split < 2; split++) {
            if (split) {
                rc = md5hip_pool_set_split(pool, 1u << 20);
                CHECK(rc == 0, "md5hip_pool_set_split = %d", rc);
            }
            struct pool_job pj[4];
            pthread_t pth[4];
            for (int t = 0; t < 4; t++) {
                pj[t] = (struct pool_job){pool, segs, first, t * nblk / 4, (t + 1) * nblk / 4, 3,
                                          want_md5, 0, 0};
                if (pthread_create(&pth[t], NULL, pool_thread, &pj[t]) != 0) pth[t] = 0;
            }
            for (int t = 0; t < 4; t++) {
                if (pth[t]) pthread_join(pth[t], NULL);
                else pool_thread(&pj[t]);
                CHECK(pj[t].rc == 0 && pj[t].bad == 0, "pool thread %d (split %d): rc %d, bad %d", t,
                      split, pj[t].rc, pj[t].bad);
            }
        }
        struct md5hip_pool_stats pst;
        rc = md5hip_pool_get_stats(pool, &pst);
        CHECK(rc == 0 && pst.routed_whole >= 13 && pst.split == 12,
              "pool stats rc %d whole %llu split %llu", rc, (unsigned long long)pst.routed_whole,
              (unsigned long long)pst.split);
        md5hip_pool_destroy(pool);
    }

    /* 7. per-message drop-in, one MD5Update per page (md5.h:41-51) */
    for (int b = 0; b < nblk; b += 41) {
        struct MD5Context ctx;
        unsigned char d[MD5_DIGEST_SIZE];
        MD5Init(&ctx);
        for (uint64_t s = first[b]; s < first[b + 1]; s++)
            MD5Update(&ctx, segs[s].base, segs[s].len);
        MD5Final(d, &ctx);
        CHECK(memcmp(d, want_md5[b], 16) == 0, "MD5Init/Update/Final block %d", b);
    }

    /* 8. device-resident producer: the blocks packed into a
     * batch arena, planned on the host, hashed by the device entry */
    {
        void *d_arena = NULL, *d_off = NULL, *d_len = NULL, *d_ord = NULL, *d_dig = NULL;
        uint64_t offs[NBLK_MAX], at = 0;
        uint32_t lens[NBLK_MAX], order[NBLK_MAX];
        for (int b = 0; b < nblk; b++) {
            lens[b] = (uint32_t)blk_valid_len(&inode, blks[b]);
            offs[b] = at;
            at += (lens[b] + 15u) & ~15u;
        }
        rc = md5hip_arena_alloc(0, at + 64, &d_arena);
        CHECK(rc == 0 && d_arena && ((uintptr_t)d_arena & ((1u << 30) - 1)) == 0,
              "md5hip_arena_alloc = %d", rc);
        const int var = md5hip_plan_desc(lens, (uint64_t)nblk, order);
        CHECK(var >= 0, "md5hip_plan_desc = %d", var);
        int ok = rc == 0 && var >= 0 &&
                 hipMalloc(&d_off, sizeof offs) == hipSuccess &&
                 hipMalloc(&d_len, sizeof lens) == hipSuccess &&
                 hipMalloc(&d_ord, sizeof order) == hipSuccess &&
                 hipMalloc(&d_dig, 16 * NBLK_MAX) == hipSuccess;
        for (int b = 0; ok && b < nblk; b++) {
            gather(&inode, blks[b], tmp);
            ok = hipMemcpy((unsigned char *)d_arena + offs[b], tmp, lens[b],
                           hipMemcpyHostToDevice) == hipSuccess;
        }
        ok = ok && hipMemcpy(d_off, offs, sizeof offs, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(d_len, lens, sizeof lens, hipMemcpyHostToDevice) == hipSuccess &&
             hipMemcpy(d_ord, order, sizeof order, hipMemcpyHostToDevice) == hipSuccess;
        CHECK(ok, "arena staging");
        if (ok) {
            rc = md5hip_digest_desc_variant(d_arena, d_off, d_len, d_ord, (uint64_t)nblk, d_dig,
                                            NULL, var);
            CHECK(rc == 0, "md5hip_digest_desc_variant(%d) = %d", var, rc);
            memset(digest, 0, sizeof digest);
            CHECK(hipMemcpy(digest, d_dig, 16 * (size_t)nblk, hipMemcpyDeviceToHost) == hipSuccess,
                  "digest copy");
            for (int b = 0; b < nblk; b++)
                CHECK(memcmp(digest[b], want_md5[b], 16) == 0, "arena block %d", b);

            /* 9. the device-input queue over the same arena */
            md5hip_batcher *q = NULL;
            rc = md5hip_queue_create(0, 0, 3, &q);
            CHECK(rc == 0 && q, "md5hip_queue_create = %d", rc);
            if (rc == 0) {
                uint64_t addr[NBLK_MAX], t_h = 0, t_d = 0;
                for (int b = 0; b < nblk; b++) addr[b] = (uint64_t)(uintptr_t)d_arena + offs[b];
                memset(digest, 0, sizeof digest);
                (void)hipMemset(d_dig, 0, 16 * NBLK_MAX);
                rc = md5_batch_submit_device_async(q, addr, lens, (uint64_t)nblk, &digest[0][0], 0, &t_h);
                CHECK(rc == 0, "submit_device_async(host digests) = %d", rc);
                rc = md5_batch_submit_device_async(q, addr, lens, (uint64_t)nblk, d_dig, 1, &t_d);
                CHECK(rc == 0, "submit_device_async(device digests) = %d", rc);
                CHECK(md5_batch_wait(q, t_d) == 0 && md5_batch_wait(q, t_h) == 0, "queue waits");
                for (int b = 0; b < nblk; b++)
                    CHECK(memcmp(digest[b], want_md5[b], 16) == 0, "queue host digest %d", b);
                memset(digest, 0, sizeof digest);
                CHECK(hipMemcpy(digest, d_dig, 16 * (size_t)nblk, hipMemcpyDeviceToHost) == hipSuccess,
                      "queue digest copy");
                for (int b = 0; b < nblk; b++)
                    CHECK(memcmp(digest[b], want_md5[b], 16) == 0, "queue device digest %d", b);
                md5hip_batcher_destroy(q);
            }

            /* 10. one device context per block, one MD5Update per 16 KiB page */
            void *d_ctx = NULL, *d_ptr = NULL, *d_pl = NULL;
            ok = hipMalloc(&d_ctx, 88 * NBLK_MAX) == hipSuccess &&
                 hipMalloc(&d_ptr, 8 * NBLK_MAX) == hipSuccess &&
                 hipMalloc(&d_pl, 4 * NBLK_MAX) == hipSuccess;
            CHECK(ok, "context buffers");
            if (ok) {
                CHECK(md5hip_init_ctx(d_ctx, (uint64_t)nblk, NULL) == 0, "md5hip_init_ctx");
                for (unsigned p = 0; p < PAGES_PER_BLOCK; p++) {
                    uint64_t ptr[NBLK_MAX];
                    uint32_t pl[NBLK_MAX];
                    for (int b = 0; b < nblk; b++) {
                        const long long rem = (long long)lens[b] - (long long)p * NC_PAGE_SIZE;
                        pl[b] = rem <= 0 ? 0u : rem < NC_PAGE_SIZE ? (uint32_t)rem : NC_PAGE_SIZE;
                        ptr[b] = (uint64_t)(uintptr_t)d_arena + offs[b] + (uint64_t)p * NC_PAGE_SIZE;
                    }
                    CHECK(hipMemcpy(d_ptr, ptr, 8 * (size_t)nblk, hipMemcpyHostToDevice) == hipSuccess &&
                          hipMemcpy(d_pl, pl, 4 * (size_t)nblk, hipMemcpyHostToDevice) == hipSuccess,
                          "page descriptors");
                    CHECK(md5hip_update_ctx(d_ctx, (const void *const *)d_ptr, d_pl, (uint64_t)nblk,
                                            NULL) == 0, "md5hip_update_ctx page %u", p);
                }
                CHECK(md5hip_final_ctx(d_ctx, (uint64_t)nblk, d_dig, NULL) == 0, "md5hip_final_ctx");
                memset(digest, 0, sizeof digest);
                CHECK(hipMemcpy(digest, d_dig, 16 * (size_t)nblk, hipMemcpyDeviceToHost) == hipSuccess,
                      "ctx digest copy");
                for (int b = 0; b < nblk; b++)
                    CHECK(memcmp(digest[b], want_md5[b], 16) == 0, "context block %d", b);
            }
            (void)hipFree(d_ctx);
            (void)hipFree(d_ptr);
            (void)hipFree(d_pl);
        }
        (void)hipFree(d_off);
        (void)hipFree(d_len);
        (void)hipFree(d_ord);
        (void)hipFree(d_dig);
        if (d_arena) CHECK(md5hip_arena_free(d_arena) == 0, "md5hip_arena_free");
    }

    /* 11. four "ASIO" threads share one batcher */
    {
        md5hip_batcher *shared = NULL;
        rc = md5hip_batcher_create(0, 16u << 20, 4, &shared);
        CHECK(rc == 0 && shared, "shared batcher = %d", rc);
        if (rc == 0) {
            struct asio_job jobs[4];
            pthread_t th[4];
            for (int t = 0; t < 4; t++) {
                jobs[t] = (struct asio_job){shared, segs, first, t * nblk / 4, (t + 1) * nblk / 4, 8,
                                            want_md5, 0, 0};
                CHECK(pthread_create(&th[t], NULL, asio_thread, &jobs[t]) == 0, "pthread_create");
            }
            for (int t = 0; t < 4; t++) {
                pthread_join(th[t], NULL);
                CHECK(jobs[t].rc == 0 && jobs[t].bad == 0, "asio thread %d: rc %d, %d bad", t,
                      jobs[t].rc, jobs[t].bad);
            }
            struct md5hip_batcher_stats st;
            CHECK(md5hip_batcher_get_stats(shared, &st) == 0 && st.submissions == 32,
                  "shared batcher stats");
            md5hip_batcher_destroy(shared);
        }
    }

    /* 12. the failure policy (§2j) */
    (void)failure_pass(&inode, blks, nblk, segs, first, want_crc, (const unsigned char (*)[16])want_md5, tmp);

    free(tmp);
    free(heap);
    if (failures) {
        fprintf(stderr, "netcache_site: %d failure(s)\n", failures);
        return 1;
    }
    printf("netcache_site ok: %d blocks (%llu bytes, %d pages scattered), MD5 / CRC-32 / fastcrc / "
           "verify / async / zero-copy x3 / pool / MD5Init-Update-Final / arena+plan / device queue / "
           "device contexts / shared batcher x4 threads bit-exact vs oracle; failure policy ok\n",
           nblk, (unsigned long long)inode.size, npages);
    return 0;
}
