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

    free(tmp);
    free(heap);
    if (failures) {
        fprintf(stderr, "netcache_site: %d failure(s)\n", failures);
        return 1;
    }
    printf("netcache_site ok: %d blocks (%llu bytes, %d pages scattered), MD5 / CRC-32 / fastcrc / "
           "verify / async / zero-copy x3 / pool / MD5Init-Update-Final / arena+plan / device queue / "
           "device contexts / shared batcher x4 threads bit-exact vs oracle\n",
           nblk, (unsigned long long)inode.size, npages);
    return 0;
}
