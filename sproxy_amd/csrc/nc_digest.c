/*
 * nc_digest.c -- per-block digest array and header CRC of netcache's on-disk
 * object header (include/nc_digest.h).
 */
#include <errno.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/nc_digest.h"
#include "../../include/md5hip.h"
#include "md5_internal.h"

uint64_t nc_canned_digest_size(uint32_t bitmaplen, uint32_t dsz)
{
    return ((uint64_t)bitmaplen * dsz + 7) / 8 * 8;           /* NC_ALIGNED_SIZE(.., 8) */
}

static int entry_fits(uint64_t arr_size, uint32_t dsz, uint64_t blkno)
{
    return dsz && blkno < arr_size / dsz;                      /* (blkno+1)*dsz <= arr_size */
}

int nc_digest_update(void *arr, uint64_t arr_size, uint32_t dsz, uint64_t mapped, uint64_t blkno,
                     const void *digest)
{
    if (!arr || !digest || dsz == 0) return -EINVAL;
    if (blkno >= mapped) return -ERANGE;
    if (!entry_fits(arr_size, dsz, blkno)) return -E2BIG;
    memcpy((unsigned char *)arr + blkno * dsz, digest, dsz);
    return 0;
}

int nc_digest_verify(const void *arr, uint64_t arr_size, uint32_t dsz, uint64_t blkno,
                     const void *digest)
{
    if (!arr || !digest || dsz == 0) return -EINVAL;
    if (!entry_fits(arr_size, dsz, blkno)) return -ERANGE;
    return memcmp((const unsigned char *)arr + blkno * dsz, digest, dsz) == 0;
}

int nc_digest_scatter(void *arr, uint64_t arr_size, uint32_t dsz, uint64_t mapped,
                      const uint64_t *blknos, uint64_t n, const void *digests)
{
    if (n == 0) return 0;
    if (!arr || !blknos || !digests || dsz == 0) return -EINVAL;
    int rejected = 0;
    for (uint64_t i = 0; i < n; i++)
        rejected += nc_digest_update(arr, arr_size, dsz, mapped, blknos[i],
                                     (const unsigned char *)digests + i * dsz) != 0;
    return rejected;
}

int nc_digest_compare(const void *arr, uint64_t arr_size, uint32_t dsz, const uint64_t *blknos,
                      uint64_t n, const void *digests, unsigned char *ok)
{
    if (n == 0) return 0;
    if (!arr || !blknos || !digests || !ok || dsz == 0) return -EINVAL;
    int bad = 0;
    for (uint64_t i = 0; i < n; i++) {
        ok[i] = nc_digest_verify(arr, arr_size, dsz, blknos[i],
                                 (const unsigned char *)digests + i * dsz) == 1;
        bad += !ok[i];
    }
    return bad;
}

/* ---------------------------------------------------------------- CRC-32 --
 * Reflected polynomial 0xEDB88320 (crc32.c:22), init ~0, final ~, eight
 * 256-entry tables processed 8 bytes at a time (crc32.c:186-240). */
static uint32_t crc_tab[8][256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;

static void crc_init(void)
{
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
        crc_tab[0][i] = c;
    }
    for (uint32_t i = 0; i < 256; i++)
        for (int s = 1; s < 8; s++) crc_tab[s][i] = (crc_tab[s - 1][i] >> 8) ^ crc_tab[0][crc_tab[s - 1][i] & 0xFF];
}

static uint32_t crc_run(uint32_t c, const unsigned char *p, uint64_t len)
{
    while (len >= 8) {
        uint32_t lo, hi;
        memcpy(&lo, p, 4);
        memcpy(&hi, p + 4, 4);
        lo ^= c;
        c = crc_tab[7][lo & 0xFF] ^ crc_tab[6][(lo >> 8) & 0xFF] ^ crc_tab[5][(lo >> 16) & 0xFF] ^
            crc_tab[4][lo >> 24] ^ crc_tab[3][hi & 0xFF] ^ crc_tab[2][(hi >> 8) & 0xFF] ^
            crc_tab[1][(hi >> 16) & 0xFF] ^ crc_tab[0][hi >> 24];
        p += 8;
        len -= 8;
    }
    while (len--) c = crc_tab[0][(c ^ *p++) & 0xFF] ^ (c >> 8);
    return c;
}

uint32_t nc_crc32(const void *data, uint64_t len)
{
    pthread_once(&crc_once, crc_init);
    return ~crc_run(0xFFFFFFFFu, (const unsigned char *)data, data ? len : 0);
}

static int32_t hdr_size(const void *header)
{
    int32_t hs;
    memcpy(&hs, (const unsigned char *)header + NC_HDR_OFF_HEADER_SIZE, 4);
    return hs;
}

/* The pieces dm_verify_header CRCs (diskcache.c:3676-3686): the first
 * header_size bytes of the header as it lies, except disk_header_size, flag
 * and crc, which it zeroes first -- wherever they fall inside those bytes,
 * since header_size has no lower bound there (a header_size of 0..19 covers
 * only part of the 20-byte fixed part).  Fills up to 5 (pointer, length)
 * pieces; header_size >= 0 (a negative one the reference would pass to
 * crc32_8bytes as a huge size_t: refused by the callers). */
static int hdr_pieces(const unsigned char *h, int32_t hs, const unsigned char **ptr, uint32_t *len)
{
    static const unsigned char zero[8];
    const struct { const unsigned char *p; uint32_t off, len; } fixed[4] = {
        {h + NC_HDR_OFF_MAGIC, NC_HDR_OFF_MAGIC, 4},
        {zero, NC_HDR_OFF_DISK_HEADER_SIZE, 4},                /* disk_header_size := 0 */
        {h + NC_HDR_OFF_HEADER_SIZE, NC_HDR_OFF_HEADER_SIZE, 4},
        {zero, NC_HDR_OFF_FLAG, 8},                            /* flag, crc := 0 */
    };
    int k = 0;
    for (int i = 0; i < 4; i++) {
        if ((int64_t)hs <= fixed[i].off) break;
        const uint32_t take = (uint32_t)hs - fixed[i].off < fixed[i].len ? (uint32_t)hs - fixed[i].off : fixed[i].len;
        ptr[k] = fixed[i].p;
        len[k++] = take;
    }
    if (hs > NC_HDR_MIN_SIZE) {
        ptr[k] = h + NC_HDR_MIN_SIZE;
        len[k++] = (uint32_t)hs - NC_HDR_MIN_SIZE;
    }
    return k;
}

uint32_t nc_header_crc(const void *header)
{
    if (!header) return 0;
    const int32_t hs = hdr_size(header);
    if (hs < 0) return 0;
    pthread_once(&crc_once, crc_init);
    const unsigned char *ptr[5];
    uint32_t len[5];
    const int k = hdr_pieces(header, hs, ptr, len);
    uint32_t c = 0xFFFFFFFFu;
    for (int i = 0; i < k; i++) c = crc_run(c, ptr[i], len[i]);
    return ~c;
}

int nc_header_seal(void *header)
{
    if (!header || hdr_size(header) < 0) return -EINVAL;
    const uint32_t c = nc_header_crc(header);
    memcpy((unsigned char *)header + NC_HDR_OFF_CRC, &c, 4);
    return 0;
}

/* dm_check_magic (diskcache.c:594-602), and a header_size crc32_8bytes can
 * take: the reference passes a negative one on as a huge size_t (a read far
 * past the header), which is the only input refused here */
static int hdr_plausible(const void *header)
{
    uint32_t magic;
    if (!header) return 0;
    memcpy(&magic, header, 4);
    return magic == NC_MAGIC_V30 && hdr_size(header) >= 0;
}

static uint32_t hdr_stored_crc(const void *header)
{
    uint32_t c;
    memcpy(&c, (const unsigned char *)header + NC_HDR_OFF_CRC, 4);
    return c;
}

int nc_header_verify(const void *header)
{
    if (!hdr_plausible(header)) return 0;
    return nc_header_crc(header) == hdr_stored_crc(header);
}

/* Each header becomes a chunk of up to 5 segments whose skipped fields point
 * at zeros (hdr_pieces), so the batcher's gather builds exactly the bytes
 * dm_verify_header's CRC is defined over -- none at all for header_size 0
 * (CRC 0, as crc32_8bytes of nothing). */
int md5hip_batch_verify_headers(md5hip_batcher *b, const void *const *headers, uint64_t n,
                                unsigned char *ok)
{
    if (!b) return -EINVAL;
    if (n == 0) return 0;
    if (!headers || !ok) return -EINVAL;
    int rc = 0;
    struct md5hip_iov *segs = malloc(sizeof *segs * 5 * n);
    uint64_t *first = malloc(sizeof *first * (n + 1));
    uint32_t *want = malloc(4 * n);
    unsigned char *got = malloc(n);
    if (!segs || !first || !want || !got) { rc = -ENOMEM; goto out; }
    uint64_t s = 0;
    first[0] = 0;
    for (uint64_t i = 0; i < n; i++) {
        const unsigned char *h = headers[i];
        if (hdr_plausible(h)) {
            const unsigned char *ptr[5];
            uint32_t len[5];
            const int k = hdr_pieces(h, hdr_size(h), ptr, len);
            for (int j = 0; j < k; j++) segs[s++] = (struct md5hip_iov){ptr[j], len[j]};
            want[i] = hdr_stored_crc(h);
        } else {
            want[i] = 0;                 /* empty chunk: crc 0, forced to fail below */
        }
        first[i + 1] = s;
    }
    /* CRC-32 for this call only: the batcher's own digest kind (it may be
     * shared with ASIO threads hashing blocks) is left alone */
    rc = md5hip_verify_iov_as(b, MD5HIP_DIGEST_CRC32, 0, segs, first, n, want, got);
    if (rc < 0) goto out;
    rc = 0;
    for (uint64_t i = 0; i < n; i++) {
        ok[i] = got[i] && hdr_plausible(headers[i]);
        rc += !ok[i];
    }
out:
    free(segs);
    free(first);
    free(want);
    free(got);
    return rc;
}
