/*
 * oracle/crc32_oracle.c -- TEST INFRASTRUCTURE ONLY (parity checker).
 *
 * Clean-room restatement of netcache's block checksum:
 *   /root/reference/netcache/netcache/crc32.c  zlib CRC-32, polynomial
 *       0xEDB88320 (crc32.c:22), init ~0, final ~ (crc32.c:186-240: the
 *       slicing-by-8 form; this restatement is the byte-at-a-time table form,
 *       which computes the same function, crc32.c:105-116)
 *   /root/reference/netcache/common/blk_io.c:354-430 blk_make_crc: with
 *       fastcrc > 0 and remained > fastcrc the block checksum is
 *       crc(head fastcrc bytes) XOR crc(last fastcrc bytes) (blk_io.c:408-424).
 * Pinned by tests/test_crc32.py against tests/golden/crc32_golden.json, made
 * by tests/golden/make_golden_crc32.py from the reference crc32.c built in place.
 */
#include <stddef.h>
#include <stdint.h>

static uint32_t o_tab[256];
static int o_ready;

static void o_init(void)
{
    for (uint32_t i = 0; i < 256; i++) {
        uint32_t c = i;
        for (int k = 0; k < 8; k++) c = (c & 1u) ? (c >> 1) ^ 0xEDB88320u : (c >> 1);
        o_tab[i] = c;
    }
    o_ready = 1;
}

uint32_t oracle_crc32(const void *data, uint64_t len)
{
    const uint8_t *p = (const uint8_t *)data;
    if (!o_ready) o_init();
    uint32_t c = 0xFFFFFFFFu;
    for (uint64_t i = 0; i < len; i++) c = o_tab[(c ^ p[i]) & 0xFFu] ^ (c >> 8);
    return ~c;
}

uint32_t oracle_blk_crc(const void *data, uint64_t remained, uint32_t fastcrc)
{
    const uint8_t *p = (const uint8_t *)data;
    if (fastcrc == 0 || remained <= fastcrc) return oracle_crc32(p, remained);
    const uint64_t toff = remained - fastcrc;
    return oracle_crc32(p, fastcrc) ^ oracle_crc32(p + toff, fastcrc);
}

/* crcs[i] = blk_crc(base + offs[i], lens[i], fastcrc) */
void oracle_crc32_batch(const void *base, const uint64_t *offs, const uint32_t *lens, uint64_t n,
                        uint32_t fastcrc, uint32_t *crcs)
{
    const uint8_t *b = (const uint8_t *)base;
    for (uint64_t i = 0; i < n; i++) crcs[i] = oracle_blk_crc(b + offs[i], lens[i], fastcrc);
}
