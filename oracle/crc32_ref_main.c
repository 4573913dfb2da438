/*
 * oracle/crc32_ref_main.c -- TEST INFRASTRUCTURE: drives the REFERENCE
 * netcache CRC32 (/root/reference/netcache/netcache/crc32.c, compiled in place
 * by oracle/Makefile into _ref/crc32_ref_tool; --gc-sections drops the unused
 * crc32_8bytes_stream and with it its reference to netcache's bs_read).
 *
 * stdin: records  [u32 len][u32 fastcrc][len bytes]
 * stdout: one line per record: "<crc32_8bytes> <crc32_bitwise> <blkcrc>" (hex)
 * where blkcrc restates blk_make_crc's combination (blk_io.c:408-424) on top of
 * the reference crc32_8bytes: fastcrc == 0 or len <= fastcrc -> crc(all);
 * else crc(first fastcrc bytes) ^ crc(bytes [max(0, len - fastcrc), len)).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

uint32_t crc32_8bytes(const void *data, size_t length);
uint32_t crc32_bitwise(const void *data, size_t length);

int main(void)
{
    uint32_t hdr[2];
    while (fread(hdr, 4, 2, stdin) == 2) {
        uint32_t len = hdr[0], fast = hdr[1];
        unsigned char *buf = malloc(len ? len : 1);
        if (len && fread(buf, 1, len, stdin) != len) return 1;
        uint32_t c8 = crc32_8bytes(buf, len);
        uint32_t cb = crc32_bitwise(buf, len);
        uint32_t blk;
        if (fast == 0 || len <= fast) {
            blk = c8;
        } else {
            uint32_t head = crc32_8bytes(buf, fast);
            uint32_t toff = len > fast ? len - fast : 0;
            blk = head ^ crc32_8bytes(buf + toff, fast);
        }
        printf("%08x %08x %08x\n", c8, cb, blk);
        free(buf);
    }
    return 0;
}
