/*
 * oracle/nc_header_probe.c -- TEST INFRASTRUCTURE: the on-disk header layout
 * of netcache (§8f row 3) taken from the reference header itself, as is:
 * offsetof() of fc_common_header_t / struct tag_fc_header_info_v30
 * (netcache/include/netcache.h:756-790) compiled against
 * /root/reference/netcache/include with no stand-in headers.
 *
 * Status: UNBUILDABLE in this image -- netcache.h includes ncapi.h, which
 * includes <uuid/uuid.h> (libuuid development headers, not installed), and
 * no stand-in is written for it.  `make -C oracle probe` retries; when it
 * builds, its JSON output is the layout fixture tests/test_nc_digest.py
 * checks include/nc_digest.h against.  Until then row 3 is "parity
 * unpinned" (DESIGN.md §9).
 */
#include <stddef.h>
#include <stdio.h>
#include "netcache.h"
int main(void) {
    printf("{\"sizeof_fc_common_header_t\": %zu, \"magic\": %zu, \"disk_header_size\": %zu, \"header_size\": %zu, \"flag\": %zu, \"crc\": %zu, \"block_size\": %zu, \"size\": %zu, \"bitmaplen\": %zu, \"vlen\": %zu, \"vbase\": %zu, \"sizeof_v30\": %zu, \"sizeof_nc_crc_t\": %zu}\n",
        sizeof(fc_common_header_t), offsetof(fc_common_header_t, magic), offsetof(fc_common_header_t, disk_header_size),
        offsetof(fc_common_header_t, header_size), offsetof(fc_common_header_t, flag),
        offsetof(struct tag_fc_header_info_v30, crc), offsetof(struct tag_fc_header_info_v30, block_size),
        offsetof(struct tag_fc_header_info_v30, size), offsetof(struct tag_fc_header_info_v30, bitmaplen),
        offsetof(struct tag_fc_header_info_v30, vlen), offsetof(struct tag_fc_header_info_v30, vbase),
        sizeof(struct tag_fc_header_info_v30), sizeof(nc_crc_t));
    return 0;
}
