/*
 * oracle/nc_header_probe.c -- TEST INFRASTRUCTURE: the on-disk header layout
 * of netcache (§8f row 3) taken from the reference header itself, as is:
 * offsetof() of fc_common_header_t / struct tag_fc_header_info_v30
 * (netcache/include/netcache.h:756-790), NC_MAGIC_V30 (:740),
 * NC_HEADER_FLAG_COMPRESSED (:749) and NC_CANNED_CRC_SIZE (:879), compiled
 * against /root/reference/netcache/include with no stand-in headers.
 *
 * netcache.h includes ncapi.h, which includes <uuid/uuid.h>.  The image
 * carries that header in conda's libuuid 1.0.3 package
 * (/opt/conda/include/uuid/uuid.h, a real library header, not a stand-in);
 * `make -C oracle probe` adds -I/opt/conda/include.  tests/golden/
 * make_nc_layout.py runs the probe and commits its JSON output as
 * tests/golden/nc_header_layout.json, which tests/test_nc_digest.py checks
 * include/nc_digest.h against.
 */
#include <stddef.h>
#include <stdio.h>
#include "netcache.h"

#define OFF30(f) offsetof(struct tag_fc_header_info_v30, f)

int main(void)
{
    static const unsigned canned[] = {0, 1, 2, 3, 64, 65, 1000};
    printf("{\"NC_MAGIC_V30\": %u, \"NC_HEADER_FLAG_COMPRESSED\": %u, \"NC_CANNED_CRC_SIZE\": [",
           (unsigned)NC_MAGIC_V30, (unsigned)NC_HEADER_FLAG_COMPRESSED);
    for (unsigned i = 0; i < sizeof canned / sizeof canned[0]; i++)
        printf("%s[%u, %zu]", i ? ", " : "", canned[i], (size_t)NC_CANNED_CRC_SIZE(canned[i]));
    printf("], \"sizeof_fc_common_header_t\": %zu, \"magic\": %zu, \"disk_header_size\": %zu, "
           "\"header_size\": %zu, \"flag\": %zu, \"crc\": %zu, \"block_size\": %zu, \"size\": %zu, "
           "\"bitmaplen\": %zu, \"vlen\": %zu, \"vbase\": %zu, \"sizeof_v30\": %zu, "
           "\"sizeof_nc_crc_t\": %zu}\n",
           sizeof(fc_common_header_t), offsetof(fc_common_header_t, magic),
           offsetof(fc_common_header_t, disk_header_size), offsetof(fc_common_header_t, header_size),
           offsetof(fc_common_header_t, flag), OFF30(crc), OFF30(block_size), OFF30(size),
           OFF30(bitmaplen), OFF30(vlen), OFF30(vbase), sizeof(struct tag_fc_header_info_v30),
           sizeof(nc_crc_t));
    return 0;
}
