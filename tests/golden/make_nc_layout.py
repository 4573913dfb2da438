#!/usr/bin/env python3
"""Regenerate tests/golden/nc_header_layout.json from the REFERENCE netcache.h.

Run in the build container only (needs /root/reference).  It builds
oracle/nc_header_probe.c against /root/reference/netcache/include as it lies,
plus the image's conda libuuid 1.0.3 header (/opt/conda/include/uuid/uuid.h,
which netcache/include/ncapi.h:6 includes) -- ``make -C oracle probe`` -- and
stores the probe's output: offsetof() of fc_common_header_t and struct
tag_fc_header_info_v30 (netcache.h:756-790), NC_MAGIC_V30 (:740),
NC_HEADER_FLAG_COMPRESSED (:749) and NC_CANNED_CRC_SIZE (:879) at a few
bitmap lengths.  The GPU box never runs this script.
"""
import json
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))


def main():
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "probe"], check=True,
                   stdout=subprocess.DEVNULL)
    out = subprocess.run([os.path.join(REPO, "oracle", "_ref", "nc_header_probe")], check=True,
                         capture_output=True, text=True).stdout
    lay = json.loads(out)
    lay["_source"] = ("oracle/nc_header_probe.c compiled against /root/reference/netcache/include "
                      "(netcache.h:740-790, :879) with -I/opt/conda/include (libuuid 1.0.3)")
    with open(os.path.join(HERE, "nc_header_layout.json"), "w") as f:
        json.dump(lay, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
