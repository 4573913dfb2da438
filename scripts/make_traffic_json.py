#!/usr/bin/env python3
"""profiles/traffic.json from a PMC summary (scripts/pmc_summary.py output;
optional 3rd argument: an older traffic.json whose entries are kept unless re-measured):
HBM bytes per launch (read: 2 x 1024 x FETCH_SIZE, write: 1024 x WRITE_SIZE,
MI355X_MICROARCH.md §HBM) per kernel variant, read by bench.py's roofline."""
import json
import sys

KERNEL = {"direct2": "md5_fixed_direct<2, 0>", "direct4": "md5_fixed_direct<4, 0>",
          "lds64": "md5_fixed_lds64", "lds128": "md5_fixed_lds128", "xpose1": "md5_fixed_xpose1",
          "xpose2": "md5_fixed_xpose2", "xpose1nt": "md5_fixed_xpose1nt",
          "xpose2nt": "md5_fixed_xpose2nt", "lds128nt": "md5_fixed_lds128nt",
          "xdma1nt": "md5_fixed_xdma1nt", "crc32 xperm16": "crc32_fixed_xperm16", "crc32 xdma16": "crc32_fixed_xdma16", "crc32 shared8": "crc32_fixed_xpose"}
summ = json.load(open(sys.argv[1]))
src = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
prev = json.load(open(sys.argv[3])) if len(sys.argv) > 3 else {}
out = {"_source": src, "_note": "HBM bytes per launch of 1,048,576 x 16 KiB; read = 2*1024*FETCH_SIZE, "
       "write = 1024*WRITE_SIZE (gfx950 corrections, MI355X_MICROARCH.md HBM section)"}
out.update({k: v for k, v in prev.items() if not k.startswith("_")})
for v, k in KERNEL.items():
    m = [val for name, val in summ.items() if name.replace(" ", "") == k.replace(" ", "")]
    if m and "hbm_read_bytes" in m[0]:
        out[v] = int(m[0]["hbm_read_bytes"] + m[0].get("hbm_write_bytes", 0))
print(json.dumps(out, indent=1))
