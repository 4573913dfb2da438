#!/usr/bin/env python3
"""profiles/traffic.json from a PMC summary (scripts/pmc_summary.py output):
HBM bytes per launch (read: 2 x 1024 x FETCH_SIZE, write: 1024 x WRITE_SIZE,
MI355X_MICROARCH.md §HBM) per kernel variant, read by bench.py's roofline."""
import json
import sys

KERNEL = {"direct2": "md5_fixed_direct<2, 0>", "direct4": "md5_fixed_direct<4, 0>",
          "lds64": "md5_fixed_lds64", "lds128": "md5_fixed_lds128", "xpose1": "md5_fixed_xpose1",
          "xpose2": "md5_fixed_xpose2", "xpose1nt": "md5_fixed_xpose1nt",
          "xpose2nt": "md5_fixed_xpose2nt", "lds128nt": "md5_fixed_lds128nt"}
summ = json.load(open(sys.argv[1]))
src = sys.argv[2] if len(sys.argv) > 2 else sys.argv[1]
out = {"_source": src, "_note": "HBM bytes per launch of 1,048,576 x 16 KiB; read = 2*1024*FETCH_SIZE, "
       "write = 1024*WRITE_SIZE (gfx950 corrections, MI355X_MICROARCH.md HBM section)"}
for v, k in KERNEL.items():
    m = [val for name, val in summ.items() if name.replace(" ", "") == k.replace(" ", "")]
    if m and "hbm_read_bytes" in m[0]:
        out[v] = int(m[0]["hbm_read_bytes"] + m[0].get("hbm_write_bytes", 0))
print(json.dumps(out, indent=1))
