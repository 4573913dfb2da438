#!/usr/bin/env python3
"""HBM read bytes of XDMA vs LINES from a `rocprofv3 --pmc FETCH_SIZE` run of
scripts/lines_ab.py (shapes in the order given to it), merged into
profiles/traffic.json as read-only entries keyed kernel@shape, with each
kernel's code hash (sproxy_amd._lib.kernel_code_hash) and the ratio to the
shape's payload (read = 2 x 1024 x FETCH_SIZE on gfx950, MI355X_MICROARCH.md).
usage: lines_traffic.py PMC_CSV LINES_AB_JSON --shapes packed16,packed128 --source TAG [--out F]"""
import argparse
import csv
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("pmc_csv")
    ap.add_argument("lines_ab_json")
    ap.add_argument("--shapes", default="packed16,packed128")
    ap.add_argument("--source", required=True)
    ap.add_argument("--out", default=os.path.join(REPO, "profiles", "traffic.json"))
    a = ap.parse_args()
    from sproxy_amd._lib import kernel_code_hash
    shapes = a.shapes.split(",")
    ab = json.loads(open(a.lines_ab_json).read().strip().splitlines()[-1])
    per = defaultdict(list)                     # kernel -> [(dispatch, bytes)]
    for r in csv.DictReader(open(a.pmc_csv)):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        k = r["Kernel_Name"].split("(")[0].replace("md5hip::", "").strip()
        if k in ("md5_desc_xdma", "md5_desc_lines"):
            per[k].append((int(r["Dispatch_Id"]), 2 * 1024 * float(r["Counter_Value"])))
    d = json.load(open(a.out))
    out = {}
    for k, v in per.items():
        v.sort()
        step = len(v) // len(shapes)
        for j, sh in enumerate(shapes):
            vals = [b for _, b in v[j * step:(j + 1) * step]]
            pay = ab[sh]["payload_bytes"]
            rb = sum(vals) / len(vals)
            e = {"read_bytes": int(rb), "payload_bytes": int(pay), "read_over_payload": round(rb / pay, 4),
                 "dispatches": len(vals), "code_hash": kernel_code_hash(k), "source": a.source,
                 "median_ms": ab[sh]["median_ms"]["lines" if k.endswith("lines") else "xdma"]}
            key = f"{k}@{sh}@{ab[sh]['chunks']}x16384"
            d["entries"][key] = e
            out[key] = e
    json.dump(d, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    sys.exit(main())
