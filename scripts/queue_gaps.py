#!/usr/bin/env python3
"""Kernel-trace timeline of a queue run (rocprofv3 --kernel-trace csv): the
descriptor launches in order, their durations and the idle gap before each
(what the batcher's host side costs between launches).
usage: queue_gaps.py TRACE_DIR"""
import csv
import glob
import json
import os
import sys


def main(d):
    rows = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0]))
    rows.sort()
    out, prev_end = [], None
    for s, e, k in rows:
        if "md5_desc" not in k and "gather_segments" not in k:
            continue
        out.append({"kernel": k.replace("void ", "").replace("md5hip::", "")[:40],
                    "ms": round((e - s) * 1e-6, 3),
                    "gap_before_ms": None if prev_end is None else round((s - prev_end) * 1e-6, 3)})
        prev_end = e
    desc = [x for x in out if "md5_desc" in x["kernel"]]
    gaps = [x["gap_before_ms"] for x in out if x["gap_before_ms"] is not None]
    print(json.dumps({"launches": len(desc), "sum_desc_ms": round(sum(x["ms"] for x in desc), 3),
                      "sum_gap_ms": round(sum(g for g in gaps if g > 0), 3), "timeline": out}, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
