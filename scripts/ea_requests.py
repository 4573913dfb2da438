#!/usr/bin/env python3
"""Per-kernel mean of rocprofv3 PMC counters (one value per dispatch, summed
over the counter's instances) from one or more `rocprofv3 --pmc ... -d DIR`
output directories.
usage: ea_requests.py DIR [DIR ...]  -> JSON {kernel: {counter: mean, "dispatches": n}}"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    return name.split("(")[0].split("<")[0].replace("void ", "").replace("md5hip::", "").strip()


def main():
    acc = defaultdict(lambda: defaultdict(list))
    for d in sys.argv[1:]:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            per = defaultdict(float)
            for r in csv.DictReader(open(f)):
                per[(short(r["Kernel_Name"]), r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
            for (k, _, c), v in per.items():
                acc[k][c].append(v)
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main()
