#!/usr/bin/env python3
"""Merge rocprofv3 PMC passes into profiles/traffic.json: one entry per
kernel@workload, with the SHA-256 of that kernel's machine code in the
library that ran (sproxy_amd._lib.kernel_code_hash), so bench.py reports
counter bytes only while the kernel's code is the code that was measured.

usage: traffic_json.py FETCH_DIR WRITE_DIR WORKLOAD [--valu VALU_DIR] [--out profiles/traffic.json]
  FETCH_DIR / WRITE_DIR: `rocprofv3 --pmc FETCH_SIZE` / `--pmc WRITE_SIZE`
  output dirs (csv) of the same bench command; WORKLOAD: the bench line's
  config tag the bytes belong to (e.g. c2@1048576x16384).  VALU_DIR: a pass
  of SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE (SURVEY §8(d) asks for
  VALUBusy beside the HBM roofline): valu_busy = SQ_ACTIVE_INST_VALU quad-
  cycles over (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs / 4).
HBM bytes per launch (MI355X_MICROARCH.md HBM section, gfx950): read =
2 x 1024 x FETCH_SIZE, write = 1024 x WRITE_SIZE, mean over the kernel's
dispatches."""
import argparse
import csv
import glob
import json
import os
import sys
from collections import defaultdict

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def short(name):
    # template arguments dropped: kernel_code_hash finds the (one) product
    # instantiation by its base name
    return name.split("(")[0].split("<")[0].replace("void ", "").replace("md5hip::", "").strip()


def per_kernel(d, counter):
    vals = defaultdict(list)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = defaultdict(float)
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] == counter:
                per[(short(r["Kernel_Name"]), r["Dispatch_Id"])] += float(r["Counter_Value"])
        for (k, _), v in per.items():
            vals[k].append(v)
    return {k: sum(v) / len(v) for k, v in vals.items()}, {k: len(v) for k, v in vals.items()}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("fetch")
    p.add_argument("write")
    p.add_argument("workload")
    p.add_argument("--out", default=os.path.join(REPO, "profiles", "traffic.json"))
    p.add_argument("--source", default="")
    p.add_argument("--valu", default=None)
    a = p.parse_args()
    from sproxy_amd._lib import kernel_code_hash
    fs, nf = per_kernel(a.fetch, "FETCH_SIZE")
    ws, _ = per_kernel(a.write, "WRITE_SIZE")
    va, vi, gr = ({}, {}, {}) if not a.valu else (per_kernel(a.valu, "SQ_ACTIVE_INST_VALU")[0],
                                                   per_kernel(a.valu, "SQ_INSTS_VALU")[0],
                                                   per_kernel(a.valu, "GRBM_GUI_ACTIVE")[0])
    d = json.load(open(a.out)) if os.path.exists(a.out) else {}
    d["_note"] = ("HBM bytes per launch from rocprofv3 PMC (read = 2*1024*FETCH_SIZE, write = "
                  "1024*WRITE_SIZE; MI355X_MICROARCH.md HBM section), per kernel@workload, with "
                  "the SHA-256 of the kernel's machine code that was measured; valu_busy = "
                  "SQ_ACTIVE_INST_VALU / (1024 SIMDs x GRBM_GUI_ACTIVE/8 / 4) from a separate pass")
    ent = d.setdefault("entries", {})
    new = {}
    for k, v in fs.items():
        if not k.startswith(("md5_", "crc32_")):
            continue
        new[f"{k}@{a.workload}"] = {
            "bytes": int(2 * 1024 * v + 1024 * ws.get(k, 0.0)),
            "read_bytes": int(2 * 1024 * v), "write_bytes": int(1024 * ws.get(k, 0.0)),
            "dispatches": nf[k], "code_hash": kernel_code_hash(k), "source": a.source}
        if k in va and gr.get(k):
            new[f"{k}@{a.workload}"].update({
                "valu_busy": round(va[k] / (1024 * gr[k] / 8 / 4), 4),
                "valu_insts": int(vi.get(k, 0)), "gpu_cycles": int(gr[k] / 8)})
    ent.update(new)
    json.dump(d, open(a.out, "w"), indent=1, sort_keys=True)
    print(json.dumps(new, indent=1))


if __name__ == "__main__":
    main()
