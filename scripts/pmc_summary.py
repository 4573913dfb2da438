#!/usr/bin/env python3
"""Summarise rocprofv3 PMC passes (scripts/pmc_passes.sh) per kernel: mean of
each counter over that kernel's dispatches, plus derived figures.

HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports exactly
half of a wide coalesced read stream on gfx950, so read bytes = 2 * 1024 *
FETCH_SIZE; WRITE_SIZE (KB) reads the bytes exactly for 16-B stores.  Effective
clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel duration."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def short(name):
    name = name.split("(")[0].replace("void ", "").replace("md5hip::", "")
    return name.strip()


def main(d):
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    for f in sorted(glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)):
        per = defaultdict(lambda: defaultdict(float))
        meta = {}
        for r in csv.DictReader(open(f)):
            key = (short(r["Kernel_Name"]), r["Dispatch_Id"])
            per[key][r["Counter_Name"]] += float(r["Counter_Value"])
            meta[key] = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-9
        for (k, _), cs in per.items():
            for c, v in cs.items():
                vals[k][c].append(v)
        for (k, _), t in meta.items():
            dur[k].append(t)
    out = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        t = sorted(dur[k])[len(dur[k]) // 2]
        o = {"dur_ms_profiled": round(t * 1e3, 4)}
        o.update({c: round(v, 1) for c, v in m.items()})
        if "FETCH_SIZE" in m:
            o["hbm_read_bytes"] = int(2 * 1024 * m["FETCH_SIZE"])
        if "WRITE_SIZE" in m:
            o["hbm_write_bytes"] = int(1024 * m["WRITE_SIZE"])
        if "GRBM_GUI_ACTIVE" in m and t > 0:
            o["clock_ghz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / t / 1e9, 3)
        if "SQ_ACTIVE_INST_VALU" in m and "GRBM_GUI_ACTIVE" in m:
            # quad-cycles of VALU activity over (SIMDs x GPU cycles / 4)
            simd_quads = 1024 * (m["GRBM_GUI_ACTIVE"] / 8) / 4
            o["valu_busy_frac"] = round(m["SQ_ACTIVE_INST_VALU"] / simd_quads, 4)
        if "SQ_WAIT_ANY" in m and "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            o["wait_any_frac"] = round(m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"], 4)
            o["wait_inst_frac"] = round(m.get("SQ_WAIT_INST_ANY", 0) / m["SQ_WAVE_CYCLES"], 4)
        out[k] = o
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
