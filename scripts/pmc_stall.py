#!/usr/bin/env python3
"""Where a kernel's wave cycles go, from rocprofv3 SQ counter passes
(attribute BALANCED's idle issue slots before another
variant).  Each PASS_DIR is one `rocprofv3 --pmc ... --output-format csv`
run of the same command; every counter found in any of them is summed per
dispatch of the kernels whose name contains --kernel, then averaged over
those dispatches.

Derived (MI355X_MICROARCH.md "rocprofv3 PMC slots": SQ_WAVE_CYCLES,
SQ_WAIT_*, SQ_ACTIVE_INST_* count quad-cycles; WAIT_ANY + WAIT_INST_ANY +
ACTIVE_INST_ANY ~ WAVE_CYCLES, disjoint):
  wave_cycles_split   WAIT_ANY (parked on s_waitcnt / barrier),
                      WAIT_INST_ANY (issue stall: dependency / pipe busy),
                      ACTIVE_INST_ANY (issuing) as fractions of WAVE_CYCLES
  active_split        ACTIVE_INST_{VALU,SCA,LDS,MISC,VMEM,FLAT} / WAVE_CYCLES
  insts_per_wave      SQ_INSTS_* / SQ_WAVES
  wave_occupancy      4 x SQ_WAVE_CYCLES / (SIMDs x GRBM_GUI_ACTIVE / 8)
usage: pmc_stall.py --kernel balanced PASS_DIR... [--out FILE]"""
import argparse
import csv
import glob
import json
import os
from collections import defaultdict


def load(dirs, kernel):
    per = defaultdict(lambda: defaultdict(float))      # (pass, dispatch) -> counter -> value
    names = {}
    for p, d in enumerate(dirs):
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if kernel not in r["Kernel_Name"]:
                    continue
                key = (p, r["Dispatch_Id"])
                per[key][r["Counter_Name"]] += float(r["Counter_Value"])
                names[key] = r["Kernel_Name"]
    tot, cnt = defaultdict(float), defaultdict(int)
    for key, cs in per.items():
        for c, v in cs.items():
            tot[c] += v
            cnt[c] += 1
    return {c: tot[c] / cnt[c] for c in tot}, {c: cnt[c] for c in cnt}, sorted(set(names.values()))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernel", required=True)
    ap.add_argument("dirs", nargs="+")
    ap.add_argument("--out")
    ap.add_argument("--simds", type=int, default=1024, help="SIMDs of the device (wave_occupancy)")
    a = ap.parse_args()
    mean, n, kernels = load(a.dirs, a.kernel)
    res = {"kernel_filter": a.kernel, "kernels": kernels, "dispatches": n, "per_dispatch": mean}
    wc = mean.get("SQ_WAVE_CYCLES")
    if wc:
        res["wave_cycles_split"] = {k: round(mean[k] / wc, 4) for k in
                                    ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY") if k in mean}
        res["active_split"] = {k: round(mean[k] / wc, 4) for k in mean if k.startswith("SQ_ACTIVE_INST_")}
        res["wait_inst_lds_frac"] = round(mean["SQ_WAIT_INST_LDS"] / wc, 4) if "SQ_WAIT_INST_LDS" in mean else None
    w = mean.get("SQ_WAVES")
    if w:
        res["insts_per_wave"] = {k: round(mean[k] / w, 1) for k in mean if k.startswith("SQ_INSTS_")}
    if "SQ_INSTS_VALU" in mean:
        other = sum(v for k, v in mean.items() if k.startswith("SQ_INSTS_") and k != "SQ_INSTS_VALU"
                    and k not in ("SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR"))   # sub-counts of VMEM
        res["non_valu_per_valu"] = round(other / mean["SQ_INSTS_VALU"], 4)
    g = mean.get("GRBM_GUI_ACTIVE")
    if wc and g:
        # wave occupancy of the launch: wave lifetimes (quad-cycles x 4) over
        # SIMDs x span (GRBM_GUI_ACTIVE is summed over the 8 XCDs).  For a
        # persistent one-wave-per-SIMD kernel (BALANCED) this is the share of
        # SIMD-time with a wave still holding work -- the list schedule's util.
        res["wave_occupancy"] = round(4 * wc / (a.simds * g / 8), 4)
        res["span_cycles"] = round(g / 8)
    txt = json.dumps(res, indent=1)
    print(txt)
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        open(a.out, "w").write(txt + "\n")


if __name__ == "__main__":
    main()
