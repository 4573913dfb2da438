#!/usr/bin/env python3
"""Join power_ab.json (case wall windows) with a rocm-smi trace: median board
power and sclk per case (samples >= 0.7 s into the window).
    python scripts/power_summary.py power_ab.json power_trace.txt"""
import json
import re
import statistics
import sys

ab = json.load(open(sys.argv[1]))
rows, cur = [], None
for ln in open(sys.argv[2]):
    if ln.startswith("T "):
        cur = {"t": float(ln.split()[1])}
        rows.append(cur)
    elif cur is not None and "Power" in ln:
        mt = re.search(r"\(W\):\s*([\d.]+)", ln)
        if mt:
            cur["p"] = float(mt.group(1))
    elif cur is not None and "sclk" in ln:
        mt = re.search(r"(\d+)Mhz", ln)
        if mt:
            cur["sclk"] = int(mt.group(1))
out = {}
for case, w in ab.items():
    sel = [r for r in rows if w["t0"] + 0.7 <= r["t"] <= w["t1"] and "p" in r]
    out[case] = {"ms": w["ms"], "payload_GBps": round(17179869184 / (w["ms"] * 1e6), 1),
                 "watts_median": statistics.median(r["p"] for r in sel) if sel else None,
                 "sclk_mhz_median": statistics.median(r["sclk"] for r in sel if "sclk" in r) if sel else None,
                 "samples": len(sel)}
print(json.dumps(out))
