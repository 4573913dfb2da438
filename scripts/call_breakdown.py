#!/usr/bin/env python3
"""Where a synchronous call's time goes: N calls of one netcache vector
(nb x 16 KiB) through one batcher, from registered host pages (zero-copy) or
device-resident chunks through a queue, with wall-clock stamps per call.
Run it under `rocprofv3 --kernel-trace --memory-copy-trace` and join the
traces with --join DIR afterwards: per call, the host call window against the
device's copies and kernels inside it (first op start - call start, op
durations, gaps, last op end - call end).
usage: call_breakdown.py [--mode host|device] [--nb 64] [--calls 200] [--crc] [--out stamps.json]
       call_breakdown.py --join TRACE_DIR --stamps stamps.json"""
import argparse
import csv
import glob
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def run(a):
    import torch
    from sproxy_amd import md5 as m
    from sproxy_amd._lib import lib
    L = lib()
    nb, Lc = a.nb, 16384
    stamps = []
    if a.mode == "host":
        heap = np.random.default_rng(5).integers(0, 256, 64 << 20, dtype=np.uint8)
        m.register_host(heap)
        b = m.Batcher(device=0)
        ptrs = (np.uint64(heap.ctypes.data) + np.arange(nb, dtype=np.uint64) * np.uint64(Lc))
        lens = np.full(nb, Lc, np.uint32)
        out = np.empty((nb, 16), np.uint8)
        call = lambda: L.md5_batch_submit(b._h, ptrs.ctypes.data, lens.ctypes.data, nb, out.ctypes.data)  # noqa: E731
    else:
        data = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
        m.fill_synthetic(data, seed=3)
        torch.cuda.synchronize()
        b = m.Queue(device=0)
        if a.crc:
            b.set_digest(m.Batcher.CRC32)
        ptrs = (np.uint64(data.data_ptr()) + np.arange(nb, dtype=np.uint64) * np.uint64(Lc))
        lens = np.full(nb, Lc, np.uint32)
        dig = torch.empty((nb, 16), dtype=torch.uint8, device="cuda")
        call = lambda: L.md5_batch_submit_device(b._h, ptrs.ctypes.data, lens.ctypes.data, nb,  # noqa: E731
                                                 dig.data_ptr(), 1)
    for i in range(a.calls + 20):
        t0 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        assert call() == 0
        t1 = time.clock_gettime_ns(time.CLOCK_MONOTONIC)
        if i >= 20:
            stamps.append((t0, t1))
    b.close()
    json.dump({"mode": a.mode, "nb": nb, "stamps": stamps}, open(a.out, "w"))
    us = [(y - x) / 1e3 for x, y in stamps]
    print(json.dumps({"mode": a.mode, "nb": nb, "median_us": round(float(np.median(us)), 1)}))


def rows(d, pat):
    out = []
    for f in glob.glob(os.path.join(d, "**", pat), recursive=True):
        out += list(csv.DictReader(open(f)))
    return out


def join(a):
    st = json.load(open(a.stamps))
    ops = []
    for r in rows(a.join, "*kernel_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K:" + r["Kernel_Name"].split("(")[0][-40:]))
    for r in rows(a.join, "*memory_copy_trace.csv"):
        ops.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C:" + r.get("Direction", r.get("Kind", "copy"))))
    ops.sort()
    per = []
    for t0, t1 in st["stamps"]:
        inside = [o for o in ops if o[0] >= t0 and o[1] <= t1 + 1000]
        if not inside:
            continue
        seq, prev = [], t0
        for s, e, name in inside:
            seq.append((name, round((s - prev) / 1e3, 1), round((e - s) / 1e3, 1)))
            prev = e
        per.append({"call_us": round((t1 - t0) / 1e3, 1), "tail_us": round((t1 - prev) / 1e3, 1), "ops": seq})
    if not per:
        print(json.dumps({"error": "no device ops inside the call windows (clock domains differ?)",
                          "ops": len(ops), "calls": len(st["stamps"])}))
        return
    names = [tuple(x[0] for x in p["ops"]) for p in per]
    common = max(set(names), key=names.count)
    sel = [p for p, n in zip(per, names) if n == common]
    med = lambda v: round(float(np.median(v)), 1)  # noqa: E731
    summary = {"mode": st["mode"], "nb": st["nb"], "calls": len(per), "calls_with_common_sequence": len(sel),
               "call_us": med([p["call_us"] for p in sel]), "tail_us": med([p["tail_us"] for p in sel]),
               "sequence": [{"op": n, "gap_before_us": med([p["ops"][k][1] for p in sel]),
                             "dur_us": med([p["ops"][k][2] for p in sel])} for k, n in enumerate(common)]}
    print(json.dumps(summary, indent=1))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mode", default="host", choices=["host", "device"])
    ap.add_argument("--nb", type=int, default=64)
    ap.add_argument("--calls", type=int, default=200)
    ap.add_argument("--out", default="stamps.json")
    ap.add_argument("--join", default=None)
    ap.add_argument("--stamps", default=None)
    ap.add_argument("--crc", action="store_true", help="device mode: CRC-32 digests")
    a = ap.parse_args()
    if a.join:
        join(a)
    else:
        run(a)


if __name__ == "__main__":
    main()
