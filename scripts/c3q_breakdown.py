#!/usr/bin/env python3
"""Where a DRAINED c3q step's time goes (bench.py --config c3q's `drained`
leg: K C3 vectors of 16 GiB submitted to one md5hip_queue, every ticket
waited for before the next step).  Host stamps (CLOCK_MONOTONIC, the clock
rocprofv3 stamps with) around each submission and each wait; run it under
`rocprofv3 --kernel-trace --memory-copy-trace` and join afterwards: per step,
submit time, the gap from the first wait to the first device op (planning,
descriptor copies), each device op, and the tail from the last op's end to
the last wait's return.
usage: c3q_breakdown.py [--steps 6] [--batches 6] [--out stamps.json]
       c3q_breakdown.py --join TRACE_DIR --stamps stamps.json"""
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


def now():
    return time.clock_gettime_ns(time.CLOCK_MONOTONIC)


def run(a):
    import torch
    import bench
    from sproxy_amd import md5 as m
    K = a.batches
    lk = [bench.c3_lens(a.c3_bytes, 3000 + 31 * j) for j in range(K)]
    ok_ = [bench.c3_offsets(x)[0] for x in lk]
    spans = [(bench.c3_offsets(x)[1] + 15) // 16 * 16 for x in lk]
    starts = np.concatenate([[0], np.cumsum(spans)[:-1]]).astype(np.int64)
    big = m.arena_empty(int(sum(spans)))
    m.fill_synthetic(big, seed=0xC3D)
    torch.cuda.synchronize()
    subs = [((big.data_ptr() + starts[j] + ok_[j]).astype(np.uint64), lk[j].astype(np.uint32)) for j in range(K)]
    outs = [torch.empty((x.size, 16), dtype=torch.uint8, device="cuda") for x in lk]
    q = m.Queue(device=0, nslots=4, inflight=1)        # as bench.py --config c3q
    steps = []
    for s in range(a.steps + 2):
        rec = {"submit": [], "wait": []}
        pend = []
        for (p, L_), o in zip(subs, outs):
            t0 = now()
            pend.append(q.submit_device_async(p, L_, o))
            rec["submit"].append((t0, now()))
        for pn in reversed(pend):
            t0 = now()
            pn.wait()
            rec["wait"].append((t0, now()))
        if s >= 2:
            steps.append(rec)
    st = q.stats()
    q.close()
    json.dump({"batches": K, "chunks": int(sum(x.size for x in lk)), "payload": int(sum(x.sum() for x in lk)),
               "steps": steps, "queue": st}, open(a.out, "w"))
    for rec in steps:
        sub = (rec["submit"][-1][1] - rec["submit"][0][0]) / 1e6
        tot = (rec["wait"][-1][1] - rec["submit"][0][0]) / 1e6
        print(f"step: submit {sub:.3f} ms, total {tot:.3f} ms", flush=True)


def load_trace(d):
    ops = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append(("K:" + r["Kernel_Name"].split("(")[0][-40:], int(r["Start_Timestamp"]),
                        int(r["End_Timestamp"])))
    for f in glob.glob(os.path.join(d, "**", "*memory_copy_trace.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            ops.append(("C:" + r.get("Direction", "copy"), int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(ops, key=lambda x: x[1])


def join(a):
    S = json.load(open(a.stamps))
    ops = load_trace(a.join)
    out = []
    for rec in S["steps"]:
        s0, s1 = rec["submit"][0][0], rec["submit"][-1][1]
        w0, w1 = rec["wait"][0][0], rec["wait"][-1][1]
        inside = [o for o in ops if o[1] >= s0 and o[2] <= w1 + 1000]
        first = inside[0][1] if inside else None
        last = inside[-1][2] if inside else None
        main = max(inside, key=lambda o: o[2] - o[1]) if inside else None
        out.append({
            "submit_ms": round((s1 - s0) / 1e6, 3),
            "submit_end_to_first_wait_ms": round((w0 - s1) / 1e6, 3),
            "first_wait_to_first_op_ms": round((first - w0) / 1e6, 3) if first else None,
            "submit_start_to_first_op_ms": round((first - s0) / 1e6, 3) if first else None,
            "ops": [(n, round((b - first) / 1e6, 3), round((e - b) / 1e6, 3)) for n, b, e in inside],
            "main_kernel_ms": round((main[2] - main[1]) / 1e6, 3) if main else None,
            "last_op_end_to_return_ms": round((w1 - last) / 1e6, 3) if last else None,
            "step_ms": round((w1 - s0) / 1e6, 3)})
    res = {"batches": S["batches"], "chunks": S["chunks"], "payload": S["payload"], "queue": S["queue"],
           "steps": out}
    keys = ["submit_ms", "first_wait_to_first_op_ms", "main_kernel_ms", "last_op_end_to_return_ms", "step_ms"]
    res["median"] = {k: float(np.median([x[k] for x in out if x[k] is not None])) for k in keys}
    print(json.dumps(res["median"]))
    json.dump(res, open(a.out, "w"), indent=1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=6)
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--c3-bytes", type=int, default=16 << 30)
    ap.add_argument("--out", default="c3q_stamps.json")
    ap.add_argument("--join", default=None)
    ap.add_argument("--stamps", default=None)
    a = ap.parse_args()
    if a.join:
        join(a)
    else:
        run(a)


if __name__ == "__main__":
    sys.exit(main())
