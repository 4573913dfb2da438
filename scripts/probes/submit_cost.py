#!/usr/bin/env python3
"""What one device-resident submission of a C3 vector (~79 K chunks) costs
on the calling thread, piece by piece: the Python binding's argument checks,
the producer-stream lookup, and the C call (md5_batch_submit_device_after)
with after = torch's current stream (the default) or none.  6 vectors per
burst like bench.py --config c3q `drained`; each burst is waited for.
usage: submit_cost.py [--bursts 8] [--out F]"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bursts", type=int, default=8)
    ap.add_argument("--out")
    a = ap.parse_args()
    import numpy as np
    import torch
    import bench
    from sproxy_amd import md5 as m
    K = 6
    lk = [bench.c3_lens(16 << 30, 3000 + 31 * j) for j in range(K)]
    ok_ = [bench.c3_offsets(x)[0] for x in lk]
    spans = [(bench.c3_offsets(x)[1] + 15) // 16 * 16 for x in lk]
    starts = np.concatenate([[0], np.cumsum(spans)[:-1]]).astype(np.int64)
    big = m.arena_empty(int(sum(spans)))
    m.fill_synthetic(big, seed=0xC3D)
    torch.cuda.synchronize()
    base = big.data_ptr()
    subs = [((base + starts[j] + ok_[j]).astype(np.uint64), lk[j].astype(np.uint32)) for j in range(K)]
    outs = [torch.empty((x.size, 16), dtype=torch.uint8, device="cuda") for x in lk]
    q = m.Queue(device=torch.cuda.current_device(), nslots=4, inflight=1)
    res = {}
    for mode in ("current", None, "current", None):
        per = {"dev_args": [], "producer": [], "c_call": [], "python_call": [], "burst": []}
        for b in range(a.bursts):
            pend = []
            t_b = time.perf_counter_ns()
            for (p, L_), o in zip(subs, outs):
                t0 = time.perf_counter_ns()
                q._dev_args(p, L_, o)
                t1 = time.perf_counter_ns()
                q._producer(mode)
                t2 = time.perf_counter_ns()
                pend.append(q.submit_device_async(p, L_, o, after=mode))
                t3 = time.perf_counter_ns()
                per["dev_args"].append((t1 - t0) / 1e3)
                per["producer"].append((t2 - t1) / 1e3)
                per["python_call"].append((t3 - t2) / 1e3)
            per["burst"].append((time.perf_counter_ns() - t_b) / 1e3)
            for pn in pend:
                pn.wait()
        # the C call alone: a direct ctypes call with the arrays prepared
        import ctypes
        for b in range(a.bursts):
            pend = []
            for (p, L_), o in zip(subs, outs):
                h, order = q._producer(mode)
                t = ctypes.c_uint64()
                t0 = time.perf_counter_ns()
                rc = q._call("submit_device_after", p.ctypes.data, L_.ctypes.data, p.size, o.data_ptr(), 1,
                             h, order, ctypes.byref(t))
                per["c_call"].append((time.perf_counter_ns() - t0) / 1e3)
                assert rc[1] == 0, rc
                pend.append(t.value)
            for t in pend:
                q._call("wait", t)
        key = f"after_{mode}"
        res.setdefault(key, [])
        res[key].append({k: round(float(np.median(v)), 1) for k, v in per.items()})
        print(key, res[key][-1], flush=True)
    rec = {"probe": "submit_cost", "vectors_per_burst": K, "chunks": [int(x.size) for x in lk],
           "us_median": res}
    print(json.dumps(rec))
    if a.out:
        open(a.out, "w").write(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    main()
