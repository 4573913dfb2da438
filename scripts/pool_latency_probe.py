#!/usr/bin/env python3
"""The multi-GPU pool's call site on one GPU: netcache
vectors (64 / 256 / 1,024 x 16 KiB blocks) from registered host memory (the
page heap registered once, md5hip_host_register) through
  batcher   one md5hip_batcher (md5_batch_submit)
  pool1     md5hip_pool over (0,)
  pool4     md5hip_pool over (0, 0, 0, 0)   (routing over 4 batchers)
Per-call latency of synchronous submits from one thread (median / p90 us),
then T threads submitting synchronously for a fixed time (vectors/s, GiB/s).
Every result is compared with the first path's digests.
usage: pool_latency_probe.py [--iters N] [--threads T] [--secs S]"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--secs", type=float, default=2.0)
    a = ap.parse_args()
    heap = np.random.default_rng(5).integers(0, 256, 256 << 20, dtype=np.uint8)   # page heap
    m.register_host(heap)
    paths = {"batcher": m.Batcher(device=0), "pool1": m.Pool((0,)), "pool4": m.Pool((0, 0, 0, 0))}
    res = {}
    for nb in (64, 256, 1024):
        L = 16384
        rng = np.random.default_rng(nb)
        starts = [int(x) * L for x in rng.integers(0, heap.size // L - nb, 64)]
        vecs = [[heap[s + i * L: s + (i + 1) * L] for i in range(nb)] for s in starts]
        ref = paths["batcher"].submit(vecs[0])
        for k, p in paths.items():
            assert np.array_equal(p.submit(vecs[0]), ref), k
        lat = {k: [] for k in paths}
        for it in range(a.iters + 10):
            v = vecs[it % len(vecs)]
            for k, p in paths.items():
                t0 = time.perf_counter()
                p.submit(v)
                t1 = time.perf_counter()
                if it >= 10:
                    lat[k].append((t1 - t0) * 1e6)
        row = {k: {"median_us": round(float(np.median(x)), 1), "p90_us": round(float(np.percentile(x, 90)), 1)}
               for k, x in lat.items()}
        for k, p in paths.items():                 # T threads, synchronous calls
            count = [0] * a.threads
            stop = time.perf_counter() + a.secs
            bad = []

            def worker(t):
                j = t
                while time.perf_counter() < stop:
                    d = p.submit(vecs[j % len(vecs)])
                    if j % 17 == 0 and not np.array_equal(d, paths["batcher"].submit(vecs[j % len(vecs)])):
                        bad.append(j)
                    count[t] += 1
                    j += a.threads

            th = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
            t0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            wall = time.perf_counter() - t0
            assert not bad, (k, bad)
            row[k]["threads"] = a.threads
            row[k]["vectors_per_s"] = round(sum(count) / wall, 1)
            row[k]["gib_s"] = round(sum(count) * nb * L / wall / (1 << 30), 2)
        if hasattr(paths["pool4"], "stats"):
            row["pool4"]["routing"] = paths["pool4"].stats()
            row["pool4"]["device_launches"] = [paths["pool4"].device_stats(g)["launches"] for g in range(4)]
        res[f"{nb}x16KiB"] = row
        print(json.dumps({f"{nb}x16KiB": row}), flush=True)
    for p in paths.values():
        p.close()
    m.unregister_host(heap)
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
