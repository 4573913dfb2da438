#!/usr/bin/env python3
"""The multi-GPU pool's call site on one GPU: netcache
vectors (64 / 256 / 1,024 x 16 KiB blocks) from registered host memory (the
page heap registered once, md5hip_host_register) through
  batcher   one md5hip_batcher (md5_batch_submit)
  pool1     md5hip_pool over (0,)             (md5hip_pool_submit)
  pool4     md5hip_pool over (0, 0, 0, 0)     (routing over 4 batchers)
Pointer / length arrays are built once and the C entries called through
ctypes (which drops the GIL), so the numbers are the library's, not Python's.
Per-call latency of synchronous submits from one thread (median / p90 us),
then T threads submitting synchronously for a fixed time (vectors/s, GiB/s).
Every result is compared with the first path's digests.
usage: pool_latency_probe.py [--iters N] [--threads T] [--secs S]"""
import argparse
import ctypes
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402
from sproxy_amd._lib import lib  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--threads", type=int, default=8)
    ap.add_argument("--secs", type=float, default=2.0)
    a = ap.parse_args()
    L = lib()
    heap = np.random.default_rng(5).integers(0, 256, 256 << 20, dtype=np.uint8)   # page heap
    m.register_host(heap)
    objs = {"batcher": m.Batcher(device=0), "pool1": m.Pool((0,)), "pool4": m.Pool((0, 0, 0, 0))}
    call = {"batcher": L.md5_batch_submit, "pool1": L.md5hip_pool_submit, "pool4": L.md5hip_pool_submit}
    res = {}
    for nb in (64, 256, 1024):
        Lc = 16384
        rng = np.random.default_rng(nb)
        starts = rng.integers(0, heap.size // Lc - nb, 64) * Lc
        vec_ptrs = [(np.uint64(heap.ctypes.data) + np.uint64(s) + np.arange(nb, dtype=np.uint64) * np.uint64(Lc))
                    for s in starts]
        lens = np.full(nb, Lc, np.uint32)

        def submit(k, j, out):
            rc = call[k](objs[k]._h, vec_ptrs[j % len(vec_ptrs)].ctypes.data, lens.ctypes.data, nb,
                         out.ctypes.data)
            assert rc == 0, (k, rc)

        ref = [np.empty((nb, 16), np.uint8) for _ in vec_ptrs]
        for j, r in enumerate(ref):
            submit("batcher", j, r)
        for k in objs:
            o = np.empty((nb, 16), np.uint8)
            submit(k, 3, o)
            assert np.array_equal(o, ref[3]), k
        lat = {k: [] for k in objs}
        out = np.empty((nb, 16), np.uint8)
        for it in range(a.iters + 10):
            for k in objs:
                t0 = time.perf_counter()
                submit(k, it, out)
                t1 = time.perf_counter()
                if it >= 10:
                    lat[k].append((t1 - t0) * 1e6)
        row = {k: {"median_us": round(float(np.median(x)), 1), "p90_us": round(float(np.percentile(x, 90)), 1)}
               for k, x in lat.items()}
        for k in objs:                             # T threads, synchronous calls
            count = [0] * a.threads
            stop = time.perf_counter() + a.secs
            bad = []

            def worker(t):
                o = np.empty((nb, 16), np.uint8)
                j = t
                while time.perf_counter() < stop:
                    submit(k, j, o)
                    if j % 7 == 0 and not np.array_equal(o, ref[j % len(ref)]):
                        bad.append(j)
                    count[t] += 1
                    j += a.threads

            before = [objs[k].device_stats(g)["launches"] for g in range(objs[k].ndev)] \
                if k != "batcher" else [objs[k].stats()["launches"]]
            th = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
            t0 = time.perf_counter()
            for x in th:
                x.start()
            for x in th:
                x.join()
            wall = time.perf_counter() - t0
            after = [objs[k].device_stats(g)["launches"] for g in range(objs[k].ndev)] \
                if k != "batcher" else [objs[k].stats()["launches"]]
            assert not bad, (k, bad)
            row[k].update(threads=a.threads, vectors_per_s=round(sum(count) / wall, 1),
                          gib_s=round(sum(count) * nb * Lc / wall / (1 << 30), 2),
                          launches=[y - x for x, y in zip(before, after)], vectors=sum(count))
        row["pool4"]["routing"] = objs["pool4"].stats()
        res[f"{nb}x16KiB"] = row
        print(json.dumps({f"{nb}x16KiB": row}), flush=True)
    for p in objs.values():
        p.close()
    m.unregister_host(heap)
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
