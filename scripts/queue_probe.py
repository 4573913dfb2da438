#!/usr/bin/env python3
"""What the queue does under bench.py's c3q loops: per submit / wait call,
its wall time and the queue's launch count after it (md5hip_batcher stats),
for the drained and the pipelined step patterns.  usage: queue_probe.py"""
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from sproxy_amd import md5 as m  # noqa: E402


def main():
    K = 6
    lk = [bench.c3_lens(16 << 30, 3000 + 31 * j) for j in range(K)]
    ok_ = [bench.c3_offsets(x)[0] for x in lk]
    spans = [(bench.c3_offsets(x)[1] + 15) // 16 * 16 for x in lk]
    starts = np.concatenate([[0], np.cumsum(spans)[:-1]]).astype(np.int64)
    big = m.arena_empty(int(sum(spans)))
    m.fill_synthetic(big, seed=0xC3D)
    base = big.data_ptr()
    subs = [((base + starts[j] + ok_[j]).astype(np.uint64), lk[j].astype(np.uint32)) for j in range(K)]
    outs = [[torch.empty((x.size, 16), dtype=torch.uint8, device="cuda") for x in lk] for _ in range(2)]
    q = m.Queue(device=0, nslots=4, inflight=1)
    t0 = time.perf_counter()
    log = []

    def ev(what):
        log.append((round((time.perf_counter() - t0) * 1e3, 3), what, q.stats()["launches"]))

    def submit(k):
        pend = []
        for (p, L), o in zip(subs, outs[k & 1]):
            pend.append(q.submit_device_async(p, L, o))
            ev(f"submit s{k}")
        return pend

    def drain(pend, k):
        for pn in reversed(pend):
            pn.wait()
        ev(f"drained s{k}")

    for k in range(3):                       # drained steps
        drain(submit(k), k)
    prev = submit(10)                         # pipelined steps
    for k in range(11, 15):
        cur = submit(k)
        drain(prev, k - 1)
        prev = cur
    drain(prev, 14)
    torch.cuda.synchronize()
    print(json.dumps({"stats": q.stats(), "log": log}))
    q.close()


if __name__ == "__main__":
    main()
