#!/usr/bin/env python3
"""C3 per-launch timeline: bench.py's C3 batch hashed by one descriptor kernel
K times back to back, an event pair around every launch (device ms per launch,
in order), with and without a host synchronize between launches.  Prints one
JSON object.   python scripts/c3_steps.py [--variant hybrid] [--steps 30]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--variant", default="hybrid")
    p.add_argument("--steps", type=int, default=30)
    p.add_argument("--prealloc", action="store_true",
                   help="allocate, fill and free a 16 GiB block first (desc_xdma_ab.py's pattern)")
    a = p.parse_args()
    rng = np.random.default_rng(1000)
    classes = np.array([4096 << k for k in range(9)], dtype=np.int64)
    lens, tot = [], 0
    while tot < (16 << 30):
        c = int(classes[rng.integers(0, 9)])
        if rng.integers(0, 8) == 0:
            c = int(rng.integers(1, c))
        lens.append(c)
        tot += c
    lens = np.array(lens, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
    total = int(offs[-1] + lens[-1] + 16)
    if a.prealloc:
        tmp = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
        m.fill_synthetic(tmp, seed=1)
        torch.cuda.synchronize()
        del tmp
        torch.cuda.empty_cache()
    data = torch.empty((total + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xC3)
    order, _ = m.plan_desc(lens.astype(np.uint32))
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    d_ord = torch.from_numpy(order.astype(np.int32)).cuda()
    out = torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    res = {"variant": a.variant}
    for mode in ("queued", "synced", "queued"):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)]
        torch.cuda.synchronize()
        ev[0].record(s)
        for k in range(a.steps):
            m.digest_desc(data, d_off, d_len, d_ord, out=out, variant=a.variant)
            ev[k + 1].record(s)
            if mode == "synced":
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        per = [round(ev[k].elapsed_time(ev[k + 1]), 3) for k in range(a.steps)]
        res.setdefault(mode, []).append({"per_launch_ms": per, "median": float(np.median(per))})
    print(json.dumps(res))


if __name__ == "__main__":
    main()
