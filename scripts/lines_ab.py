#!/usr/bin/env python3
"""XDMA against LINES (md5hip_digest_desc_variant 4 vs 7) on netcache-shaped
descriptor batches in one process: 983,040 blocks of 16 KiB with 1-in-8
ragged tails (~15 GiB), packed at 16 B, at 128 B, and uniform 16 KiB.
Interleaved rounds, hipEvent ms per launch, digests of the two compared.
Under rocprofv3 --pmc FETCH_SIZE the two kernels (md5_desc_xdma,
md5_desc_lines) give the HBM bytes of each shape (--shapes to restrict).
Prints one JSON object.
usage: lines_ab.py [--rounds 7] [--shapes packed16,packed128,uniform]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402


def shape(name, nb=983040, S=16384, seed=5):
    rng = np.random.default_rng(seed)
    bl = np.full(nb, S, dtype=np.int64)
    if name != "uniform":
        tail = rng.integers(0, 8, nb) == 0
        bl[tail] = rng.integers(1, S, int(tail.sum()))
    align = 16 if name == "packed16" else 128
    offs = np.concatenate([[0], np.cumsum((bl + align - 1) // align * align)[:-1]]).astype(np.int64)
    return bl, offs


def timed(f):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    ap.add_argument("--shapes", default="packed16,packed128,uniform")
    a = ap.parse_args()
    res = {}
    for name in a.shapes.split(","):
        bl, offs = shape(name)
        nb = bl.size
        arena = m.arena_empty(int(offs[-1] + bl[-1] + 256))
        m.fill_synthetic(arena, seed=0x16)
        order, planned = m.plan_desc(bl.astype(np.uint32))
        _, planned_at = m.plan_desc_at(bl.astype(np.uint32), offs.astype(np.uint64))
        dO = torch.from_numpy(offs).cuda()
        dL = torch.from_numpy(bl.astype(np.int32)).cuda()
        dR = torch.from_numpy(order.astype(np.int32)).cuda()
        outs = {v: torch.empty((nb, 16), dtype=torch.uint8, device="cuda") for v in ("xdma", "lines")}
        run = {v: (lambda v=v: m.digest_desc(arena, dO, dL, dR, out=outs[v], variant=v)) for v in outs}
        for v in run:
            run[v]()
        torch.cuda.synchronize()
        equal = bool(torch.equal(outs["xdma"], outs["lines"]))
        for _ in range(3):
            for v in run:
                run[v]()
        torch.cuda.synchronize()
        ms = {v: [] for v in run}
        for _ in range(a.rounds):
            for v in run:
                ms[v].append(round(timed(run[v]), 4))
        med = {v: sorted(x)[len(x) // 2] for v, x in ms.items()}
        res[name] = {"chunks": int(nb), "payload_bytes": int(bl.sum()), "equal": equal,
                     "plan_desc": planned, "plan_desc_at": planned_at, "ms": ms, "median_ms": med,
                     "lines_vs_xdma": round(med["xdma"] / med["lines"], 4),
                     "payload_tb_s": {v: round(int(bl.sum()) / (med[v] * 1e-3) / 1e12, 3) for v in med}}
        print(json.dumps({name: res[name]}), flush=True)
        del arena, dO, dL, dR, outs, run
        torch.cuda.empty_cache()
    print(json.dumps(res))
    return 0 if all(r["equal"] for r in res.values()) else 1


if __name__ == "__main__":
    sys.exit(main())
