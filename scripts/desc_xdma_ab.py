#!/usr/bin/env python3
"""Descriptor kernel A/B: XPOSE (VGPR-staged image, the default) vs XDMA
(image filled by LDS-DMA) vs the fixed-length xdma1nt kernel on netcache-shaped
16 GiB batches (chunk_size 4-256 KiB, 1 in 8 chunks a ragged last block,
longest-first lanes) and on the C3 mixed batch.  Interleaved: every round
times each kernel once, the order rotating per round.  Also checks the two
descriptor kernels' digests are identical.  Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

GIB = float(1 << 30)


def time_once(f, reps=5):
    s = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(reps):
        f()
    e1.record(s)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def ab(fns, rounds=6):
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    ts = {k: [] for k in fns}
    keys = list(fns)
    for r in range(rounds):
        for k in keys[r % len(keys):] + keys[:r % len(keys)]:
            ts[k].append(time_once(fns[k]))
    return {k: round(float(np.median(v)), 4) for k, v in ts.items()}


def main():
    data = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xD3A)
    res = {}
    for S in (4096, 16384, 65536, 262144):
        n = (16 << 30) // S
        rng = np.random.default_rng(S)
        lens = np.full(n, S, dtype=np.int64)
        tail = rng.integers(0, 8, n) == 0
        lens[tail] = rng.integers(1, S, int(tail.sum()))
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * S
        d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
        order = torch.from_numpy(m.plan_order(lens.astype(np.uint32)).astype(np.int32)).cuda()
        outs = {k: torch.empty((n, 16), dtype=torch.uint8, device="cuda") for k in ("xpose", "xdma", "fixed")}
        fns = {k: (lambda k=k: m.digest_desc(data, offs, d_len, order, out=outs[k], variant=k))
               for k in ("xpose", "xdma")}
        fns["fixed"] = lambda: m.digest_fixed(data, n, S, out=outs["fixed"])
        t = ab(fns)
        same = bool(torch.equal(outs["xpose"], outs["xdma"]))
        res[f"ragged_{S}"] = {"ms": t, "payload_GiBps": {k: round(float(lens.sum()) / GIB / (v * 1e-3), 1)
                                                         for k, v in t.items() if k != "fixed"},
                              "digests_equal": same}
        print(json.dumps({S: res[f"ragged_{S}"]}), file=sys.stderr, flush=True)
        assert same
        del outs
    # C3 mixed batch (bench.py run_c3 shape)
    rng = np.random.default_rng(1000)
    classes = [4096 << k for k in range(9)]
    lens, tot = [], 0
    while tot < (16 << 30) - (2 << 20):
        c = classes[int(rng.integers(0, 9))]
        if rng.integers(0, 8) == 0:
            c = int(rng.integers(1, c))
        lens.append(c)
        tot += c
    lens = np.array(lens, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
    keep = offs + lens <= data.numel()
    lens, offs = lens[keep], offs[keep]
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    order = torch.from_numpy(m.plan_order(lens.astype(np.uint32)).astype(np.int32)).cuda()
    outs = {k: torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda") for k in ("xpose", "xdma")}
    fns = {k: (lambda k=k: m.digest_desc(data, d_off, d_len, order, out=outs[k], variant=k))
           for k in ("xpose", "xdma")}
    t = ab(fns, rounds=4)
    res["c3_mixed"] = {"ms": t, "chunks": int(lens.size), "digests_equal": bool(torch.equal(outs["xpose"], outs["xdma"]))}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
