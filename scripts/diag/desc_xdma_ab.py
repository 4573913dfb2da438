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

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
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


def ab(fns, rounds=6, reps=5):
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    ts = {k: [] for k in fns}
    keys = list(fns)
    for r in range(rounds):
        for k in keys[r % len(keys):] + keys[:r % len(keys)]:
            ts[k].append(time_once(fns[k], reps))
    return {k: round(float(np.median(v)), 4) for k, v in ts.items()}


def main():
    data = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xD3A)
    res = {}
    sweep = (4096, 16384, 65536, 262144, 524288, 1048576)
    kinds = ("xdma", "hybrid") if "--hybrid" in sys.argv else ("xpose", "xdma")
    for S in (() if "--c3-only" in sys.argv else sweep):
        n = (16 << 30) // S
        rng = np.random.default_rng(S)
        lens = np.full(n, S, dtype=np.int64)
        tail = rng.integers(0, 8, n) == 0
        lens[tail] = rng.integers(1, S, int(tail.sum()))
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * S
        d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
        order = torch.from_numpy(m.plan_order(lens.astype(np.uint32)).astype(np.int32)).cuda()
        outs = {k: torch.empty((n, 16), dtype=torch.uint8, device="cuda") for k in kinds + ("fixed",)}
        fns = {k: (lambda k=k: m.digest_desc(data, offs, d_len, order, out=outs[k], variant=k))
               for k in kinds}
        fns["fixed"] = lambda: m.digest_fixed(data, n, S, out=outs["fixed"])
        t = ab(fns)
        same = bool(torch.equal(outs[kinds[0]], outs[kinds[1]]))
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
    exact = "--bench-batch" in sys.argv     # bench.py run_c3's batch exactly (own arena)
    while tot < (16 << 30) - (0 if exact else 2 << 20):
        c = classes[int(rng.integers(0, 9))]
        if rng.integers(0, 8) == 0:
            c = int(rng.integers(1, c))
        lens.append(c)
        tot += c
    lens = np.array(lens, dtype=np.int64)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
    if exact:
        del data
        torch.cuda.empty_cache()
        total = int(offs[-1] + lens[-1] + 16)
        data = torch.empty((total + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
        m.fill_synthetic(data, seed=0xC3)
    keep = offs + lens <= data.numel()
    lens, offs = lens[keep], offs[keep]
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    order = torch.from_numpy(m.plan_order(lens.astype(np.uint32)).astype(np.int32)).cuda()
    ks = ("xdma", "hybrid") if "--hybrid" in sys.argv else ("xpose", "xdma", "hybrid")
    outs = {k: torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda") for k in ks}
    fns = {k: (lambda k=k: m.digest_desc(data, d_off, d_len, order, out=outs[k], variant=k)) for k in ks}
    t = ab(fns, rounds=6)
    res["c3_mixed_sustained50"] = ab(fns, rounds=2, reps=50)
    if "--solo" in sys.argv:      # each kernel alone, 3 x 50 back-to-back, no alternation
        res["c3_mixed_solo"] = {k: ab({k: f}, rounds=3, reps=50)[k] for k, f in fns.items()}
    res["c3_mixed"] = {"ms": t, "chunks": int(lens.size),
                       "digests_equal": all(torch.equal(outs[ks[0]], outs[k]) for k in ks)}
    # its longest chunks alone (the batch's serial-chain bound)
    il = np.flatnonzero(lens == lens.max())
    o1, l1 = torch.from_numpy(offs[il]).cuda(), torch.from_numpy(lens[il].astype(np.int32)).cuda()
    out1 = torch.empty((il.size, 16), dtype=torch.uint8, device="cuda")
    res["c3_longest_alone"] = {"n": int(il.size), "ms": ab({k: (lambda k=k: m.digest_desc(
        data, o1, l1, out=out1, variant=k)) for k in ks}, rounds=4)}
    if "--c3-only" in sys.argv:
        res = {k: v for k, v in res.items() if k.startswith("c3")}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
