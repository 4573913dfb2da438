#!/usr/bin/env python3
"""Does the placement of the 16 GiB input change the kernels' speed?  One
process per call: the batch buffer is either the process's first device
allocation ("fresh") or allocated after a 16 GiB block was allocated, filled
and freed ("prealloc").  Times the C2 product kernel (xdma1nt) and the C3 batch
with the HYBRID and XDMA descriptor kernels, 30 launches each, and reports the
buffer's virtual address alignment.  Prints one JSON object.

    python scripts/alloc_probe.py [--prealloc]"""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402


def per_launch(fn, steps=30, warmup=5):
    for _ in range(warmup):
        fn()
    s = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
    torch.cuda.synchronize()
    ev[0].record(s)
    for k in range(steps):
        fn()
        ev[k + 1].record(s)
    torch.cuda.synchronize()
    return float(np.median([ev[k].elapsed_time(ev[k + 1]) for k in range(steps)]))


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--prealloc", action="store_true")
    p.add_argument("--arena", action="store_true", help="md5hip_arena_alloc (1 GiB-aligned VA)")
    p.add_argument("--c2-all", action="store_true")
    a = p.parse_args()
    if a.prealloc:
        tmp = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
        m.fill_synthetic(tmp, seed=1)
        torch.cuda.synchronize()
        del tmp
        torch.cuda.empty_cache()
    n, L = 1 << 20, 16384
    data = (m.arena_empty(n * L + (64 << 20)) if a.arena else
            torch.empty(n * L + (64 << 20), dtype=torch.uint8, device="cuda"))
    m.fill_synthetic(data, seed=0xC3)
    addr = data.data_ptr()
    res = {"mode": "arena" if a.arena else "prealloc" if a.prealloc else "fresh", "addr": hex(addr),
           "align_log2": int((addr & -addr).bit_length() - 1)}
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    res["c2_xdma1nt_ms"] = per_launch(lambda: m.digest_fixed(data, n, L, out=out))
    if "--c2-all" in sys.argv:
        for v in ("direct2", "direct4", "xpose1nt"):
            res[f"c2_{v}_ms"] = per_launch(lambda: m.digest_fixed(data, n, L, out=out, variant=v))
        res["c2_xdma1nt_ms_again"] = per_launch(lambda: m.digest_fixed(data, n, L, out=out))
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
    assert offs[-1] + lens[-1] <= data.numel()
    order, _ = m.plan_desc(lens.astype(np.uint32))
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    d_ord = torch.from_numpy(order.astype(np.int32)).cuda()
    o3 = torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda")
    for v in ("hybrid", "xdma"):
        res[f"c3_{v}_ms"] = per_launch(lambda: m.digest_desc(data, d_off, d_len, d_ord, out=o3, variant=v))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
