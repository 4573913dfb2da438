#!/usr/bin/env python3
"""Why the first ~15 C2 launches run slow.

Replays bench.py's C2 sequence (16 GiB torch.empty, md5hip_fill_synthetic,
then back-to-back launches with no host gap) with the product kernel body
carrying per-wave clock stamps (diag kind 90 = md5_fixed_xdma1nt + s_memtime /
s_memrealtime), one clock buffer per launch.  Per launch: hipEvent ms, median
in-kernel shader clock (GHz), median wave time, the launch's span on the
device's 100 MHz clock, and the idle gap before it.

    python scripts/startup_probe.py --mode bench|arena|gap|compute|loads|repeat
        [--launches 25]

  bench    exactly bench.py's order: torch.empty, fill, 25 launches
  arena    the batch in md5hip_arena_alloc memory (1 GiB-aligned VA) instead
  gap      bench, but 0.5 s idle between the fill and the first launch
  prefill  the fill re-run just before the launches (two fills)
  compute  the compute-only body (kind 49: MD5 on LDS words, no HBM reads)
  loads    the load-only body (kind 50: the same loads, a fold for a hash)
  repeat   bench, then 1 s idle, then the launches again
"""
import argparse
import ctypes
import json
import os
import sys
import time

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

DIAG = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
DIAG.md5diag_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]


def run_launches(kind, data, n, L, k, words):
    waves = n // 64
    s = torch.cuda.current_stream()
    outs = [torch.zeros(n * 16 + waves * 8 * words, dtype=torch.uint8, device="cuda") for _ in range(k)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(k + 1)]
    torch.cuda.synchronize()
    ev[0].record(s)
    for i in range(k):
        assert DIAG.md5diag_run(kind, data.data_ptr(), n, L, L, outs[i].data_ptr(), s.cuda_stream) == 0
        ev[i + 1].record(s)
    torch.cuda.synchronize()
    rows, prev_end = [], None
    for i in range(k):
        clk = outs[i][n * 16:].view(torch.int64).view(waves, words).cpu().double()
        ghz = (clk[:, 0] / clk[:, 1]).median().item() * 0.1
        r = {"launch": i + 1, "ms": round(ev[i].elapsed_time(ev[i + 1]), 4), "ghz": round(ghz, 3),
             "wave_us": round((clk[:, 1] / 100.0).median().item(), 2)}
        if words == 4:
            t0, t1 = clk[:, 2].min().item(), clk[:, 3].max().item()
            r["span_ms"] = round((t1 - t0) / 1e5, 4)
            if prev_end is not None:
                r["gap_us"] = round((t0 - prev_end) / 100.0, 1)
            prev_end = t1
        rows.append(r)
    return rows


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--mode", default="bench")
    p.add_argument("--launches", type=int, default=25)
    a = p.parse_args()
    n, L = 1 << 20, 16384
    t_start = time.time()
    if a.mode == "arena":
        data = m.arena_empty(n * L)
    else:
        data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0x5EED0000)
    if a.mode == "prefill":
        m.fill_synthetic(data, seed=0x5EED0000)
    if a.mode == "gap":
        torch.cuda.synchronize()
        time.sleep(0.5)
    kind, words = {"compute": (49, 2), "loads": (50, 2)}.get(a.mode, (90, 4))
    res = {"mode": a.mode, "kind": kind, "launches": run_launches(kind, data, n, L, a.launches, words)}
    if a.mode == "repeat":
        time.sleep(1.0)
        res["after_1s_idle"] = run_launches(kind, data, n, L, a.launches, words)
    res["wall_s"] = round(time.time() - t_start, 2)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
