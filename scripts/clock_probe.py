#!/usr/bin/env python3
"""In-kernel clock of the product kernel vs the compute-only kernel
(MI355X_MICROARCH 'DVFS give-back' item 6): >= 2 s of back-to-back launches of
each, then per-wave (s_memtime, s_memrealtime) deltas -> median GHz.
    python scripts/clock_probe.py [--secs S]"""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

DIAG = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
DIAG.md5diag_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--secs", type=float, default=2.0)
    p.add_argument("--kinds", default="48,49")
    a = p.parse_args()
    n, L = 1 << 20, 16384
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=1)
    waves = n // 64
    out = torch.zeros(n * 16 + waves * 16, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    res = {}
    for rnd in range(2):
        for kind in [int(k) for k in a.kinds.split(",")]:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = max(1, int(a.secs / 3e-3))
            e0.record(s)
            for _ in range(reps):
                assert DIAG.md5diag_run(kind, data.data_ptr(), n, L, L, out.data_ptr(), s.cuda_stream) == 0
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1) / reps
            clk = out[n * 16:].view(torch.int64).view(-1, 2).cpu().double()
            ghz = (clk[:, 0] / clk[:, 1]).median().item() * 0.1
            wave_us = (clk[:, 1] / 100.0).median().item()
            res[f"kind{kind}_round{rnd}"] = {"ms_per_launch": round(ms, 4), "clock_ghz_median": round(ghz, 3),
                                            "wave_us_median": round(wave_us, 1),
                                            "wave_cycles_median": int((clk[:, 0]).median().item())}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
