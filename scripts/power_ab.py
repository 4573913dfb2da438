#!/usr/bin/env python3
"""Back-to-back runs (~secs each) of C2-shape kernels for board-power
sampling (scripts/power_probe.sh samples rocm-smi meanwhile).  Prints one JSON
object: per case, wall start/end (time.time) and ms per launch.
    python scripts/power_ab.py --cases xpose1nt,diag:6,...  [--secs S]"""
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--cases", required=True)
    p.add_argument("--secs", type=float, default=4.0)
    a = p.parse_args()
    n, L = 1 << 20, 16384
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=1)
    out = torch.zeros(max(n, 8192 * 256) * 16 + (n // 64) * 16, dtype=torch.uint8, device="cuda")
    crc_out = torch.empty(n, dtype=torch.int32, device="cuda")
    s = torch.cuda.current_stream()
    res = {}
    for case in a.cases.split(","):
        if case.startswith("diag:"):
            kind = int(case[5:])
            f = lambda: DIAG.md5diag_run(kind, data.data_ptr(), n, L, L, out.data_ptr(), s.cuda_stream)  # noqa
        elif case.startswith("crc:"):
            v = case[4:]
            f = lambda: m.crc32_fixed(data, n, L, out=crc_out, variant=v)  # noqa
        else:
            f = lambda: m.digest_fixed(data, n, L, out=out[:n * 16].view(n, 16), variant=case)  # noqa
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 0
        t0 = time.time()
        e0.record(s)
        while time.time() - t0 < a.secs:
            for _ in range(50):
                f()
            reps += 50
            torch.cuda.synchronize()
        e1.record(s)
        torch.cuda.synchronize()
        t1 = time.time()
        res[case] = {"t0": t0, "t1": t1, "ms": round(e0.elapsed_time(e1) / reps, 4)}
        time.sleep(1.0)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
