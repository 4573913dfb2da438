#!/usr/bin/env python3
"""PROBE: a low-priority filler wave beside a lone MD5 chain wave on each
SIMD (scripts/probes/prio_fill.hip).  Reports the chain waves' time alone
and with fillers at s_setprio 0 (chain waves at prio 0..3), and the fillers'
compressions as a fraction of the chain waves' -- the share of the lone
wave's idle issue slots a second wave can take without slowing it.
usage: prio_fill.py --build | prio_fill.py [--out FILE]"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(REPO, "scripts", "probes", "prio_fill.hip")
SO = os.path.join(REPO, "build", "probes", "prio_fill.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.build:
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                        SRC, "-o", SO], check=True)
        return
    import torch
    P = ctypes.CDLL(SO)
    P.prio_fill_run.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_int, ctypes.c_uint32, ctypes.c_void_p,
                                ctypes.c_void_p, ctypes.c_void_p]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    fills = torch.zeros(cus * 4, dtype=torch.int32, device="cuda")
    out = torch.empty(cus * 512 * 4, dtype=torch.int32, device="cuda")
    iters = 2000
    res = {}
    for name, mode, hi in (("alone", 0, 0), ("fill_hi0", 1, 0), ("fill_hi1", 1, 1), ("fill_hi3", 1, 3)):
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        run = lambda: P.prio_fill_run(iters, mode, hi, cus, fills.data_ptr(), out.data_ptr(), st)  # noqa: E731
        for _ in range(3):
            assert run() == 0
        torch.cuda.synchronize()
        t = []
        for _ in range(9):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            t.append(e0.elapsed_time(e1))
        t.sort()
        ms = t[4]
        f = fills.float().mean().item() if mode else 0.0
        res[name] = {"ms": round(ms, 4), "chain_waves_prio": hi, "filler_compressions_per_chain": round(f / iters, 4)}
        print(name, json.dumps(res[name]), flush=True)
    base = res["alone"]["ms"]
    for k in res:
        res[k]["chain_time_vs_alone"] = round(res[k]["ms"] / base, 4)
        res[k]["simd_work_vs_alone"] = round((1 + res[k]["filler_compressions_per_chain"]) / (res[k]["ms"] / base), 4)
    rec = {"probe": "prio_fill", "iters": iters, "cus": cus, "results": res}
    print(json.dumps(rec))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        open(a.out, "w").write(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    main()
