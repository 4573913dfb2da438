#!/usr/bin/env python3
"""MD5Update on few contexts (md5hip_update_ctx, n x 16 KiB per update,
16-B aligned data, no pending bytes): the fed pairs (md5_update_ctx_fed)
against the loader kernel of the library before them, HIP events per launch
(after 10 untimed), interleaved; the resulting contexts compared.
usage: ctx_small_ab.py --lib name=path ... [--sizes 64,1024,16384]"""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
vp, u64 = ctypes.c_void_p, ctypes.c_uint64


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", nargs="+", required=True)
    ap.add_argument("--sizes", default="64,1024,16384")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    libs = {}
    for spec in a.lib:
        k, p = spec.split("=", 1)
        L = ctypes.CDLL(os.path.join(REPO, p), mode=ctypes.RTLD_LOCAL)
        L.md5hip_init_ctx.argtypes = [vp, u64, vp]
        L.md5hip_update_ctx.argtypes = [vp, vp, vp, u64, vp]
        L.md5hip_fill_synthetic.argtypes = [vp, u64, u64, vp]
        libs[k] = L
    first = next(iter(libs.values()))
    nmax = max(int(x) for x in a.sizes.split(","))
    Lb = 16384
    data = torch.empty(nmax * Lb, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    assert first.md5hip_fill_synthetic(data.data_ptr(), data.numel(), 7, st) == 0
    out = {"len": Lb, "sizes": {}}
    for n in (int(x) for x in a.sizes.split(",")):
        ptrs = (torch.arange(n, dtype=torch.int64, device="cuda") * Lb + data.data_ptr())
        lens = torch.full((n,), Lb, dtype=torch.int32, device="cuda")
        ctx = {k: torch.zeros((n, 88), dtype=torch.uint8, device="cuda") for k in libs}
        ms = {k: [] for k in libs}
        for k, L in libs.items():
            assert L.md5hip_init_ctx(ctx[k].data_ptr(), n, st) == 0
            assert L.md5hip_update_ctx(ctx[k].data_ptr(), ptrs.data_ptr(), lens.data_ptr(), n, st) == 0
        torch.cuda.synchronize()
        same = all(torch.equal(ctx[k], ctx[next(iter(libs))]) for k in libs)
        for _ in range(2):
            for k, L in libs.items():
                for _w in range(10):
                    L.md5hip_update_ctx(ctx[k].data_ptr(), ptrs.data_ptr(), lens.data_ptr(), n, st)
                ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]
                for i in range(a.iters):
                    ev[2 * i].record()
                    L.md5hip_update_ctx(ctx[k].data_ptr(), ptrs.data_ptr(), lens.data_ptr(), n, st)
                    ev[2 * i + 1].record()
                torch.cuda.synchronize()
                ms[k] += [ev[2 * i].elapsed_time(ev[2 * i + 1]) * 1e3 for i in range(a.iters)]
        row = {k: round(sorted(v)[len(v) // 2], 1) for k, v in ms.items()}
        row["contexts_equal_after_first_update"] = same
        out["sizes"][str(n)] = row
        print(n, json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
