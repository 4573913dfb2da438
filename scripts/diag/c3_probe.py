#!/usr/bin/env python3
"""Where does C3's time go?  Per-class batches (same chunk counts as C3 draws)
through the descriptor kernel and the fixed kernels."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

D = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
D.md5diag_desc.argtypes = [i, vp, vp, vp, vp, u64, vp, vp]
D.md5diag_run.argtypes = [i, vp, u64, u32, u64, vp, vp]


def timeit(f, reps=2, rounds=3):
    s = torch.cuda.current_stream()
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[1]


res = {}
st = torch.cuda.current_stream().cuda_stream
for L, n in [(1 << 20, 8832), (1 << 20, 16384), (1 << 18, 8832), (1 << 16, 8832), (1 << 20, 2048)]:
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=5)
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * L
    lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
    key = f"{L >> 10}KiBx{n}"
    r = {}
    for v in ("xpose1nt", "direct2", "direct4"):
        r[v] = round(timeit(lambda: m.digest_fixed(data, n, L, out=out, variant=v)), 3)
    for kind, name in [(0, "desc_r1"), (3, "desc_D8")]:
        r[name] = round(timeit(lambda: D.md5diag_desc(kind, data.data_ptr(), offs.data_ptr(),
                                                      lens.data_ptr(), None, n, out.data_ptr(), st)), 3)
    buf = torch.empty(n * 16 + 1024, dtype=torch.uint8, device="cuda")
    r["chain_compute_only_64thr"] = round(timeit(lambda: D.md5diag_run(13, None, n, L, 0, buf.data_ptr(), st)), 3)
    r["chain_compute_only_256thr"] = round(timeit(lambda: D.md5diag_run(0, None, n, L, 0, buf.data_ptr(), st)), 3)
    res[key] = r
    del data
    torch.cuda.empty_cache()
print(json.dumps(res))
