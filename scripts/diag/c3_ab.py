#!/usr/bin/env python3
"""C3 (mixed lengths) A/B of the descriptor kernel: latency-form step (kLat)
x long-chain priority (kPrio), plus the single-chain latency probe and the
compute-only throughput of both step forms.  Interleaved in one process."""
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
D.md5diag_run.argtypes = [i, vp, u64, u32, u64, vp, vp]
D.md5diag_desc.argtypes = [i, vp, vp, vp, vp, u64, vp, vp]


def c3_batch(target, seed=1000):
    rng = np.random.default_rng(seed)
    classes = np.array([4096 << k for k in range(9)], dtype=np.int64)
    lens, tot = [], 0
    while tot < target:
        c = int(classes[rng.integers(0, 9)])
        if rng.integers(0, 8) == 0:
            c = int(rng.integers(1, c))
        lens.append(c)
        tot += c
    return np.array(lens, dtype=np.int64)


def timeit(f, reps=3, rounds=3):
    s = torch.cuda.current_stream()
    ts = []
    f()
    torch.cuda.synchronize()
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[len(ts) // 2]


def main():
    res = {}
    lens = c3_batch(16 << 30)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
    total = int(offs[-1] + lens[-1] + 16)
    data = torch.empty((total + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=3)
    order = torch.from_numpy(m.plan_order(lens.astype(np.uint32)).astype(np.int32)).cuda()
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    out = torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    ref = None
    cases = [(0, "r1"), (1, "lat_prio_D2"), (3, "D8"), (16, "r1_t64"),
             (17, "lat_prio_D2_t64"), (18, "D4_t64"), (19, "D8_t64"), (20, "D8_noprio_t64"),
             (22, "D8_pair_t64")]
    if "--pair" in sys.argv:
        cases = [(19, "D8_t64"), (22, "D8_pair_t64"), (19, "D8_t64_again"), (22, "D8_pair_t64_again")]
    for kind, name in cases:
        f = lambda: D.md5diag_desc(kind, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),  # noqa
                                   order.data_ptr(), lens.size, out.data_ptr(), st)
        ms = timeit(f, reps=2, rounds=3)
        if ref is None:
            ref = out.clone()
        assert torch.equal(out, ref), name
        res["c3_" + name] = {"ms": round(ms, 3), "GBps": round(lens.sum() / ms / 1e6, 1)}
    if "--pair" in sys.argv:
        print(json.dumps(res))
        return
    del data
    torch.cuda.empty_cache()
    # uniform small chunks through the descriptor kernel (occupancy check)
    n4 = 1 << 22
    lens4 = np.full(n4, 4096, dtype=np.int64)
    offs4 = torch.arange(n4, dtype=torch.int64, device="cuda") * 4096
    d4 = torch.empty(n4 * 4096, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(d4, seed=4)
    l4 = torch.from_numpy(lens4.astype(np.int32)).cuda()
    o4 = torch.empty((n4, 16), dtype=torch.uint8, device="cuda")
    for kind, name in [(0, "r1"), (1, "lat_prio_D2"), (3, "D8"), (16, "r1_t64"), (17, "lat_prio_D2_t64"),
                       (19, "D8_t64")]:
        f = lambda: D.md5diag_desc(kind, d4.data_ptr(), offs4.data_ptr(), l4.data_ptr(), None,  # noqa
                                   n4, o4.data_ptr(), st)
        ms = timeit(f, reps=3, rounds=3)
        res["u4k_" + name] = {"ms": round(ms, 3), "GBps": round(n4 * 4096 / ms / 1e6, 1)}
    del d4
    torch.cuda.empty_cache()
    # single-chain latency: 16384 lanes = one wave per CU, 1 MiB each (no HBM)
    buf = torch.empty(16384 * 16 + 1 << 20, dtype=torch.uint8, device="cuda")
    for kind, name in [(13, "chain_base"), (14, "chain_lat")]:
        f = lambda: D.md5diag_run(kind, None, 16384, 1 << 20, 0, buf.data_ptr(), st)  # noqa
        ms = timeit(f, reps=1, rounds=3)
        res[name] = {"ms": round(ms, 3), "us_per_block": round(ms * 1e3 / 16385, 4)}
    for kind, name in [(0, "throughput_base"), (12, "throughput_lat")]:
        f = lambda: D.md5diag_run(kind, None, 1 << 20, 16384, 0, buf.data_ptr(), st)  # noqa
        res[name] = {"ms": round(timeit(f, reps=10, rounds=3), 4)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
