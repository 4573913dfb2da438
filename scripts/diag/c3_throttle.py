#!/usr/bin/env python3
"""C3 experiment: does the mixed batch finish sooner if its short chunks run
throttled beside the long chains (so the board stays under its power cap and
the chains keep the top clock)?  The bench's C3 batch is split at --split
bytes into a long and a short descriptor batch; the long one runs on stream
A, the short one on stream B with extra LDS per workgroup capping how many of
its waves a CU holds.  Prints one JSON object (ms, median of --reps)."""
import argparse
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
vp, u64, u32 = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32
D.md5diag_desc_xpose_lds.argtypes = [vp, vp, vp, vp, u64, vp, u32, vp]


def c3_lens(target, seed=1000):
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


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--split", type=int, default=256 << 10)
    p.add_argument("--reps", type=int, default=7)
    a = p.parse_args()
    lens = c3_lens(16 << 30)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
    total = int(offs[-1] + lens[-1] + 16)
    data = torch.empty((total + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xC3)

    def part(mask):
        L, O = lens[mask], offs[mask]
        order = m.plan_order(L.astype(np.uint32)).astype(np.int32)
        return (torch.from_numpy(O).cuda(), torch.from_numpy(L.astype(np.int32)).cuda(),
                torch.from_numpy(order).cuda(), int(mask.sum()), np.nonzero(mask)[0])

    full = part(np.ones(lens.size, dtype=bool))
    long_ = part(lens >= a.split)
    short = part(lens < a.split)
    out_full = torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda")
    out_l = torch.empty((long_[3], 16), dtype=torch.uint8, device="cuda")
    out_s = torch.empty((short[3], 16), dtype=torch.uint8, device="cuda")
    cur = torch.cuda.current_stream()
    sa, sb = torch.cuda.Stream(), torch.cuda.Stream()

    def launch(pt, out, extra, stream):
        rc = D.md5diag_desc_xpose_lds(data.data_ptr(), pt[0].data_ptr(), pt[1].data_ptr(),
                                      pt[2].data_ptr(), pt[3], out.data_ptr(), extra,
                                      stream.cuda_stream)
        assert rc == 0, rc

    def timed(fn):
        ts = []
        fn()
        torch.cuda.synchronize()
        for _ in range(a.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(cur)
            fn()
            e1.record(cur)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        return round(sorted(ts)[len(ts) // 2], 3)

    def concurrent(extra):
        def f():
            sa.wait_stream(cur)
            sb.wait_stream(cur)
            launch(long_, out_l, 0, sa)
            launch(short, out_s, extra, sb)
            cur.wait_stream(sa)
            cur.wait_stream(sb)
        return f

    res = {"split": a.split, "n_long": long_[3], "n_short": short[3],
           "full": timed(lambda: launch(full, out_full, 0, cur)),
           "long_only": timed(lambda: launch(long_, out_l, 0, cur)),
           "short_only": timed(lambda: launch(short, out_s, 0, cur))}
    ref = out_full.cpu().numpy()

    def long_lane(stream):
        with torch.cuda.stream(stream):
            m.digest_desc(data, long_[0], long_[1], long_[2], out=out_l, variant="lane")

    res["long_only_lane"] = timed(lambda: long_lane(cur))

    def concurrent_lane():
        sa.wait_stream(cur)
        sb.wait_stream(cur)
        long_lane(sa)
        launch(short, out_s, 0, sb)
        cur.wait_stream(sa)
        cur.wait_stream(sb)

    res["concurrent_long_lane_short_xpose"] = timed(concurrent_lane)
    assert np.array_equal(out_l.cpu().numpy(), ref[long_[4]])
    for extra in (0, 40960):
        res[f"concurrent_extra{extra}"] = timed(concurrent(extra))
        res[f"short_only_extra{extra}"] = timed(lambda: launch(short, out_s, extra, cur))
        got_l, got_s = out_l.cpu().numpy(), out_s.cpu().numpy()
        assert np.array_equal(got_l, ref[long_[4]]) and np.array_equal(got_s, ref[short[4]]), extra
    print(json.dumps(res))


if __name__ == "__main__":
    main()
