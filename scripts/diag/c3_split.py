#!/usr/bin/env python3
"""C3 A/B: one descriptor launch (64-thread workgroups, D=8 ring, priority)
vs a split launch -- the longest chunks in a kernel that holds the whole
register file (md5diag_desc kind 7: one wave per SIMD, so a long serial chain
never shares its SIMD) on one stream, the rest concurrently on a second
stream.  Prints one JSON object."""
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts", "diag"))
from sproxy_amd import md5 as m  # noqa: E402
from c3_ab import c3_batch  # noqa: E402

D = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
vp, u64, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
D.md5diag_desc.argtypes = [i, vp, vp, vp, vp, u64, vp, vp]


def main():
    lens = c3_batch(16 << 30)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
    total = int(offs[-1] + lens[-1] + 16)
    data = torch.empty((total + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=3)
    order_h = m.plan_order(lens.astype(np.uint32))
    order = torch.from_numpy(order_h.astype(np.int32)).cuda()
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    out = torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda")
    N = lens.size
    s0 = torch.cuda.current_stream()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    sorted_lens = lens[order_h]

    def one():
        D.md5diag_desc(19, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), order.data_ptr(), N,
                       out.data_ptr(), s0.cuda_stream)

    def split(na, hog_kind):
        def f():
            ev = torch.cuda.Event()
            ev.record(s0)
            s1.wait_event(ev)
            s2.wait_event(ev)
            D.md5diag_desc(hog_kind, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), order.data_ptr(),
                           na, out.data_ptr(), s1.cuda_stream)
            D.md5diag_desc(19, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                           order.data_ptr() + 4 * na, N - na, out.data_ptr(), s2.cuda_stream)
            e1, e2 = torch.cuda.Event(), torch.cuda.Event()
            e1.record(s1)
            e2.record(s2)
            s0.wait_event(e1)
            s0.wait_event(e2)
        return f

    def timeit(f, rounds=5):
        f()
        torch.cuda.synchronize()
        ts = []
        for _ in range(rounds):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s0)
            f()
            b.record(s0)
            torch.cuda.synchronize()
            ts.append(a.elapsed_time(b))
        return sorted(ts)[len(ts) // 2]

    res = {"chunks": int(N), "bytes": int(lens.sum())}
    one()
    torch.cuda.synchronize()
    ref = out.clone()
    cases = [("one", one)]
    for thr in (1 << 20, 512 << 10, 256 << 10, 128 << 10):
        na = int((sorted_lens >= thr).sum()) // 64 * 64
        cases.append((f"split_ge{thr >> 10}k_n{na}", split(na, 23)))
        cases.append((f"split_ge{thr >> 10}k_n{na}_nohog", split(na, 19)))
    cases.append(("one_again", one))
    for name, f in cases:
        out.zero_()
        ms = timeit(f)
        assert torch.equal(out, ref), name
        res[name] = {"ms": round(ms, 3), "GiBps": round(lens.sum() / ms / 1e-3 / 2**30, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
