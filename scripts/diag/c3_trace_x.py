#!/usr/bin/env python3
"""Where the time of a mixed (C3) descriptor launch goes, per wave and per
SIMD: K C3 batches (the bench's c3q/coalesced shapes) coalesced into one
planned launch, run through the product kernels' traced copies in the
diagnostic library (md5diag_desc_x: HW_ID, XCC_ID, s_memrealtime per wave).

Prints one JSON object: per kind, the launch time (hipEvent, untraced,
interleaved), and for the traced run the wave/SIMD statistics -- span,
per-SIMD busy time (sum of its waves' durations), SIMD end-time quantiles
(the tail), the long waves' durations against the 1 MiB chain alone.

usage: c3_trace_x.py [--batches K] [--rounds R]
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from sproxy_amd import md5 as m  # noqa: E402

DIAG = os.path.join(REPO, "build", "diag", "libmd5hip_diag.so")


def batch(K, seed0):
    lk = [bench.c3_lens(16 << 30, seed0 + 31 * j) for j in range(K)]
    ok_ = [bench.c3_offsets(x)[0] for x in lk]
    spans = [(bench.c3_offsets(x)[1] + 15) // 16 * 16 for x in lk]
    starts = np.concatenate([[0], np.cumsum(spans)[:-1]])
    big = m.arena_empty(int(sum(spans)))
    m.fill_synthetic(big, seed=0xC3D)
    L = np.concatenate(lk)
    O = np.concatenate([o + s for o, s in zip(ok_, starts)])
    order, var = m.plan_desc(L.astype(np.uint32))
    return big, L, O, order, var


def stats(rec, L, order, clk_hz=100e6, persistent=False):
    hw, xcc, t0, t1 = rec[:, 0], rec[:, 1], rec[:, 2].astype(np.int64), rec[:, 3].astype(np.int64)
    base = t0.min()
    s, e = (t0 - base) / clk_hz * 1e3, (t1 - base) / clk_hz * 1e3        # ms
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = (((xcc.astype(np.int64) * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    uniq, inv = np.unique(key, return_inverse=True)
    busy = np.bincount(inv, weights=e - s)
    end = np.zeros(uniq.size)
    np.maximum.at(end, inv, e)
    nw = np.bincount(inv)
    nwave = rec.shape[0]
    q = lambda a: [round(float(x), 3) for x in np.quantile(a, [0, 0.1, 0.5, 0.9, 1.0])]
    if persistent:
        return {"waves": int(nwave), "simds_used": int(uniq.size), "span_ms": round(float(e.max()), 3),
                "waves_per_simd_q": q(nw), "wave_end_ms_q": q(e), "groups_per_wave_q": q(rec[:, 4]),
                "busy_frac": round(float((e - s).sum() / (nwave * e.max())), 3)}
    wave_max = np.array([L[order[64 * w:64 * w + 64]].max() for w in range(nwave)])
    longw = wave_max == (1 << 20)
    return {"waves": int(nwave), "simds_used": int(uniq.size), "span_ms": round(float(e.max()), 3),
            "waves_per_simd_q": q(nw), "simd_busy_ms_q": q(busy), "simd_end_ms_q": q(end),
            "busy_sum_over_simds_x_span": round(float(busy.sum() / (uniq.size * e.max())), 3),
            "long_1mib_waves": int(longw.sum()),
            "long_wave_ms_q": q((e - s)[longw]) if longw.any() else None,
            "long_wave_start_ms_q": q(s[longw]) if longw.any() else None,
            "long_waves_per_simd_max": int(np.bincount(inv[longw]).max()) if longw.any() else 0}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batches", type=int, nargs="+", default=[1, 5])
    p.add_argument("--rounds", type=int, default=3)
    a = p.parse_args()
    D = ctypes.CDLL(DIAG)
    vp = ctypes.c_void_p
    D.md5diag_desc_x.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, vp]
    D.md5diag_desc_balanced.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, vp, vp, vp]
    BAL = {0: "bal_w4_nb1", 1: "bal_w4_nb2", 2: "bal_w8_nb1", 3: "bal_w8_split", 4: "bal_w8_split_nb2"}
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    out = {}
    for K in a.batches:
        big, L, O, order, var = batch(K, 3000)
        dO, dL = torch.from_numpy(O).cuda(), torch.from_numpy(L.astype(np.int32)).cuda()
        dR = torch.from_numpy(order.astype(np.int32)).cuda()
        n = L.size
        dig = {k: torch.empty((n, 16), dtype=torch.uint8, device="cuda") for k in range(3)}
        st = torch.cuda.current_stream().cuda_stream
        run = lambda k, rec=None: D.md5diag_desc_x(k, big.data_ptr(), dO.data_ptr(), dL.data_ptr(),  # noqa
                                                  dR.data_ptr(), n, dig[k].data_ptr(), cus,
                                                  rec.data_ptr() if rec is not None else None, st)
        for k in range(3):
            assert run(k) == 0
        torch.cuda.synchronize()
        ms = {k: [] for k in range(3)}
        for _ in range(a.rounds):
            for k in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                run(k)
                e1.record()
                torch.cuda.synchronize()
                ms[k].append(e0.elapsed_time(e1))
        for v in ("xdma", "hybrid", "balanced"):        # the product kernels themselves
            ms["product_" + v] = []
        for _ in range(a.rounds):
            for v in ("xdma", "hybrid", "balanced"):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                m.digest_desc(big, dO, dL, dR, out=dig[0], variant=v)
                e1.record()
                torch.cuda.synchronize()
                ms["product_" + v].append(e0.elapsed_time(e1))
        digb = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
        runb = lambda k, rec=None: D.md5diag_desc_balanced(k, big.data_ptr(), dO.data_ptr(), dL.data_ptr(),  # noqa
                                                          dR.data_ptr(), n, digb.data_ptr(),
                                                          rec.data_ptr() if rec is not None else None, st)
        for k in BAL:
            assert runb(k) == 0
            ms[BAL[k]] = []
        for _ in range(a.rounds):
            for k in BAL:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                runb(k)
                e1.record()
                torch.cuda.synchronize()
                ms[BAL[k]].append(e0.elapsed_time(e1))
        ref = m.digest_desc(big, dO, dL, dR, variant=var)
        assert run(0) == 0
        same = {k: bool(torch.equal(dig[k], ref)) for k in range(3)}
        res = {"chunks": int(n), "payload_gib": round(float(L.sum()) / 2**30, 2), "planner": var,
               "ms": {name: [round(x, 3) for x in ms[k]] for k, name in
                      ((0, "xdma"), (1, "hybrid_pair"), (2, "hybrid_nopair"), ("product_xdma", "product_xdma"),
                       ("product_hybrid", "product_hybrid"), ("product_balanced", "product_balanced"))
                      + tuple((v, v) for v in BAL.values())},
               "digests_equal_product": same}
        for k, name in ((0, "xdma"), (1, "hybrid_pair")):
            rec = torch.zeros(((n + 63) // 64, 4), dtype=torch.int64, device="cuda")
            assert run(k, rec) == 0
            torch.cuda.synchronize()
            res["trace_" + name] = stats(rec.cpu().numpy().astype(np.uint64), L, order)
        for k in (0, 3):
            recb = torch.zeros(((8 if k >= 2 else 4) * cus, 5), dtype=torch.int64, device="cuda")
            assert runb(k, recb) == 0
            torch.cuda.synchronize()
            res["trace_" + BAL[k]] = stats(recb.cpu().numpy().astype(np.uint64), L, order, persistent=True)
            res[BAL[k] + "_equal_product"] = bool(torch.equal(digb, ref))
        out[f"K{K}"] = res
        del big, dO, dL, dR, dig
        torch.cuda.empty_cache()
        print(json.dumps({f"K{K}": res}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
