#!/usr/bin/env python3
"""BALANCED on K coalesced C3 batches: what the memory side of the one-wave-
per-SIMD descriptor kernel can deliver, and whether wider stages (W x 128 B
contiguous per chunk per visit) or a second buffer help.

For each diagnostic kind of md5diag_desc_balanced (md5_diag.hip: waves per
WG / buffers / stages per wide stage, with and without the compression) the
launch time (hipEvent, interleaved rounds) and the payload rate; the hashing
kinds' digests are compared with the product kernel's.

usage: c3_wide_ab.py [--batches K ...] [--rounds R] [--kinds k ...]
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
sys.path.insert(0, os.path.join(REPO, "scripts", "diag"))
from c3_trace_x import DIAG, batch  # noqa: E402
from sproxy_amd import md5 as m  # noqa: E402

NAMES = {0: "w4_nb1_s1", 1: "w4_nb2_s1", 5: "w4_nb1_s2", 6: "w4_nb1_s4", 7: "w4_nb2_s2",
         8: "loads_w4_nb1_s1", 9: "loads_w4_nb1_s2", 10: "loads_w4_nb1_s4", 11: "loads_w4_nb2_s2",
         12: "loads_w4_nb2_s1", 13: "loads_w8_nb1_s1", 14: "w4_nb1_s5", 15: "loads_w4_nb1_s5",
         16: "w4_nb1_s4_cached", 17: "loads_w4_nb1_s4_cached", 18: "w4_nb1_s2_cached", 19: "w4_nb1_s1_cached",
         20: "w4_nb2_s1_cached", 21: "w8_nb1_s1_cached", 22: "loads_w4_nb1_s1_cached",
         23: "w8_split_s1_cached", 24: "product_shape_long_lane_256k", 25: "product_shape_long_lane_1m",
         26: "product_shape_3_images_regpipe"}
HASHING = (0, 1, 5, 6, 7, 14, 16, 18, 19, 20, 21, 23, 24, 25, 26)
PRODUCT = ("balanced", "hybrid", "xdma")


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batches", type=int, nargs="+", default=[3, 5])
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--kinds", type=int, nargs="*", default=sorted(NAMES))
    a = p.parse_args()
    D = ctypes.CDLL(DIAG)
    vp = ctypes.c_void_p
    D.md5diag_desc_balanced.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, vp, vp, vp]
    out = {}
    for K in a.batches:
        big, L, O, order, var = batch(K, 3000)
        dO, dL = torch.from_numpy(O).cuda(), torch.from_numpy(L.astype(np.int32)).cuda()
        dR = torch.from_numpy(order.astype(np.int32)).cuda()
        n = L.size
        payload = float(L.sum())
        st = torch.cuda.current_stream().cuda_stream
        dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
        run = lambda k: D.md5diag_desc_balanced(k, big.data_ptr(), dO.data_ptr(), dL.data_ptr(),  # noqa
                                                dR.data_ptr(), n, dig.data_ptr(), None, st)
        ref = m.digest_desc(big, dO, dL, dR, variant="balanced")
        same = {}
        for k in a.kinds:
            assert run(k) == 0, k
            torch.cuda.synchronize()
            if k in HASHING:
                same[NAMES[k]] = bool(torch.equal(dig, ref))
        ms = {NAMES[k]: [] for k in a.kinds}
        for v in PRODUCT:
            ms["product_" + v] = []
        for _ in range(a.rounds):
            for k in a.kinds + list(PRODUCT):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if isinstance(k, str):
                    m.digest_desc(big, dO, dL, dR, out=dig, variant=k)
                else:
                    run(k)
                e1.record()
                torch.cuda.synchronize()
                ms["product_" + k if isinstance(k, str) else NAMES[k]].append(e0.elapsed_time(e1))
        res = {"chunks": int(n), "payload_gib": round(payload / 2**30, 2), "planner": var,
               "ms": {k: [round(x, 3) for x in v] for k, v in ms.items()},
               "gb_s_best": {k: round(payload / min(v) / 1e6, 1) for k, v in ms.items()},
               "digests_equal_product": same}
        out[f"K{K}"] = res
        print(json.dumps({f"K{K}": res}), flush=True)
        del big, dO, dL, dR, dig, ref
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
