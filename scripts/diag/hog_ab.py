#!/usr/bin/env python3
"""HYBRID on the bench's C3 batch with its waves per SIMD capped by registers
(md5diag_desc_x kinds: 1 = HYBRID as shipped, 163 VGPRs = 3 per SIMD;
11 = 2 per SIMD; 12 = 1 per SIMD, a long chain then owns its SIMD), plus the
product launch.  Digests compared with the product's; hipEvent ms, interleaved.
Prints one JSON object.  usage: hog_ab.py [--rounds R]"""
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

vp = ctypes.c_void_p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    a = ap.parse_args()
    D = ctypes.CDLL(DIAG)
    D.md5diag_desc_x.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, vp]
    big, L, O, order, var = batch(1, 1000)
    n = L.size
    dO, dL = torch.from_numpy(O).cuda(), torch.from_numpy(L.astype(np.int32)).cuda()
    dR = torch.from_numpy(order.astype(np.int32)).cuda()
    st = torch.cuda.current_stream().cuda_stream
    dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    ref = m.digest_desc(big, dO, dL, dR, variant="hybrid")
    legs = {"product_hybrid": lambda: m.digest_desc(big, dO, dL, dR, out=dig, variant="hybrid")}
    for k, name in ((1, "hybrid_3_per_simd"), (11, "hybrid_2_per_simd"), (12, "hybrid_1_per_simd")):
        legs[name] = (lambda k=k: D.md5diag_desc_x(k, big.data_ptr(), dO.data_ptr(), dL.data_ptr(),
                                                   dR.data_ptr(), n, dig.data_ptr(), cus, None, st))
    same = {}
    for k, f in legs.items():
        r = f()
        assert not isinstance(r, int) or r == 0, (k, r)
        torch.cuda.synchronize()
        same[k] = bool(torch.equal(dig, ref))
    ms = {k: [] for k in legs}
    for _ in range(a.rounds):
        for k, f in legs.items():
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            f()
            e1.record()
            torch.cuda.synchronize()
            ms[k].append(round(e0.elapsed_time(e1), 3))
    print(json.dumps({"chunks": int(n), "planner": var, "equal_product": same, "ms": ms}))


if __name__ == "__main__":
    sys.exit(main())
