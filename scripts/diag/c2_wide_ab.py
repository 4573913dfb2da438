#!/usr/bin/env python3
"""C2 energy per byte: fewer LDS round trips per byte.
md5diag_variant_fixed kinds 70 (2 stages per DMA round, 2 waves/SIMD),
71 (1 stage, LDS padded to 2 waves/SIMD: the occupancy control), 72 (4
stages, 1 wave/SIMD), 73 (1 stage: the product's loop, 5 waves/SIMD) against
the product xdma1nt, on 1,048,576 x 16 KiB: ms per launch sustained (mean of
the last `burst` of 2*burst back-to-back launches), interleaved rounds.
usage: c2_wide_ab.py [--rounds R] [--burst B]"""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

DIAG = os.path.join(REPO, "build", "diag", "libmd5hip_diag.so")
KINDS = {73: "w1_5perSIMD", 70: "w2_2perSIMD", 71: "w1_2perSIMD_pad", 72: "w4_1perSIMD"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--burst", type=int, default=10)
    a = p.parse_args()
    D = ctypes.CDLL(DIAG)
    vp = ctypes.c_void_p
    D.md5diag_variant_fixed.argtypes = [ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                        vp, vp]
    n, L = 1 << 20, 16384
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xC2)
    st = torch.cuda.current_stream().cuda_stream
    ref = m.digest_fixed(data, n, L)
    outs = {k: torch.empty((n, 16), dtype=torch.uint8, device="cuda") for k in KINDS}
    run = lambda k: D.md5diag_variant_fixed(k, data.data_ptr(), n, L, L, outs[k].data_ptr(), st)  # noqa
    same = {}
    for k in KINDS:
        assert run(k) == 0
        torch.cuda.synchronize()
        same[KINDS[k]] = bool(torch.equal(outs[k], ref))
    ms = {v: [] for v in KINDS.values()}
    ms["product_xdma1nt"] = []
    po = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    for _ in range(a.rounds):
        for k in list(KINDS) + [0]:
            f = (lambda: m.digest_fixed(data, n, L, out=po)) if k == 0 else (lambda: run(k))
            for _w in range(a.burst):
                f()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _w in range(a.burst):
                f()
            e1.record()
            torch.cuda.synchronize()
            ms["product_xdma1nt" if k == 0 else KINDS[k]].append(round(e0.elapsed_time(e1) / a.burst, 4))
    res = {"ms": ms, "equal_product": same,
           "gib_s_best": {k: round(n * L / (min(v) * 1e-3) / 2**30, 1) for k, v in ms.items()}}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
