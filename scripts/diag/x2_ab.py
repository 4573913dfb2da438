#!/usr/bin/env python3
"""Descriptor XDMA with two LDS-DMA images per wave (md5diag_desc_x2 kind 0)
vs one image at the same 16 KiB LDS per wave (kind 1) vs the product XDMA
(8 KiB, variant 4), on netcache-shaped ragged batches: 16 KiB blocks with 1-in-8
ragged tails, packed at 16 B and at 128 B, and uniform 16 KiB line-aligned.
Digests compared with the product; hipEvent ms, interleaved rounds.
usage: x2_ab.py [--rounds R]"""
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

vp = ctypes.c_void_p


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=7)
    a = ap.parse_args()
    D = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
    D.md5diag_desc_x2.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, vp, vp]
    st = torch.cuda.current_stream().cuda_stream
    rng = np.random.default_rng(5)
    S, nb = 16384, 983040
    res = {}
    for name, align, ragged in (("ragged_16B", 16, True), ("ragged_128B", 128, True), ("uniform_16k", 128, False)):
        bl = np.full(nb, S, dtype=np.int64)
        if ragged:
            tail = rng.integers(0, 8, nb) == 0
            bl[tail] = rng.integers(1, S, int(tail.sum()))
        offs = np.concatenate([[0], np.cumsum((bl + align - 1) // align * align)[:-1]]).astype(np.int64)
        arena = m.arena_empty(int(offs[-1] + bl[-1] + 64))
        m.fill_synthetic(arena, seed=0x16)
        order, _ = m.plan_desc(bl.astype(np.uint32))
        dO = torch.from_numpy(offs).cuda()
        dL = torch.from_numpy(bl.astype(np.int32)).cuda()
        dR = torch.from_numpy(order.astype(np.int32)).cuda()
        dig = torch.empty((nb, 16), dtype=torch.uint8, device="cuda")
        ref = m.digest_desc(arena, dO, dL, dR, variant="xdma").clone()
        legs = {"product_xdma": lambda: m.digest_desc(arena, dO, dL, dR, out=dig, variant="xdma"),
                "x2_two_images": lambda: D.md5diag_desc_x2(0, arena.data_ptr(), dO.data_ptr(), dL.data_ptr(),
                                                           dR.data_ptr(), nb, dig.data_ptr(), st),
                "x2_one_image_16k": lambda: D.md5diag_desc_x2(1, arena.data_ptr(), dO.data_ptr(), dL.data_ptr(),
                                                              dR.data_ptr(), nb, dig.data_ptr(), st)}
        same = {}
        for k, f in legs.items():
            r = f()
            assert not isinstance(r, int) or r == 0, (k, r)
            torch.cuda.synchronize()
            same[k] = bool(torch.equal(dig, ref))
        for _ in range(3):
            for f in legs.values():
                f()
        torch.cuda.synchronize()
        ms = {k: [] for k in legs}
        for _ in range(a.rounds):
            for k, f in legs.items():
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                torch.cuda.synchronize()
                ms[k].append(round(e0.elapsed_time(e1), 4))
        res[name] = {"payload_gib": round(float(bl.sum()) / 2**30, 3), "equal": same, "ms": ms}
        print(json.dumps({name: res[name]}), flush=True)
        del arena, dO, dL, dR, dig, ref
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
