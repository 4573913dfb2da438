#!/usr/bin/env python3
"""The descriptor kernels' LDS-DMA cache policy: `nt` (the product's XDMA /
HYBRID, as the C2 kernel) against the default policy (md5diag_desc_x kinds
3/4), on batches whose chunks are and are not 128-B line aligned:

  c3        the bench's C3 batch (16 GiB, 4 KiB-1 MiB + ragged tails, packed
            16-B aligned, arena), planner order
  u16k      1,048,576 x 16 KiB as descriptors, line aligned (C2's bytes)
  rag16     16 GiB of 16 KiB netcache blocks, 1 in 8 a ragged last block,
            packed 16-B aligned (most blocks start mid-line)
  rag128    the same blocks packed 128-B aligned

hipEvent ms per launch, interleaved rounds; digests compared across kinds.
usage: desc_policy_ab.py [--rounds R] [--sets c3 u16k rag16 rag128]
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
KINDS = {0: "xdma_nt", 3: "xdma_default", 1: "hybrid_nt", 4: "hybrid_default",
         5: "xdma_16w", 6: "xdma_12w", 7: "xdma_8w",
         8: "xdma_4perSIMD", 9: "xdma_3perSIMD", 10: "xdma_2perSIMD"}


def ragged(total, align, seed):
    rng = np.random.default_rng(seed)
    n = total // 16384
    L = np.full(n, 16384, np.int64)
    tail = rng.random(n) < 0.125
    L[tail] = rng.integers(1, 16384, int(tail.sum()))
    O = np.concatenate([[0], np.cumsum((L + align - 1) // align * align)[:-1]])
    return L, O, int(O[-1] + L[-1])


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=3)
    p.add_argument("--sets", nargs="+", default=["c3", "u16k", "rag16", "rag128"])
    p.add_argument("--kinds", type=int, nargs="*", default=[0, 3, 1, 4])
    p.add_argument("--products", nargs="*", default=[],
                   help="product descriptor variants timed beside the planner's (xdma hybrid balanced)")
    a = p.parse_args()
    D = ctypes.CDLL(DIAG)
    vp = ctypes.c_void_p
    D.md5diag_desc_x.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, vp, ctypes.c_uint32, vp, vp]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    out = {}
    for name in a.sets:
        if name == "c3":
            L = bench.c3_lens(16 << 30, 1000)
            O, total = bench.c3_offsets(L)
        elif name == "u16k":
            L = np.full(1 << 20, 16384, np.int64)
            O, total = np.arange(1 << 20, dtype=np.int64) * 16384, 16 << 30
        else:
            L, O, total = ragged(16 << 30, 16 if name == "rag16" else 128, 77)
        data = m.arena_empty((total + 127) // 128 * 128)
        m.fill_synthetic(data, seed=0xD5)
        order, var = m.plan_desc(L.astype(np.uint32))
        dO, dL = torch.from_numpy(O.astype(np.int64)).cuda(), torch.from_numpy(L.astype(np.int32)).cuda()
        dR = torch.from_numpy(order.astype(np.int32)).cuda()
        n = L.size
        st = torch.cuda.current_stream().cuda_stream
        kinds = {k: KINDS[k] for k in a.kinds}
        digs = {k: torch.empty((n, 16), dtype=torch.uint8, device="cuda") for k in list(kinds) + [0]}
        run = lambda k: D.md5diag_desc_x(k, data.data_ptr(), dO.data_ptr(), dL.data_ptr(),  # noqa
                                         dR.data_ptr(), n, digs[k].data_ptr(), cus, None, st)
        for k in kinds:
            assert run(k) == 0
        torch.cuda.synchronize()
        prods = list(dict.fromkeys([var] + a.products))
        ms = {v: [] for v in kinds.values()}
        for v in prods:
            ms["product_" + v] = []
        pdig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
        for _ in range(a.rounds):
            for k in list(kinds) + prods:
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                if isinstance(k, str):
                    m.digest_desc(data, dO, dL, dR, out=pdig, variant=k)
                else:
                    run(k)
                e1.record()
                torch.cuda.synchronize()
                ms["product_" + k if isinstance(k, str) else kinds[k]].append(round(e0.elapsed_time(e1), 3))
        ref = m.digest_desc(data, dO, dL, dR, variant=var)
        for k in kinds:
            assert run(k) == 0
        torch.cuda.synchronize()
        same = all(torch.equal(digs[k], ref) for k in kinds)
        for v in prods:
            same = same and torch.equal(m.digest_desc(data, dO, dL, dR, variant=v), ref)
        pay = float(L.sum())
        res = {"chunks": int(n), "payload_gib": round(pay / 2**30, 2), "planner": var, "ms": ms,
               "gib_s_best": {k: round(pay / (min(v) * 1e-3) / 2**30, 1) for k, v in ms.items()},
               "digests_equal": same}
        out[name] = res
        print(json.dumps({name: res}), flush=True)
        del data, dO, dL, dR, digs, pdig, ref
        torch.cuda.empty_cache()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
