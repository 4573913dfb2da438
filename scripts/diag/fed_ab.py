#!/usr/bin/env python3
"""Fed chains (md5_kernels.h md5_desc_hybrid_fed) against the product HYBRID.

1. Chain probe: a lone wave's 1 MiB serial chain with the product step
   (diag kind 32: 5 VALU per step, kLat) vs the fed step (kind 80: 4 VALU,
   the addends read from LDS), 256 and 1024 one-wave workgroups.
2. Digests: fed == product (the product is oracle-checked by the GPU tests)
   on a ragged mixed batch with long chunks at odd lengths, and on the C3
   batch.
3. Timing, interleaved rounds (hipEvent per launch): the bench's C3 batch
   (seed 1000), its 1 MiB chunks alone (the chain floor), and K coalesced
   batches.

   Round 3 adds the exclusive split (md5diag_fed_split_excl): the longest
   groups' pairs (or, as the control, HYBRID's lone chain waves) padded to a
   whole CU's LDS so no XDMA wave of the rest shares their CU.

Prints one JSON object.  usage: fed_ab.py [--rounds R] [--batches K ...]
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
sys.path.insert(0, os.path.join(REPO, "tests"))
from c3_trace_x import DIAG, batch  # noqa: E402
import gen  # noqa: E402
from sproxy_amd import md5 as m  # noqa: E402

vp, u64, u32, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int


def timed(f, rounds):
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return ts


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batches", type=int, nargs="*", default=[2])
    a = ap.parse_args()
    D = ctypes.CDLL(DIAG)
    D.md5diag_run.argtypes = [ci, vp, u64, u32, u64, vp, vp]
    D.md5diag_variant_desc.argtypes = [ci, vp, vp, vp, vp, u64, vp, vp]
    D.md5diag_fed_split.argtypes = [ci, vp, vp, vp, vp, u64, vp, vp]
    D.md5diag_fed_split_excl.argtypes = [ci, u64, vp, vp, vp, vp, u64, vp, vp]
    st = torch.cuda.current_stream().cuda_stream
    res = {}

    # 1. chain probe
    L = 1 << 20
    out = torch.empty((1024 * 64 + 64, 4), dtype=torch.int32, device="cuda")
    probe = {}
    for nw in (256, 1024):
        for kind, name in [(32, "step5_kLat"), (80, "fed_step4_lds")]:
            f = lambda: D.md5diag_run(kind, None, nw, L, 0, out.data_ptr(), st)  # noqa: E731
            assert f() == 0
            torch.cuda.synchronize()
            ms = sorted(timed(f, 3))[1]
            probe[f"w{nw}_{name}"] = {"ms": round(ms, 3), "ns_per_step": round(ms * 1e6 / (L // 64) / 64, 3)}
    res["chain_probe"] = probe
    print(json.dumps({"chain_probe": probe}), flush=True)

    def fed(base, dO, dL, dR, n, dig, v=4, L=0):
        if v >= 200:   # exclusive chain CUs: 200 = fed pairs + XDMA, 201 = HYBRID part + XDMA,
            # 203 = fed pairs + the rest as HYBRID
            return D.md5diag_fed_split_excl(v - 200, L, base.data_ptr(), dO.data_ptr(), dL.data_ptr(),
                                            dR.data_ptr(), n, dig.data_ptr(), st)
        if v >= 100:   # split launches: 100 = fed pairs + XDMA, 101 = HYBRID part + XDMA
            return D.md5diag_fed_split(v - 100, base.data_ptr(), dO.data_ptr(), dL.data_ptr(),
                                       dR.data_ptr(), n, dig.data_ptr(), st)
        return D.md5diag_variant_desc(v, base.data_ptr(), dO.data_ptr(), dL.data_ptr(), dR.data_ptr(), n,
                                      dig.data_ptr(), st)

    # 2. digests on a ragged batch: long chunks (>= 256 KiB: the fed path) at odd lengths
    rng = np.random.default_rng(7)
    lens = np.concatenate([rng.integers(256 << 10, (1 << 20) + 200, 700),
                           rng.integers(0, 70000, 3000), [0, 1, 55, 56, 63, 64, 65]]).astype(np.uint32)
    rng.shuffle(lens)
    offs, total = gen.pack_offsets(lens, align=16)
    buf = torch.from_numpy(gen.xorshift_array(total + 64, seed=11)).cuda()
    dO = torch.tensor(offs, dtype=torch.int64, device="cuda")
    dL = torch.from_numpy(lens.astype(np.int32)).cuda()
    order = m.plan_order(lens)
    dR = torch.from_numpy(order.astype(np.int32)).cuda()
    n = lens.size
    ref = m.digest_desc(buf, dO, dL, dR, variant="hybrid")
    dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    eqs = []
    for v in (4, 100, 101):
        assert fed(buf, dO, dL, dR, n, dig, v) == 0
        torch.cuda.synchronize()
        eqs.append(bool(torch.equal(dig, ref)))
    res["ragged_equal"] = eqs
    print(json.dumps({"ragged_equal": res["ragged_equal"], "chunks": int(n)}), flush=True)
    del buf

    # 3. C3 batch, its 1 MiB chunks alone, coalesced batches
    for K in [1] + list(a.batches):
        big, Lk, O, order, var = batch(K, 1000)
        n = Lk.size
        dO = torch.from_numpy(O).cuda()
        dL = torch.from_numpy(Lk.astype(np.int32)).cuda()
        dR = torch.from_numpy(order.astype(np.int32)).cuda()
        dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
        ref = m.digest_desc(big, dO, dL, dR, variant="hybrid")
        # the longest groups (first chunk of the group, in order, at the batch's maximum)
        firsts = Lk[order[::64]]
        Lmax = int((firsts == firsts.max()).sum())
        eq = []
        for v in (4, 100, 101, 200, 201, 203):
            assert fed(big, dO, dL, dR, n, dig, v, Lmax) == 0
            torch.cuda.synchronize()
            eq.append(bool(torch.equal(dig, ref)))
        legs = {"hybrid": lambda: m.digest_desc(big, dO, dL, dR, out=dig, variant="hybrid"),
                "fed_split_excl": lambda: fed(big, dO, dL, dR, n, dig, 200, Lmax),
                "hybrid_split_excl": lambda: fed(big, dO, dL, dR, n, dig, 201, Lmax),
                "fed_excl_rest_hybrid": lambda: fed(big, dO, dL, dR, n, dig, 203, Lmax),
                "fed_one_launch": lambda: fed(big, dO, dL, dR, n, dig, 4),
                "fed_split": lambda: fed(big, dO, dL, dR, n, dig, 100),
                "hybrid_split": lambda: fed(big, dO, dL, dR, n, dig, 101)}
        if K > 1:
            legs["balanced"] = lambda: m.digest_desc(big, dO, dL, dR, out=dig, variant="balanced")
        ms = {k: [] for k in legs}
        for _ in range(a.rounds):
            for k, f in legs.items():
                ms[k] += timed(f, 1)
        entry = {"chunks": int(n), "payload_gib": round(float(Lk.sum()) / 2**30, 3), "planner": var,
                 "excl_groups": Lmax,
                 "fed_equal_hybrid": eq, "ms": {k: [round(x, 3) for x in v] for k, v in ms.items()}}
        if K == 1:   # the 1 MiB chunks alone: the chain floor
            sel = np.nonzero(Lk == (1 << 20))[0]
            sO = torch.from_numpy(O[sel]).cuda()
            sL = torch.from_numpy(Lk[sel].astype(np.int32)).cuda()
            sR = torch.arange(sel.size, dtype=torch.int32, device="cuda")
            sd = torch.empty((sel.size, 16), dtype=torch.uint8, device="cuda")
            fl = {"hybrid": lambda: m.digest_desc(big, sO, sL, sR, out=sd, variant="hybrid"),
                  "fed_one_launch": lambda: fed(big, sO, sL, sR, sel.size, sd, 4),
                  "fed_split": lambda: fed(big, sO, sL, sR, sel.size, sd, 100),
                  "fed_excl": lambda: fed(big, sO, sL, sR, sel.size, sd, 202)}
            fms = {k: [] for k in fl}
            for _ in range(a.rounds):
                for k, f in fl.items():
                    fms[k] += timed(f, 1)
            entry["long_1mib_alone"] = {"chunks": int(sel.size),
                                        "ms": {k: [round(x, 3) for x in v] for k, v in fms.items()}}
        res[f"K{K}"] = entry
        print(json.dumps({f"K{K}": entry}), flush=True)
        del big
        torch.cuda.empty_cache()
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
