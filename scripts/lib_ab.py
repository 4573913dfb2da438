#!/usr/bin/env python3
"""In-process A/B of two builds of libmd5hip.so on the same device buffers:
OLD (build/ab/libmd5hip_old.so, the library before a change) against NEW
(sproxy_amd/lib/libmd5hip.so).  Both are loaded with ctypes side by side;
every workload runs both, interleaved, and their outputs are compared.

Workloads:
  c2        md5hip_digest_fixed_variant xdma1nt on 1,048,576 x 16 KiB (bench C2)
  ctx       md5hip_update_ctx on 1,048,576 contexts x 16 KiB (bench --config ctx)
  ragged16  md5hip_digest_desc_variant XDMA, netcache blocks packed at 16 B
  c3k3      BALANCED on 3 coalesced C3 batches (bench --config c3 coalesced leg)
Prints one JSON object (ms per launch, hipEvent, interleaved rounds).
usage: lib_ab.py [--rounds R] [--extra name=path ...]"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from sproxy_amd import md5 as m  # noqa: E402

vp, u64, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int


def load(path):
    L = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    L.md5hip_update_ctx.argtypes = [vp, vp, vp, u64, vp]
    L.md5hip_init_ctx.argtypes = [vp, u64, vp]
    L.md5hip_digest_desc_variant.argtypes = [vp, vp, vp, vp, u64, vp, vp, ci]
    L.md5hip_digest_fixed_variant.argtypes = [vp, u64, ctypes.c_uint32, u64, vp, vp, ci]
    return L


def batch(K, seed0):
    """K C3 batches (bench.py's lengths) in one arena: (arena, lens, offsets,
    longest-first order, planned variant)."""
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


def timed(f):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    rc = f()
    e1.record()
    torch.cuda.synchronize()
    assert rc == 0, rc
    return e0.elapsed_time(e1)


def ab(libs, run, out, rounds):
    """run(lib) -> rc; out() -> tensor to compare; returns ms lists and equality"""
    res = {}
    for name, L in libs.items():
        assert run(L) == 0
        torch.cuda.synchronize()
        res[name] = out().clone()
    eq = all(bool(torch.equal(res["old"], v)) for v in res.values())
    for _ in range(3):                   # clocks settle
        for L in libs.values():
            run(L)
    torch.cuda.synchronize()
    ms = {k: [] for k in libs}
    for _ in range(rounds):
        for k, L in libs.items():
            ms[k].append(round(timed(lambda: run(L)), 4))
    return {"ms": ms, "equal": eq, "best_new_vs_old": round(min(ms["old"]) / min(ms["new"]), 4),
            "median_new_vs_old": round(sorted(ms["old"])[rounds // 2] / sorted(ms["new"])[rounds // 2], 4)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--extra", nargs="*", default=[], help="name=path of more builds to compare")
    ap.add_argument("--old", default="build/ab/libmd5hip_old.so", help="the baseline build")
    ap.add_argument("--only", default="", help="comma list of workloads (c2,ctx,ragged16,c3k3_balanced,c3k6_balanced,c3_hybrid)")
    a = ap.parse_args()
    only = set(a.only.split(",")) if a.only else None
    libs = {"old": load(os.path.join(REPO, a.old))}
    for extra in a.extra:               # name=path, between old and new
        k, v = extra.split("=", 1)
        libs[k] = load(os.path.join(REPO, v))
    libs["new"] = load(os.path.join(REPO, "sproxy_amd", "lib", "libmd5hip.so"))
    st = torch.cuda.current_stream().cuda_stream
    res = {}

    if only is None or "c2" in only:
        c2_ab(libs, st, res, a.rounds)
    # ctx: 1 M contexts x 16 KiB (one update launch; contexts re-initialised per run)
    if only is None or "ctx" in only:
        ctx_ab(libs, st, res, a.rounds)
    if only is None or "ragged16" in only:
        ragged_ab(libs, st, res, a.rounds)
    for K, name, var in ((3, "c3k3_balanced", 5), (6, "c3k6_balanced", 5), (1, "c3_hybrid", 3)):
        if only is None or name in only:
            c3_ab(libs, st, res, a.rounds, K, name, var)
    print(json.dumps(res))


def c2_ab(libs, st, res, rounds):
    """C2: 1,048,576 x 16 KiB fixed-length, md5_fixed_xdma1nt (variant 10)"""
    n, L = 1 << 20, 16384
    data = m.arena_empty(n * L)
    m.fill_synthetic(data, seed=0xC2)
    dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    run = lambda Lb: Lb.md5hip_digest_fixed_variant(data.data_ptr(), n, L, L, dig.data_ptr(), st, 10)  # noqa
    res["c2"] = ab(libs, run, lambda: dig, rounds)
    print(json.dumps({"c2": res["c2"]}), flush=True)
    del data, dig
    torch.cuda.empty_cache()


def ctx_ab(libs, st, res, rounds):
    """1 M contexts x 16 KiB (one update launch; contexts re-initialised per run)"""
    n, L = 1 << 20, 16384
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xC7)
    ctx = torch.zeros((n, 88), dtype=torch.uint8, device="cuda")
    ptrs = torch.arange(n, dtype=torch.int64, device="cuda") * L + data.data_ptr()
    lens = torch.full((n,), L, dtype=torch.int32, device="cuda")

    def run_ctx(Lb):
        rc = Lb.md5hip_init_ctx(ctx.data_ptr(), n, st)
        return rc or Lb.md5hip_update_ctx(ctx.data_ptr(), ptrs.data_ptr(), lens.data_ptr(), n, st)
    res["ctx"] = ab(libs, run_ctx, lambda: ctx, rounds)
    print(json.dumps({"ctx": res["ctx"]}), flush=True)
    del data, ctx, ptrs, lens
    torch.cuda.empty_cache()


def ragged_ab(libs, st, res, rounds):
    """ragged netcache blocks packed at 16 B (descriptor XDMA)"""
    rng = np.random.default_rng(5)
    S, nb = 16384, 983040                       # ~15 GiB
    bl = np.full(nb, S, dtype=np.int64)
    tail = rng.integers(0, 8, nb) == 0
    bl[tail] = rng.integers(1, S, int(tail.sum()))
    offs = np.concatenate([[0], np.cumsum((bl + 15) // 16 * 16)[:-1]]).astype(np.int64)
    arena = m.arena_empty(int(offs[-1] + bl[-1] + 64))
    m.fill_synthetic(arena, seed=0x16)
    order, _ = m.plan_desc(bl.astype(np.uint32))
    dO = torch.from_numpy(offs).cuda()
    dL = torch.from_numpy(bl.astype(np.int32)).cuda()
    dR = torch.from_numpy(order.astype(np.int32)).cuda()
    dig = torch.empty((nb, 16), dtype=torch.uint8, device="cuda")
    run_r = lambda Lb: Lb.md5hip_digest_desc_variant(arena.data_ptr(), dO.data_ptr(), dL.data_ptr(),  # noqa
                                                     dR.data_ptr(), nb, dig.data_ptr(), st, 4)
    res["ragged16"] = ab(libs, run_r, lambda: dig, rounds)
    print(json.dumps({"ragged16": res["ragged16"]}), flush=True)
    del arena, dO, dL, dR, dig
    torch.cuda.empty_cache()


def c3_ab(libs, st, res, rounds, K, name, var):
    """K coalesced C3 batches (bench.py's lengths) launched with `var`
    (5 = BALANCED, the queue's choice for coalesced batches; 3 = HYBRID for one)"""
    big, Lk, O, order, _ = batch(K, 1000)
    nk = Lk.size
    dO = torch.from_numpy(O).cuda()
    dL = torch.from_numpy(Lk.astype(np.int32)).cuda()
    dR = torch.from_numpy(order.astype(np.int32)).cuda()
    dig = torch.empty((nk, 16), dtype=torch.uint8, device="cuda")
    run_b = lambda Lb: Lb.md5hip_digest_desc_variant(big.data_ptr(), dO.data_ptr(), dL.data_ptr(),  # noqa
                                                     dR.data_ptr(), nk, dig.data_ptr(), st, var)
    res[name] = ab(libs, run_b, lambda: dig, rounds)
    res[name]["payload_bytes"] = int(Lk.sum())
    print(json.dumps({name: res[name]}), flush=True)
    del big, dO, dL, dR, dig
    torch.cuda.empty_cache()


if __name__ == "__main__":
    sys.exit(main())
