#!/usr/bin/env python3
"""Why one c3q launch (6 C3 batches through md5hip_queue) runs ~5 % longer
than the same-size launch coalesced by hand (bench.py --config c3
--c3-legs coalesced --c3-coalesce 6): the same 6-batch layout as bench.py
run_c3q, one BALANCED launch each with

  host     md5hip_plan_desc's order (stable: equal keys in address order)
  device   md5hip_plan_hist + md5hip_order_device (the queue's planner:
           equal keys in wave-arrival order)
  shuffle  longest-first by key, equal keys in random order
  queue    the 6 batches submitted to an md5hip_queue and waited (drained)

  device_sorted  the device order with each key bucket sorted by index
  device_stable  md5hip_order_device_stable (ABI 5, rocPRIM radix sort)
  host_rev       equal keys in descending chunk order
  batch_rr       equal keys round-robin over the batches

interleaved over rounds in a shuffled order with the same 50 ms idle before
each launch, timed with HIP events on the launch stream (queue: wall clock
of submit + wait).  Every order's digests are compared with the
host order's.  usage: order_ab.py [--rounds 5] [--out FILE]"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from bench import c3_lens, c3_offsets  # noqa: E402
from sproxy_amd import _lib, md5 as m  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--batches", type=int, default=6)
    ap.add_argument("--out")
    a = ap.parse_args()
    K = a.batches
    lk = [c3_lens(16 << 30, 3000 + 31 * j) for j in range(K)]
    ok_ = [c3_offsets(x)[0] for x in lk]
    spans = [(c3_offsets(x)[1] + 15) // 16 * 16 for x in lk]
    starts = np.concatenate([[0], np.cumsum(spans)[:-1]]).astype(np.int64)
    big = m.arena_empty(int(sum(spans)))
    m.fill_synthetic(big, seed=0xC3D)
    torch.cuda.synchronize()
    L_all = np.concatenate(lk).astype(np.uint32)
    O_all = np.concatenate([o + st for o, st in zip(ok_, starts)]).astype(np.int64)
    n = L_all.size
    dO = torch.from_numpy(O_all).cuda()
    dL = torch.from_numpy(L_all.view(np.int32)).cuda()
    # host order + the planner's variant
    ord_h, var = m.plan_desc(L_all)
    orders = {"host": torch.from_numpy(ord_h.astype(np.int32)).cuda()}
    # the queue's device order
    lib = _lib.lib()
    keys = (L_all >> 6) + 1
    kmax = int(keys.max())
    hist = np.bincount(keys, minlength=kmax + 1).astype(np.uint32)
    bstart = np.zeros(kmax + 1, np.uint32)
    assert lib.md5hip_plan_hist(hist.ctypes.data, kmax, n, bstart.ctypes.data) >= 0
    d_next = torch.from_numpy(bstart.view(np.int32)).cuda()
    d_ord = torch.empty(n, dtype=torch.int32, device="cuda")
    assert lib.md5hip_order_device(dL.data_ptr(), n, kmax, d_next.data_ptr(), d_ord.data_ptr(),
                                   torch.cuda.current_stream().cuda_stream) == 0
    orders["device"] = d_ord
    # ABI 5: the stable device order (rocPRIM radix sort), what the batcher now uses
    need = lib.md5hip_order_stable_scratch(n, kmax)
    scratch = torch.empty(need, dtype=torch.uint8, device="cuda")
    d_st = torch.empty(n, dtype=torch.int32, device="cuda")
    assert lib.md5hip_order_device_stable(dL.data_ptr(), n, kmax, scratch.data_ptr(), need, d_st.data_ptr(),
                                          torch.cuda.current_stream().cuda_stream) == 0
    orders["device_stable"] = d_st
    # equal keys shuffled
    rng = np.random.default_rng(7)
    perm = rng.permutation(n)
    sh = perm[np.argsort(-keys[perm].astype(np.int64), kind="stable")]
    orders["shuffle"] = torch.from_numpy(sh.astype(np.int32)).cuda()
    # equal keys in DESCENDING chunk order, and equal keys round-robin over
    # the batches (chunk k of batch 0, of batch 1, ...)
    kk = -keys.astype(np.int64)
    idx = np.arange(n, dtype=np.int64)
    orders["host_rev"] = torch.from_numpy(np.lexsort((-idx, kk)).astype(np.int32)).cuda()
    bat = np.concatenate([np.full(x.size, j, np.int64) for j, x in enumerate(lk)])
    rank_in_batch_key = np.zeros(n, np.int64)
    o = np.lexsort((idx, bat, kk))                  # by key, batch, index
    kb = np.stack([kk[o], bat[o]])
    starts_kb = np.flatnonzero(np.r_[True, (kb[:, 1:] != kb[:, :-1]).any(axis=0)])
    run_id = np.repeat(np.arange(starts_kb.size), np.diff(np.r_[starts_kb, n]))
    rank_in_batch_key[o] = np.arange(n) - starts_kb[run_id]
    orders["batch_rr"] = torch.from_numpy(np.lexsort((bat, rank_in_batch_key, kk)).astype(np.int32)).cuda()
    # the device order with each key bucket sorted by chunk index (= host's)
    dv = d_ord.cpu().numpy().view(np.uint32).astype(np.int64)
    ds = dv[np.lexsort((dv, -keys[dv].astype(np.int64)))]
    orders["device_sorted"] = torch.from_numpy(ds.astype(np.int32)).cuda()
    # how far the device order is from the host's: chunks whose position differs
    res_diff = {"device_vs_host_positions_differing": int((dv != ord_h.astype(np.int64)).sum()),
                "device_sorted_equals_host": bool(np.array_equal(ds, ord_h.astype(np.int64))),
                "device_stable_equals_host": bool(np.array_equal(d_st.cpu().numpy().view(np.uint32),
                                                                 ord_h))}
    # the stable sort's own time (the batcher runs it per large slot)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    st = torch.cuda.current_stream()
    e0.record(st)
    for _ in range(10):
        lib.md5hip_order_device_stable(dL.data_ptr(), n, kmax, scratch.data_ptr(), need, d_st.data_ptr(),
                                       st.cuda_stream)
    e1.record(st)
    torch.cuda.synchronize()
    res_diff["device_stable_sort_ms"] = round(e0.elapsed_time(e1) / 10, 4)
    outs = {k: torch.empty((n, 16), dtype=torch.uint8, device="cuda") for k in orders}
    # the queue
    base = big.data_ptr()
    subs = [((base + starts[j] + ok_[j]).astype(np.uint64), lk[j].astype(np.uint32)) for j in range(K)]
    qouts = [torch.empty((x.size, 16), dtype=torch.uint8, device="cuda") for x in lk]
    q = m.Queue(device=0, nslots=4, inflight=1)

    def launch(k):
        m.digest_desc(big, dO, dL, orders[k], out=outs[k], variant=var)

    def queue_step():
        pend = [q.submit_device_async(p, L_, o) for (p, L_), o in zip(subs, qouts)]
        for pn in reversed(pend):
            pn.wait()

    res = {k: [] for k in list(orders) + ["queue"]}
    for k in orders:                       # warm-up
        launch(k)
    queue_step()
    torch.cuda.synchronize()
    s = torch.cuda.current_stream()
    prng = np.random.default_rng(11)
    for r in range(a.rounds):
        for k in [list(orders)[j] for j in prng.permutation(len(orders))]:   # shuffled per round
            time.sleep(0.05)                                                  # same idle before each
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            launch(k)
            e1.record(s)
            torch.cuda.synchronize()
            res[k].append(e0.elapsed_time(e1))
        t0 = time.perf_counter()
        queue_step()
        torch.cuda.synchronize()
        res["queue"].append((time.perf_counter() - t0) * 1e3)
    q.close()
    same = {k: bool(torch.equal(outs[k], outs["host"])) for k in orders}
    qsame = all(torch.equal(qouts[j], outs["host"][int(sum(x.size for x in lk[:j])):
                                                   int(sum(x.size for x in lk[:j + 1]))]) for j in range(K))
    alg = float(L_all.sum()) + 16.0 * n
    out = {"batches": K, "chunks": int(n), "variant": var, "alg_bytes": int(alg),
           "ms": {k: [round(x, 3) for x in v] for k, v in res.items()},
           "median_ms": {k: round(float(np.median(v)), 3) for k, v in res.items()},
           "frac": {k: round(alg / (float(np.median(v)) * 1e-3) / 8e12, 4) for k, v in res.items()},
           "digests_equal_host_order": same, "queue_digests_equal": qsame, **res_diff}
    print(json.dumps(out))
    if a.out:
        json.dump(out, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
