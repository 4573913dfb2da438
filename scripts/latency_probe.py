#!/usr/bin/env python3
"""Per-call latency of the device-input queue (md5hip_queue_create +
md5_batch_submit_device, synchronous, digests left on the device) for
netcache-vector-sized submissions, against the kernel time of the same batch
(md5hip_digest_desc through the planner, hipEvent).  Each library given
(name=path; default: the product library) gets its own queue; calls are
interleaved.  Prints one JSON object: median / p90 microseconds per call.
With --crc the queues hash CRC-32 (md5hip_batcher_set_digest: the netcache
blk_make_crc checksum) and the kernel alone is crc32hip_desc.
usage: latency_probe.py [--iters N] [--crc] [--lib name=path ...]"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

vp, u64, u32, ci = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int


def load(path):
    L = ctypes.CDLL(path, mode=ctypes.RTLD_LOCAL)
    L.md5hip_queue_create.argtypes = [ci, u64, u32, ctypes.POINTER(vp)]
    L.md5_batch_submit_device.argtypes = [vp, vp, vp, u64, vp, ci]
    L.md5hip_batcher_destroy.argtypes = [vp]
    L.md5hip_batcher_set_digest.argtypes = [vp, ci, u32]
    return L


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--lib", nargs="*", default=["product=sproxy_amd/lib/libmd5hip.so"])
    ap.add_argument("--crc", action="store_true")
    a = ap.parse_args()
    dsz = 4 if a.crc else 16
    libs = {}
    for spec in a.lib:
        k, p = spec.split("=", 1)
        L = load(os.path.join(REPO, p))
        h = vp()
        assert L.md5hip_queue_create(0, 0, 0, ctypes.byref(h)) == 0
        if a.crc:
            assert L.md5hip_batcher_set_digest(h, 1, 0) == 0      # MD5HIP_DIGEST_CRC32
        libs[k] = (L, h)
    data = torch.empty(64 << 20, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0x1A7)
    res = {}
    for n, L_ in ((16, 65536), (64, 16384), (256, 16384), (1024, 16384)):
        P = (data.data_ptr() + np.arange(n, dtype=np.uint64) * np.uint64(L_)).astype(np.uint64)
        lens = np.full(n, L_, dtype=np.uint32)
        dig = torch.empty((n, dsz), dtype=torch.uint8, device="cuda")
        ref = None
        for k, (L, h) in libs.items():
            assert L.md5_batch_submit_device(h, P.ctypes.data, lens.ctypes.data, n, dig.data_ptr(), 1) == 0
            torch.cuda.synchronize()
            ref = dig.clone() if ref is None else ref
            assert torch.equal(dig, ref), k
        # kernel alone: the planner's choice on the same chunks
        dO = torch.from_numpy((P - np.uint64(data.data_ptr())).astype(np.int64)).cuda()
        dL = torch.from_numpy(lens.astype(np.int32)).cuda()
        order, var = m.plan_desc(lens)
        dR = torch.from_numpy(order.astype(np.int32)).cuda()
        if a.crc:
            var = "crc32hip_desc"
        ks = []
        for _ in range(20):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            if a.crc:
                m.crc32_desc(data, dO, dL, dR, out=dig.view(torch.int32).view(-1))
            else:
                m.digest_desc(data, dO, dL, dR, out=dig, variant=var)
            e1.record()
            torch.cuda.synchronize()
            ks.append(e0.elapsed_time(e1) * 1e3)
        lat = {k: [] for k in libs}
        for it in range(a.iters + 20):
            for k, (L, h) in libs.items():
                t0 = time.perf_counter()
                rc = L.md5_batch_submit_device(h, P.ctypes.data, lens.ctypes.data, n, dig.data_ptr(), 1)
                t1 = time.perf_counter()
                assert rc == 0
                if it >= 20:
                    lat[k].append((t1 - t0) * 1e6)
        q = lambda v, p: round(float(np.percentile(v, p)), 1)  # noqa: E731
        res[f"{n}x{L_ // 1024}KiB"] = {"kernel_us_median": q(ks, 50), "planner": var,
                                      **{k: {"median_us": q(v, 50), "p90_us": q(v, 90)} for k, v in lat.items()}}
        print(json.dumps({f"{n}x{L_ // 1024}KiB": res[f"{n}x{L_ // 1024}KiB"]}), flush=True)
    for L, h in libs.values():
        L.md5hip_batcher_destroy(h)
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
