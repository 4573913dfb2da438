#!/usr/bin/env python3
"""Does a lone wave issue faster with two independent MD5 chains per lane?
diag kind 32 (one chain per lane, kLat step) vs kind 81 (two interleaved
chains per lane), 1 MiB per chain, 256 and 1024 one-wave workgroups (one
wave per CU / per SIMD).  ns per step per chain-pair-equivalent: a chain
pair hashes twice the bytes, so 'bytes_per_ns' compares throughput."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
D.md5diag_run.argtypes = [i, vp, u64, u32, u64, vp, vp]


def main():
    L = 1 << 20
    out = torch.empty((1024 * 64, 4), dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for nw in (256, 1024):
        for kind, name, chains in [(32, "one_chain", 1), (81, "two_chains", 2)]:
            f = lambda: D.md5diag_run(kind, None, nw, L, 0, out.data_ptr(), st)  # noqa: E731
            assert f() == 0
            torch.cuda.synchronize()
            ts = []
            for _ in range(5):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[2]
            res[f"w{nw}_{name}"] = {"ms": round(ms, 3), "ns_per_step": round(ms * 1e6 / (L // 64) / 64, 3),
                                    "GB_s": round(nw * 64 * chains * L / ms / 1e6, 1)}
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
