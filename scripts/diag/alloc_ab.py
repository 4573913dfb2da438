#!/usr/bin/env python3
"""Does the memory type of the C2 batch change the product kernel's rate?
The 16 GiB C2 batch (1,048,576 x 16 KiB) is allocated with hipMalloc and with
hipExtMallocWithFlags(fine-grained / uncached / contiguous), filled with the
same seed, and md5hip_digest_fixed (the product, xdma1nt) is launched 25 times
untimed (past the power controller's ramp) and 20 times timed
with HIP events, in interleaved rounds.  The memory path is ~55 % of the
kernel's power at the cap, so a memory type whose reads cost
less energy would show up as a shorter launch.  Digests must equal the
hipMalloc run's.  Prints one JSON object.
usage: alloc_ab.py [--rounds 2] [--chunks 1048576]"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

FLAGS = {"hipMalloc": None, "finegrained": 0x1, "uncached": 0x3, "contiguous": 0x4}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--chunks", type=int, default=1 << 20)
    ap.add_argument("--variants", default=",".join(FLAGS))
    a = ap.parse_args()
    import torch
    from sproxy_amd import md5 as m
    from sproxy_amd._lib import lib
    L = lib()
    hip = ctypes.CDLL("libamdhip64.so")
    hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    hip.hipMalloc.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t]
    hip.hipFree.argtypes = [ctypes.c_void_p]
    n, clen = a.chunks, 16384
    nbytes = n * clen
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    dig = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    ref = None
    out = {"chunks": n, "chunk_bytes": clen, "warm_launches": 25, "timed_launches": 20, "rounds": []}
    for r in range(a.rounds):
        row = {}
        for name in a.variants.split(","):
            p = ctypes.c_void_p()
            flag = FLAGS[name]
            rc = hip.hipMalloc(ctypes.byref(p), nbytes) if flag is None else \
                hip.hipExtMallocWithFlags(ctypes.byref(p), nbytes, flag)
            if rc != 0:
                row[name] = {"alloc_error": rc}
                continue
            try:
                with torch.cuda.stream(stream):
                    rc = L.md5hip_fill_synthetic(p, nbytes, 0x9E3779B97F4A7C15, sp)
                    assert rc == 0, rc
                    for _ in range(25):
                        rc = L.md5hip_digest_fixed(p, n, clen, clen, ctypes.c_void_p(dig.data_ptr()), sp)
                        assert rc == 0, rc
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(21)]
                    ev[0].record(stream)
                    for k in range(20):
                        L.md5hip_digest_fixed(p, n, clen, clen, ctypes.c_void_p(dig.data_ptr()), sp)
                        ev[k + 1].record(stream)
                stream.synchronize()
                ms = [ev[k].elapsed_time(ev[k + 1]) for k in range(20)]
                d = dig.cpu()
                if ref is None:
                    ref = d
                mean = sum(ms) / len(ms)
                row[name] = {"mean_ms": round(mean, 4), "min_ms": round(min(ms), 4), "max_ms": round(max(ms), 4),
                             "gib_s": round(nbytes / 2**30 / (mean / 1e3), 1),
                             "digests_equal": bool(torch.equal(d, ref))}
            finally:
                torch.cuda.synchronize()
                hip.hipFree(p)
            print(f"round {r} {name} {row[name]}", file=sys.stderr, flush=True)
        out["rounds"].append(row)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
