#!/usr/bin/env python3
"""PROBE: one wave per SIMD hashing C interleaved MD5 chains per lane
(scripts/probes/chain_ilp.hip), C = 1, 2, 3, and C = 1 at 2 waves per SIMD
for contrast.  ns per compression per chain (hipEvent, median of 9): equal
per-chain time at C = 2 means the chains do not overlap (a lone wave already
issues at the SIMD's rate); lower means the lone wave leaves issue slots
that a second chain fills.
usage: chain_ilp.py --build | chain_ilp.py [--out FILE]"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(REPO, "scripts", "probes", "chain_ilp.hip")
SO = os.path.join(REPO, "build", "probes", "chain_ilp.so")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.build:
        os.makedirs(os.path.dirname(SO), exist_ok=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-shared", "-fPIC",
                        SRC, "-o", SO], check=True)
        return
    import torch
    P = ctypes.CDLL(SO)
    P.chain_ilp.argtypes = [ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p,
                            ctypes.c_void_p]
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    out = torch.empty(cus * 4 * 256 * 4, dtype=torch.int32, device="cuda")
    iters = 2000
    res = {}
    for name, C, wpc, lds in (("c1_1wps", 1, 1, 96 << 10), ("c2_1wps", 2, 1, 96 << 10),
                              ("c3_1wps", 3, 1, 96 << 10), ("c1_2wps", 1, 2, 40 << 10)):
        st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        run = lambda: P.chain_ilp(C, iters, cus * wpc, lds, out.data_ptr(), st)  # noqa: E731
        for _ in range(3):
            assert run() == 0
        torch.cuda.synchronize()
        t = []
        for _ in range(9):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            run()
            e1.record()
            e1.synchronize()
            t.append(e0.elapsed_time(e1))
        t.sort()
        ms = t[4]
        per = ms * 1e6 / (iters * C * wpc)        # ns per compression per chain per SIMD slot
        res[name] = {"ms": round(ms, 4), "chains_per_lane": C, "waves_per_simd": wpc,
                     "ns_per_compression_per_chain": round(ms * 1e6 / iters / C, 2),
                     "ns_per_compression_simd": round(per, 3)}
        print(name, json.dumps(res[name]), flush=True)
    rec = {"probe": "chain_ilp", "iters": iters, "cus": cus, "results": res}
    print(json.dumps(rec))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        open(a.out, "w").write(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    main()
