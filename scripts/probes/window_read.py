#!/usr/bin/env python3
"""PROBE: the ceiling fastcrc's access pattern leaves it (VERDICT r04 item
6).  scripts/probes/window_read.hip reads blk_make_crc's two F-byte windows
per 16 KiB block (blk_io.c:408-424) with no CRC arithmetic; its rate beside
crc32_fast_pipe's (the product kernel, md5hip crc32hip_fixed) at 1 M / 4 M /
8 M blocks per launch says how much of the gap to 8 TB/s is the pattern.
Algorithmic bytes per block: 2F read + 4 written.  hipEvent timing, median
of 15 launches after 5 warm-up ones.
usage: window_read.py --build            (here, on the CPU: hipcc)
       window_read.py [--out FILE]       (on the GPU box)"""
import argparse
import ctypes
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(REPO, "scripts", "probes", "window_read.hip")
SO = os.path.join(REPO, "build", "probes", "window_read.so")
sys.path.insert(0, REPO)


def build():
    os.makedirs(os.path.dirname(SO), exist_ok=True)
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-shared", "-fPIC", SRC, "-o", SO],
                   check=True)


def med_ms(fn, torch):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    t = []
    for _ in range(15):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        e1.synchronize()
        t.append(e0.elapsed_time(e1))
    t.sort()
    return t[len(t) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--build", action="store_true")
    ap.add_argument("--out")
    a = ap.parse_args()
    if a.build:
        build()
        return
    import torch
    from sproxy_amd import md5 as m
    W = ctypes.CDLL(SO)
    W.window_read.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                              ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    L = 16384
    res = {}
    nmax = 8 << 20
    buf = m.arena_empty(nmax * L)                           # 128 GiB
    m.fill_synthetic(buf, seed=11)
    out = torch.empty(nmax, dtype=torch.int32, device="cuda")
    for n in (1 << 20, 4 << 20, 8 << 20):
        for F in (128,):
            alg = n * (2 * F + 4)
            row = {}
            for nt in (0, 1):
                ms = med_ms(lambda: W.window_read(buf.data_ptr(), n, L, L, F, nt, out.data_ptr(),
                                                  ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)),
                            torch)
                row[f"read_only_nt{nt}"] = {"ms": round(ms, 4), "tb_s": round(alg / ms / 1e9, 3),
                                            "frac_of_8tbs": round(alg / ms / 1e9 / 8.0, 4)}
            ms = med_ms(lambda: m.crc32_fixed(buf, n, L, L, fastcrc=F, out=out), torch)
            row["crc32_fast_pipe"] = {"ms": round(ms, 4), "tb_s": round(alg / ms / 1e9, 3),
                                      "frac_of_8tbs": round(alg / ms / 1e9 / 8.0, 4),
                                      "g_blocks_s": round(n / ms / 1e6, 2)}
            res[f"{n}_f{F}"] = row
            print(n, F, json.dumps(row), flush=True)
    rec = {"probe": "window_read", "block_bytes": L, "alg_bytes_per_block": "2F + 4", "results": res}
    print(json.dumps(rec))
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        open(a.out, "w").write(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    main()
