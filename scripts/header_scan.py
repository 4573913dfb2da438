#!/usr/bin/env python3
"""SURVEY §8f row 3, measured: dm_verify_header over a volume scan's headers.

When netcache loads a volume it verifies every cached object's header
(dm_verify_header, diskcache.c:3660-3690: CRC-32 over header_size bytes with
crc, disk_header_size and flag read as zero).  This times that check for a
batch of in-memory headers three ways:

  gpu        md5hip_batch_verify_headers through a batcher (host gather into
             pinned staging -> H2D -> CRC-32 kernel -> D2H), headers in
             ordinary host memory as the scan leaves them;
  host       the library's own nc_header_verify per header (one thread, called
             from Python through ctypes, so ~1 us per call of overhead);
  reference  the reference crc32.c (oracle/_ref/crc32_cpu_bench, compiled in
             place) over the same byte volume at the mean header size, 1 thread
             and the box's 16-core share: the CPU baseline.

Header shape (netcache.h:763-792): ~1.5 KiB of fixed part and vstrings, then
the block bitmap (align8(blocks/8)) and the per-block CRC array
(align8(blocks*4), NC_CANNED_CRC_SIZE), for objects log-uniform in
16 KiB .. 4 GiB at chunk_size 64 KiB.  2 % of the headers are corrupted; all
three paths must agree on which (the gpu and host ok arrays are compared).

    python scripts/header_scan.py [--n 100000] [--reps 5]  -> one JSON line
"""
import argparse
import ctypes
import json
import os
import struct
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402
from sproxy_amd import nc_digest as nd  # noqa: E402
from sproxy_amd._lib import lib  # noqa: E402


def build_headers(n, seed):
    rng = np.random.default_rng(seed)
    obj = np.exp(rng.uniform(np.log(16 << 10), np.log(4 << 30), n))
    blocks = np.ceil(obj / (64 << 10)).astype(np.int64)
    fixed = 1024 + rng.integers(0, 1024, n)               # fixed part + vstrings
    size = fixed + (blocks + 63) // 64 * 8 + (blocks * 4 + 7) // 8 * 8
    offs = np.concatenate([[0], np.cumsum((size + 7) // 8 * 8)[:-1]])
    total = int(offs[-1] + size[-1])
    buf = np.frombuffer(rng.bytes(total + 8), np.uint8).copy()
    base = buf.ctypes.data
    L = lib()
    for i in range(n):
        o = int(offs[i])
        buf[o:o + 20] = np.frombuffer(struct.pack("<IiiII", nd.NC_MAGIC_V30, 0, int(size[i]),
                                                  0, 0), np.uint8)
        if L.nc_header_seal(base + o) != 0:
            raise RuntimeError("nc_header_seal")
        buf[o + 4:o + 8] = np.frombuffer(struct.pack("<i", int(size[i]) // 2), np.uint8)
    want = np.ones(n, bool)
    bad = rng.choice(n, max(1, n // 50), replace=False)
    for i in bad:
        buf[int(offs[i]) + int(rng.integers(20, int(size[i])))] ^= 0x10
        want[i] = False
    return buf, offs, size, want


def cpu_reference(mean_len, total_bytes, threads):
    exe = os.path.join(REPO, "oracle", "_ref", "crc32_cpu_bench")
    kind = "reference"
    if not os.path.exists(exe):
        exe, kind = os.path.join(REPO, "oracle", "_build", "crc32_cpu_bench_port"), "port"
    nn = max(threads, int(total_bytes // mean_len))
    out = subprocess.run([exe, str(nn), str(int(mean_len)), "5", str(threads)], capture_output=True,
                         text=True, timeout=600, check=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    return {"gib_s": round(r["gib_s"], 3), "threads": threads, "kind": kind,
            "headers_per_s": round(r["gib_s"] * (1 << 30) / mean_len, 1)}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--n", type=int, default=100000)
    p.add_argument("--reps", type=int, default=5)
    p.add_argument("--slice-mib", type=int, default=0, help="batcher slice (0 = library default)")
    a = p.parse_args()
    t0 = time.perf_counter()
    buf, offs, size, want = build_headers(a.n, 11)
    build_s = time.perf_counter() - t0
    ptrs = (buf.ctypes.data + offs).astype(np.uint64)
    ok = np.empty(a.n, np.uint8)
    L = lib()
    nbytes = float(size.sum())
    res = {"workload": "volume-scan header verify (dm_verify_header, diskcache.c:3660-3690)",
           "headers": a.n, "bytes": int(nbytes), "mean_header_bytes": round(nbytes / a.n, 1),
           "max_header_bytes": int(size.max()), "corrupted": int((~want).sum()),
           "build_s": round(build_s, 2)}

    # host product path (nc_header_verify per header), parity reference for the gpu path
    t0 = time.perf_counter()
    host_ok = np.array([L.nc_header_verify(int(q)) == 1 for q in ptrs])
    host_s = time.perf_counter() - t0
    assert np.array_equal(host_ok, want), "host nc_header_verify disagrees with the corruption set"
    res["host"] = {"s": round(host_s, 4), "headers_per_s": round(a.n / host_s, 1),
                   "gib_s": round(nbytes / host_s / (1 << 30), 3), "threads": 1,
                   "note": "libmd5hip nc_header_verify via ctypes (includes ~1 us/call Python overhead)"}

    with m.Batcher(device=0, slice_bytes=a.slice_mib << 20, nslots=0) as b:
        ts = []
        for r in range(a.reps + 2):
            ok[:] = 2
            t0 = time.perf_counter()
            rc = L.md5hip_batch_verify_headers(b._h, ptrs.ctypes.data, a.n, ok.ctypes.data)
            dt = time.perf_counter() - t0
            if rc < 0:
                raise RuntimeError(f"md5hip_batch_verify_headers = {rc}")
            assert rc == int((~want).sum()) and np.array_equal(ok.astype(bool), want), \
                "gpu header verify disagrees with nc_header_verify"
            if r >= 2:
                ts.append(dt)
        g = float(np.median(ts))
    res["gpu"] = {"s_median": round(g, 4), "headers_per_s": round(a.n / g, 1),
                  "gib_s": round(nbytes / g / (1 << 30), 3), "reps": a.reps,
                  "path": "host gather -> pinned staging -> H2D -> crc32 desc kernel -> D2H",
                  "parity": "ok[] identical to nc_header_verify, mismatch count exact"}
    mean = nbytes / a.n
    res["cpu_baseline"] = cpu_reference(mean, min(nbytes, 2 << 30), 1)
    res["cpu_baseline_all_cores"] = cpu_reference(mean, min(nbytes, 2 << 30), 16)
    res["gpu_vs_cpu_1core"] = round(res["gpu"]["gib_s"] / res["cpu_baseline"]["gib_s"], 2)
    res["gpu_vs_cpu_16core"] = round(res["gpu"]["gib_s"] / res["cpu_baseline_all_cores"]["gib_s"], 2)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
