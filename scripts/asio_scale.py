#!/usr/bin/env python3
"""The netcache checksum call site at the reference's scale, measured with
build/c/asio_scale (tests/c/asio_scale.c: T threads each submitting a vector
of B blocks of L bytes synchronously; latency, CPU per call, every digest
checked against the oracle).

  --matrix threads  VERDICT r03 item 1: 8 / 64 / 256 synchronous callers of
                    64 x 16 KiB on one batcher and on a pool over (0, 0), from
                    pageable memory (host copy into the pinned staging) and
                    from registered pages (zero-copy: the queue's own cost)
  --matrix chunk    VERDICT r03 item 2: netcache's shipped chunk_size 128 KiB
                    (httpd.c:8627) and 1 MiB next to 16 KiB, vectors of 8 and
                    64 blocks, 1 / 8 / 64 callers, through the batcher and on
                    the calling thread (product MD5Init/Update/Final)
  --matrix bigchunk VERDICT r04 item 2: the rest of netcache's chunk_size
                    range (clamped to 4-10,240 KiB, httpd.c:7968): 2, 4 and
                    10 MiB blocks in vectors of 1, 4 and 8, 1 / 8 / 64
                    callers, batcher vs the calling thread
  --matrix fastcrc  netcache's CRC-32 with fastcrc = 128 (and whole-block
                    CRC) at the call site, 64 x 16 KiB vectors from pageable
                    pages, 1 / 8 / 64 callers: this library (host blocks stage
                    only their windows) against the round-5 library before
                    that change (build/abr05/old, via LD_LIBRARY_PATH) and the
                    calling thread
  --matrix watch    VERDICT r04 item 3: the blocked caller's watcher policy
                    (MD5HIP_WATCH spin / tail / block, md5_submit.c
                    watch_launch) at 8 / 64 / 256 callers of 64 x 16 KiB from
                    registered pages, batcher and pool, interleaved rounds

Writes one JSON file (--out) with every run; prints each run as it ends.
usage: asio_scale.py --matrix threads|chunk [--secs 3] [--out FILE]"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(REPO, "build", "c", "asio_scale")


def run(target, threads, blocks, L, secs, mode="pageable", timeout=150, env=None, tag=None, slice_mib=0):
    cmd = [EXE, target, str(threads), str(blocks), str(L), str(secs), mode]
    if slice_mib:
        cmd += [str(slice_mib), "4"]
    t0 = time.time()
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout,
                         env=dict(os.environ, **(env or {})))
    line = out.stdout.strip().splitlines()[-1] if out.stdout.strip() else "{}"
    rec = json.loads(line)
    rec["exit"] = out.returncode
    if tag:
        rec.update(tag)
    rec["run_s"] = round(time.time() - t0, 1)
    if out.returncode != 0:
        rec["stderr"] = out.stderr[-2000:]
    print(json.dumps(rec), flush=True)
    return rec


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--matrix", choices=["threads", "chunk", "bigchunk", "watch", "fastcrc"], required=True)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--policies", default="spin,tail,block", help="--matrix watch: MD5HIP_WATCH values")
    ap.add_argument("--slice-mib", type=int, default=0, help="batcher slice (0 = the library default)")
    ap.add_argument("--secs", type=float, default=3.0)
    ap.add_argument("--sizes-kib", default="16,128,1024", help="--matrix chunk: block sizes in KiB")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    runs = []
    if a.matrix == "threads":
        for mode in ("registered", "pageable"):
            for target in ("batcher", "pool"):
                for T in (8, 64, 256):
                    runs.append(run(target, T, 64, 16384, a.secs, mode))
    elif a.matrix == "watch":
        for r in range(a.rounds):
            for target in ("batcher", "pool"):
                for T in (8, 64, 256):
                    for pol in a.policies.split(","):
                        runs.append(run(target, T, 64, 16384, a.secs, "registered",
                                        env={"MD5HIP_WATCH": pol}, tag={"watch": pol, "round": r}))
    elif a.matrix == "fastcrc":
        old = os.path.join(REPO, "build", "abr05", "old")
        for F in (128, 0):
            for T in (1, 8, 64):
                for lib in ("new", "old"):
                    env = {"ASIO_CRC": str(F)}
                    if lib == "old":
                        env["LD_LIBRARY_PATH"] = old + ":" + os.environ.get("LD_LIBRARY_PATH", "")
                    runs.append(run("batcher", T, 64, 16384, a.secs, env=env, tag={"lib": lib}))
                if F:
                    runs.append(run("host", T, 64, 16384, a.secs, env={"ASIO_CRC": str(F)}, tag={"lib": "host"}))
    elif a.matrix == "bigchunk":
        if a.slice_mib:      # the queue alone, with slices sized for many long chains in flight
            for L in (2 << 20, 10 << 20):
                for B in (4, 8):
                    runs.append(run("batcher", 64, B, L, a.secs, timeout=300, slice_mib=a.slice_mib,
                                    tag={"slice_mib": a.slice_mib}))
        else:
            for L in (2 << 20, 4 << 20, 10 << 20):
                for B in (1, 4, 8):
                    for T in (1, 8, 64):
                        for target in ("batcher", "host"):
                            runs.append(run(target, T, B, L, a.secs, timeout=300))
    else:
        for L in [int(k) << 10 for k in a.sizes_kib.split(",")]:
            for B in (8, 64):
                for T in (1, 8, 64):
                    for target in ("batcher", "host"):
                        runs.append(run(target, T, B, L, a.secs))
    res = {"matrix": a.matrix, "secs": a.secs, "runs": runs,
           "all_digests_equal_oracle": all(r.get("mismatches", 1) == 0 and r.get("exit") == 0 for r in runs)}
    if a.out:
        os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)
    return 0 if res["all_digests_equal_oracle"] else 1


if __name__ == "__main__":
    sys.exit(main())
