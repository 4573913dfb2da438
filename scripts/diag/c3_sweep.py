#!/usr/bin/env python3
"""netcache chunk_size sweep (BASELINE config 3): for each
chunk size 4 KiB..1 MiB, a device-resident batch of `--batch-gib` GiB
  fixed : every chunk exactly chunk_size (md5hip_digest_fixed)
  ragged: 1 in 8 chunks is an object's last block of random length in
          [1, chunk_size) (blk_io.c:377), descriptor batch, longest-first lanes
and, for the largest sizes, bigger batches: one lane hashes one chunk, so a
batch of N chunks keeps at most N lanes busy and a 1 MiB chunk is 16,385
dependent compressions -- the batch needs enough chunks in flight.
Prints one JSON object."""
import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

GIB = float(1 << 30)


def timeit(f, reps=3, rounds=3):
    s = torch.cuda.current_stream()
    f()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(reps):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1) / reps)
    return sorted(ts)[len(ts) // 2]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--batch-gib", type=int, default=16)
    p.add_argument("--big", default="64,128", help="extra batch sizes (GiB) for 256 KiB..1 MiB")
    a = p.parse_args()
    big = [int(x) for x in a.big.split(",") if x]
    cap = max([a.batch_gib] + big) << 30
    data = torch.empty(cap, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xC35)
    rows = []
    for k in range(9):
        S = 4096 << k
        for gib in [a.batch_gib] + (big if S >= (256 << 10) else []):
            n = (gib << 30) // S
            out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
            ms_fixed = timeit(lambda: m.digest_fixed(data, n, S, out=out))
            row = {"chunk_size": S, "batch_gib": gib, "chunks": n, "fixed_ms": round(ms_fixed, 3),
                   "fixed_GiBps": round(n * S / GIB / (ms_fixed * 1e-3), 1)}
            if gib == a.batch_gib:
                rng = np.random.default_rng(S)
                lens = np.full(n, S, dtype=np.int64)
                tail = rng.integers(0, 8, n) == 0
                lens[tail] = rng.integers(1, S, int(tail.sum()))
                offs = torch.arange(n, dtype=torch.int64, device="cuda") * S
                d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
                order = torch.from_numpy(m.plan_order(lens.astype(np.uint32)).astype(np.int32)).cuda()
                ms_r = timeit(lambda: m.digest_desc(data, offs, d_len, order, out=out))
                row.update({"ragged_ms": round(ms_r, 3),
                            "ragged_GiBps": round(float(lens.sum()) / GIB / (ms_r * 1e-3), 1)})
            rows.append(row)
            print(json.dumps(row), file=sys.stderr, flush=True)
            del out
    print(json.dumps({"sweep": rows}))


if __name__ == "__main__":
    main()
