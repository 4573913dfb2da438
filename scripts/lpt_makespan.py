#!/usr/bin/env python3
"""The list-scheduling ceiling of one BALANCED launch (md5_desc_balanced_t)
over K coalesced C3 batches -- bench.py's own lengths (c3_lens, the seeds of
--config c3's coalesced leg or of --config c3q).

BALANCED runs one wave per SIMD (1,024 on MI355X) that takes 64-chunk groups
from a device counter, longest first (md5hip_plan_desc's order).  A group's
lanes run in lockstep, so it costs its longest chunk's compressions,
floor((len + 8) / 64) + 1 (md5.c:221-265 padding).  Simulating that list
schedule gives, per launch:

  mean      total group cost / 1,024 SIMDs   (perfect balance)
  makespan  when the last SIMD finishes      (a 1 MiB chunk is a serial chain
                                              of 16,385 compressions on one lane)
  util      mean / makespan                  -- the share of SIMD-time the
            launch can keep busy, whatever the kernel does inside a group

so a launch's roofline fraction is at most util x (VALU issue share of a lone
wave, 0.85 measured in DESIGN §5.3) x (clock).  Usage:
  lpt_makespan.py [--batches 1 2 3 6] [--seeds coalesced|c3q] [--out FILE]"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import c3_lens, lpt_schedule  # noqa: E402  (numpy only; bench.py imports torch lazily)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batches", type=int, nargs="+", default=[1, 2, 3, 4, 6, 8])
    ap.add_argument("--bytes", type=int, default=16 << 30)
    ap.add_argument("--seeds", choices=["coalesced", "c3q"], default="coalesced",
                    help="coalesced: bench.py c3_coalesced's seeds (1000, 2000+17j); c3q: run_c3q's (3000+31j)")
    ap.add_argument("--out")
    a = ap.parse_args()
    res = {"simds": 1024, "group": 64, "cost": "longest chunk's compressions per 64-chunk group",
           "seeds": a.seeds, "launches": []}
    for k in a.batches:
        if a.seeds == "coalesced":
            lk = [c3_lens(a.bytes, 1000)] + [c3_lens(a.bytes, 2000 + 17 * j) for j in range(1, k)]
        else:
            lk = [c3_lens(a.bytes, 3000 + 31 * j) for j in range(k)]
        lens = np.concatenate(lk)
        s = lpt_schedule(lens)
        longest = int((lens.max() + 8) // 64 + 1)
        r = {"batches": k, "chunks": int(lens.size), **s, "longest_chain": longest,
             "bound": "longest chain" if s["makespan_compressions"] <= longest * 1.001 else "load"}
        res["launches"].append(r)
        print(json.dumps(r))
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
