#!/usr/bin/env python3
"""fastcrc (F = 128 / 64) on 1,048,576 x 16 KiB blocks: the product kernel
(crc32_fast_pipe) against diagnostic depths -- window groups in flight per
wave (md5diag_crc_fast_pipe: 2 @ 16 waves/CU, 3 @ 12, 4 @ 8, 2 @ 12; and
2 @ 16 with each window's halves loaded as two runs, the pre-round-3 order) --
hipEvent ms per launch over interleaved rounds, results compared.
usage: fastcrc_ab.py [--rounds R] [--F 128 64]"""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

DIAG = os.path.join(REPO, "build", "diag", "libmd5hip_diag.so")
DEPTHS = {2: "d2_16w", 3: "d3_12w", 4: "d4_8w", 13: "d2_12w", 20: "d2_16w_runs"}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--F", type=int, nargs="*", default=[128, 64])
    a = p.parse_args()
    D = ctypes.CDLL(DIAG)
    vp = ctypes.c_void_p
    D.md5diag_crc_fast_pipe.argtypes = [ctypes.c_int, vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint64,
                                        ctypes.c_uint32, vp, vp]
    n, L = 1 << 20, 16384
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xFA)
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    for F in a.F:
        ref = m.crc32_fixed(data, n, L, fastcrc=F)
        outs = {k: torch.empty(n, dtype=torch.int32, device="cuda") for k in DEPTHS}
        run = lambda k: D.md5diag_crc_fast_pipe(k, data.data_ptr(), n, L, L, F, outs[k].data_ptr(), st)  # noqa
        same = {}
        for k in DEPTHS:
            assert run(k) == 0
            torch.cuda.synchronize()
            same[DEPTHS[k]] = bool(torch.equal(outs[k], ref))
        ms = {v: [] for v in DEPTHS.values()}
        ms["product"] = []
        po = torch.empty(n, dtype=torch.int32, device="cuda")
        for _ in range(a.rounds):
            for k in list(DEPTHS) + [0]:
                for _w in range(3):                  # back to back, the last timed
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    if k == 0:
                        m.crc32_fixed(data, n, L, fastcrc=F, out=po)
                    else:
                        run(k)
                    e1.record()
                torch.cuda.synchronize()
                ms["product" if k == 0 else DEPTHS[k]].append(round(e0.elapsed_time(e1), 4))
        res[f"F{F}"] = {"ms": ms, "equal_product": same,
                        "gblocks_s_best": {k: round(n / min(v) / 1e6, 2) for k, v in ms.items()}}
        print(json.dumps({f"F{F}": res[f"F{F}"]}), flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
