#!/usr/bin/env python3
"""Times every batched-MD5 kernel variant and the diagnostic ceilings
(build/diag/libmd5hip_diag.so) on the C2 workload, interleaved in one process
(cdna_hip_programming.md §5.4 rule 24).  Prints one JSON object.

    python scripts/profile_kernels.py [--rounds R] [--chunks N] [--len L] [--only NAMES]

Also the driver for rocprofv3 passes (scripts/gpu_profile.sh)."""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

DIAG = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
DIAG.md5diag_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--rounds", type=int, default=5)
    p.add_argument("--reps", type=int, default=3)
    p.add_argument("--chunks", type=int, default=1 << 20)
    p.add_argument("--len", type=int, default=16384)
    p.add_argument("--only", default="")
    p.add_argument("--no-rotate", action="store_true",
                   help="keep one case order every round (default: rotate it, so no case always "
                        "follows the same predecessor's clock state)")
    a = p.parse_args()
    n, L = a.chunks, a.len
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=1)
    out = torch.empty((max(n, 8192 * 256), 16), dtype=torch.uint8, device="cuda")
    stream = torch.cuda.current_stream()

    def prod(v):
        return lambda: m.digest_fixed(data, n, L, out=out[:n], variant=v)

    crc_out = torch.empty(n, dtype=torch.int32, device="cuda")

    def crc(v="auto"):
        return lambda: m.crc32_fixed(data, n, L, out=crc_out, variant=v)

    def diag(kind):
        def f():
            rc = DIAG.md5diag_run(kind, data.data_ptr(), n, L, L, out.data_ptr(), stream.cuda_stream)
            assert rc == 0, rc
        return f

    cases = {"direct2": prod("direct2"), "direct4": prod("direct4"), "lds64": prod("lds64"),
             "lds128": prod("lds128"), "compute_only": diag(0), "load_direct2": diag(1),
             "load_direct4": diag(2), "load_lds64": diag(3), "load_lds128": diag(4),
             "stream_read": diag(5), "xpose1": prod("xpose1"), "xpose2": prod("xpose2"),
             "xpose1nt": prod("xpose1nt"), "xdma1nt": prod("xdma1nt"), "xpose2nt": prod("xpose2nt"), "lds128nt": prod("lds128nt"),
             "load_xpose1": diag(6), "load_xpose2": diag(7), "crc32": crc(),
             "load_direct2p": diag(8), "load_direct4p": diag(9), "direct2p": diag(10), "direct4p": diag(11),
             "crc_lane32u": diag(27),
             "x64nt": diag(38), "x64": diag(39), "d64nt": diag(44), "d64": diag(45),
             "x2pairnt": diag(46), "x2pair": diag(47), "dyn5": diag(52), "dyn4": diag(53), "nopeel": diag(54), "plain3": diag(55), "comp_plain3": diag(56), "xdmant": diag(57), "xdma": diag(58), "xdma2w2": diag(59), "xdma2w1": diag(60), "xdma_occ16": diag(61), "xdma_occ12": diag(62),
             "xdma_cp3": diag(63), "xdma_cp18": diag(64), "xdma_cp19": diag(65), "xdma_cp1": diag(66),
             "comp32": diag(40), "comp24": diag(41), "comp20": diag(42), "comp16": diag(43),
             "occ20": diag(34), "occ16": diag(35), "occ12": diag(36), "occ8": diag(37), "crc_shared8": crc("shared8"), "crc_lane32": crc("lane32"), "crc_lane16": crc("lane16"), "crc_xlane16": crc("xlane16"), "crc_xperm16": crc("xperm16"), "crc_xdma16": crc("xdma16"),
             "cp0": diag(20), "cp_sc0": diag(21), "cp_nt": diag(22), "cp_sc0nt": diag(23),
             "cp_sc1": diag(24), "cp_sc1nt": diag(25), "cp_sc0sc1nt": diag(26)}
    if a.only:
        cases = {k: v for k, v in cases.items() if k in a.only.split(",")}
    times = {k: [] for k in cases}
    for f in cases.values():
        f()
    torch.cuda.synchronize()
    names = list(cases)
    for rnd in range(a.rounds):
        order = names if a.no_rotate else names[rnd % len(names):] + names[:rnd % len(names)]
        for k in order:
            f = cases[k]
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(stream)
            for _ in range(a.reps):
                f()
            e1.record(stream)
            torch.cuda.synchronize()
            times[k].append(e0.elapsed_time(e1) / a.reps)
    res = {}
    for k, t in times.items():
        t = sorted(t)
        med = t[len(t) // 2]
        res[k] = {"ms_median": round(med, 4), "ms_min": round(t[0], 4),
                  "payload_GBps": round(n * L / med / 1e6, 1)}
    print(json.dumps({"chunks": n, "len": L, "results": res}))


if __name__ == "__main__":
    main()
