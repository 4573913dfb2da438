#!/usr/bin/env python3
"""Does the DRAM locality of the C2 access pattern change the clock the board
holds?  The memory path is the larger share of the kernel's energy (DESIGN.md
§5.1), so a pattern that opens fewer DRAM rows per byte would raise the clock
at the power cap.  The product body with its chunk -> wave mapping changed
(diag kinds 91-95, md5_diag.hip diag_xdma_map; 90 = the product mapping with
stamps), on 1,048,576 x 16 KiB: sustained ms per launch (hipEvent, 10 launches
after 10) and the median in-kernel clock, interleaved rounds; every variant's
digests equal the product's.
usage: locality_probe.py [--rounds R]"""
import argparse
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402

DIAG = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
DIAG.md5diag_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                             ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p]
KINDS = {"product_stamped": (90, 4), "groups_permuted": (91, 2), "lane_stride4": (92, 2),
         "lane_stride16": (93, 2), "lane_stride64": (94, 2), "stride16_permuted": (95, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    a = ap.parse_args()
    n, L = 1 << 20, 16384
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0x5EED0000)
    waves = n // 64
    out = torch.zeros(n * 16 + waves * 32, dtype=torch.uint8, device="cuda")
    ref = m.digest_fixed(data, n, L)
    s = torch.cuda.current_stream()
    res = {k: {"ms": [], "ghz": []} for k in ["product"] + list(KINDS)}
    eq = {}

    def launch(k):
        if k == "product":
            m.digest_fixed(data, n, L, out=out[:n * 16].view(n, 16))
        else:
            assert DIAG.md5diag_run(KINDS[k][0], data.data_ptr(), n, L, L, out.data_ptr(), s.cuda_stream) == 0

    for k in KINDS:
        out.zero_()
        launch(k)
        torch.cuda.synchronize()
        eq[k] = bool(torch.equal(out[:n * 16].view(n, 16), ref))
    for _ in range(a.rounds):
        for k in res:
            for _ in range(10):
                launch(k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            for _ in range(10):
                launch(k)
            e1.record(s)
            torch.cuda.synchronize()
            res[k]["ms"].append(round(e0.elapsed_time(e1) / 10, 4))
            if k != "product":
                words = KINDS[k][1]
                clk = out[n * 16:n * 16 + waves * 8 * words].view(torch.int64).view(waves, words).cpu().double()
                res[k]["ghz"].append(round((clk[:, 0] / clk[:, 1]).median().item() * 0.1, 3))
    print(json.dumps({"what": __doc__.split("\n")[0], "equal_product": eq, "result": res}))


if __name__ == "__main__":
    main()
