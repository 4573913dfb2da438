#!/usr/bin/env python3
"""Serial MD5 chain latency vs active lanes per wave (diag kinds 28-33):
one 64-thread workgroup per CU (n = 256) or four per CU (n = 1024), each
lane hashing one 1 MiB chain.  Prints one JSON object (ms and ns per step).
--mix (round 3): the step's instruction mix instead, one wave per CU (a lone
chain): product kLat=false (28) and kLat (32, both 316 VALU per block), the
fed step (80: v_bitop3 v_add3 v_alignbit v_add, addends from LDS), and all
additions as single v_add (84: 6 per step; 85: fed, 5 per step)."""
import ctypes
import json
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
D = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
vp, u64, u32, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_int
D.md5diag_run.argtypes = [i, vp, u64, u32, u64, vp, vp]


def main():
    mix = "--mix" in sys.argv
    L = 1 << 20
    out = torch.empty((4096 * 64, 4), dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream().cuda_stream
    res = {}
    kinds = ([(28, "product_step"), (32, "product_step_klat"), (80, "fed_add3"), (84, "single_adds"),
              (85, "fed_single_adds")] if mix else
             [(28, "act64"), (29, "act32"), (30, "act16"), (31, "act1"), (32, "act64_lat"), (33, "act32_lat")])
    for nw in ((256,) if mix else (256, 1024)):
        for kind, name in kinds:
            f = lambda: D.md5diag_run(kind, None, nw, L, 0, out.data_ptr(), st)  # noqa: E731
            assert f() == 0
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f()
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1))
            ms = sorted(ts)[1]
            res[f"w{nw}_{name}"] = {"ms": round(ms, 3), "ns_per_step": round(ms * 1e6 / (L // 64) / 64, 3)}
    print(json.dumps(res))


if __name__ == "__main__":
    sys.exit(main())
