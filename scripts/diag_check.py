#!/usr/bin/env python3
"""Bit-exact check of diagnostic MD5 kernels (build/diag) against the product
kernel on the C2 shape plus a ragged batch:  python scripts/diag_check.py KIND..."""
import ctypes
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
    kinds = [int(k) for k in sys.argv[1:]]
    s = torch.cuda.current_stream()
    bad = 0
    for n, L, stride in [(1 << 20, 16384, 16384), (1000, 4160, 4160), (77, 16384 + 64, 20480), (3, 64, 64), (130, 0, 64)]:
        data = torch.empty(max(n * stride, 1), dtype=torch.uint8, device="cuda")
        m.fill_synthetic(data, seed=7)
        ref = m.digest_fixed(data, n, L, stride=stride, variant="direct2")
        for k in kinds:
            out = torch.zeros((n, 16), dtype=torch.uint8, device="cuda")
            rc = DIAG.md5diag_run(k, data.data_ptr(), n, L, stride, out.data_ptr(), s.cuda_stream)
            torch.cuda.synchronize()
            ok = rc == 0 and torch.equal(out, ref)
            bad += not ok
            print(f"kind {k} n={n} len={L} stride={stride}: {'ok' if ok else 'MISMATCH rc=%d' % rc}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
