#!/usr/bin/env python3
"""CRC-32 descriptor batch (crc32hip_desc) on netcache-shaped 16 GiB batches:
chunk_size blocks with 1 in 8 ragged last blocks, lanes longest-first.
The kernel follows CRC32HIP_VARIANT (XPERM16 default -> crc32_desc_xperm16,
else the lane-direct crc32_desc).  Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts", "diag"))
from sproxy_amd import md5 as m  # noqa: E402
from c3_sweep import timeit  # noqa: E402

res = {}
data = torch.empty(16 << 30, dtype=torch.uint8, device="cuda")
m.fill_synthetic(data, seed=0xCD)
for S in (4096, 16384, 65536, 262144):
    n = (16 << 30) // S
    rng = np.random.default_rng(S)
    lens = np.full(n, S, dtype=np.int64)
    tail = rng.integers(0, 8, n) == 0
    lens[tail] = rng.integers(1, S, int(tail.sum()))
    offs = torch.arange(n, dtype=torch.int64, device="cuda") * S
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    order = torch.from_numpy(m.plan_order(lens.astype(np.uint32)).astype(np.int32)).cuda()
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    ms = timeit(lambda: m.crc32_desc(data, offs, d_len, order, out=out))
    res[str(S)] = {"ms": round(ms, 3), "payload_GiBps": round(float(lens.sum()) / (1 << 30) / (ms * 1e-3), 1)}
res["variant"] = m.crc_variant_name(0)
print(json.dumps(res))
