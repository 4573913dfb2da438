#!/usr/bin/env python3
"""K coalesced C3 batches (c3_trace_x.py's shape) hashed R times by one
descriptor variant -- a short program for rocprofv3 PMC passes on the
BALANCED kernel (clock, VALU busy, waits).  usage: c3_balanced_pmc.py [K] [variant] [R]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts", "diag"))
from c3_trace_x import batch  # noqa: E402
from sproxy_amd import md5 as m  # noqa: E402

K = int(sys.argv[1]) if len(sys.argv) > 1 else 5
var = sys.argv[2] if len(sys.argv) > 2 else "balanced"
R = int(sys.argv[3]) if len(sys.argv) > 3 else 3
big, L, O, order, _ = batch(K, 3000)
dO, dL = torch.from_numpy(O).cuda(), torch.from_numpy(L.astype(np.int32)).cuda()
dR = torch.from_numpy(order.astype(np.int32)).cuda()
out = torch.empty((L.size, 16), dtype=torch.uint8, device="cuda")
for _ in range(R):
    m.digest_desc(big, dO, dL, dR, out=out, variant=var)
torch.cuda.synchronize()
print("ok", K, var, R)
