#!/usr/bin/env python3
"""HYBRID's lane-direct wave budget (MD5HIP_DESC_NLONG, read per launch) on
chain-bound netcache batches: 16 GiB of ragged 512 KiB / 1 MiB blocks and the
C3 mix, in a batch arena, nlong = one or two waves per CU, interleaved.
Prints one JSON object."""
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts", "diag"))
from sproxy_amd import md5 as m  # noqa: E402
from desc_xdma_ab import time_once  # noqa: E402


def main():
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    coal = "--coalesced" in sys.argv
    data = m.arena_empty((52 if coal else 16) << 30)
    m.fill_synthetic(data, seed=0x4E4C)
    res = {"cus": cus}
    shapes = {}
    for S in (() if coal else (262144, 524288, 1048576)):
        n = (16 << 30) // S
        rng = np.random.default_rng(S)
        lens = np.full(n, S, dtype=np.int64)
        tail = rng.integers(0, 8, n) == 0
        lens[tail] = rng.integers(1, S, int(tail.sum()))
        shapes[f"ragged_{S}"] = (lens, np.arange(n, dtype=np.int64) * S)
    def c3(seed):
        rng = np.random.default_rng(seed)
        lens, tot = [], 0
        while tot < (16 << 30) - (2 << 20):
            c = 4096 << int(rng.integers(0, 9))
            if rng.integers(0, 8) == 0:
                c = int(rng.integers(1, c))
            lens.append(c)
            tot += c
        return np.array(lens, dtype=np.int64)
    lens = c3(1000) if not coal else np.concatenate([c3(1000), c3(2017), c3(2034)])
    shapes["c3x3" if coal else "c3"] = (lens, np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]]))
    for name, (lens, offs) in shapes.items():
        order, v = m.plan_desc(lens.astype(np.uint32))
        d_off = torch.from_numpy(offs).cuda()
        d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
        d_ord = torch.from_numpy(order.astype(np.int32)).cuda()
        out = torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda")
        ts = {}
        for r in range(4):
            for k in ("xdma", "h1", "h2", "h4"):
                if k == "xdma":
                    f = lambda: m.digest_desc(data, d_off, d_len, d_ord, out=out, variant="xdma")  # noqa: E731
                else:
                    os.environ["MD5HIP_DESC_NLONG"] = str(cus * int(k[1]))
                    f = lambda: m.digest_desc(data, d_off, d_len, d_ord, out=out, variant="hybrid")  # noqa: E731
                f()
                ts.setdefault(k, []).append(time_once(f, 5))
        os.environ.pop("MD5HIP_DESC_NLONG", None)
        res[name] = {"plan": v, "ms": {k: round(float(np.median(x)), 4) for k, x in ts.items()}}
        print(json.dumps({name: res[name]}), file=sys.stderr, flush=True)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
