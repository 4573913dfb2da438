#!/usr/bin/env python3
"""Per-wave placement + timing of the descriptor kernel on the C3 batch."""
import ctypes
import json
import os
import sys
from collections import Counter, defaultdict

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "scripts", "diag"))
from sproxy_amd import md5 as m  # noqa: E402
from c3_ab import c3_batch  # noqa: E402

D = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"))
vp, u64, i = ctypes.c_void_p, ctypes.c_uint64, ctypes.c_int
D.md5diag_desc_trace.argtypes = [i, vp, vp, vp, vp, u64, vp, vp, vp]

lens = c3_batch(16 << 30)
offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
total = int(offs[-1] + lens[-1] + 16)
data = torch.empty((total + 15) // 16 * 16, dtype=torch.uint8, device="cuda")
m.fill_synthetic(data, seed=3)
order_np = m.plan_order(lens.astype(np.uint32))
order = torch.from_numpy(order_np.astype(np.int32)).cuda()
d_off = torch.from_numpy(offs).cuda()
d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
out = torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda")
nw = (lens.size + 63) // 64
rec = torch.zeros(4 * nw, dtype=torch.int64, device="cuda")
st = torch.cuda.current_stream().cuda_stream
res = {}
for tpb in (64,):
    for _ in range(2):
        assert D.md5diag_desc_trace(tpb, data.data_ptr(), d_off.data_ptr(), d_len.data_ptr(),
                                    order.data_ptr(), lens.size, out.data_ptr(), rec.data_ptr(), st) == 0
        torch.cuda.synchronize()
    r = rec.view(-1, 4).cpu().numpy()
    hw, xcc, t0, t1 = r[:, 0], r[:, 1], r[:, 2], r[:, 3]
    t00 = t0.min()
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    key = [(int(x), int(s_), int(h), int(c)) for x, s_, h, c in zip(xcc & 15, se, sh, cu)]
    wave_len = [int(lens[order_np[w * 64]]) for w in range(nw)]
    per_cu = Counter(key[w] for w in range(nw) if wave_len[w] >= (1 << 20))
    per_simd = Counter((key[w], int(simd[w])) for w in range(nw) if wave_len[w] >= (1 << 20))
    dur = (t1 - t0) / 100.0   # us
    end = (t1 - t00) / 100.0
    start = (t0 - t00) / 100.0
    by_len = defaultdict(list)
    for w in range(nw):
        by_len[wave_len[w]].append((start[w], dur[w], end[w]))
    summary = {str(k): {"waves": len(v), "start_med_us": round(float(np.median([x[0] for x in v])), 1),
                        "dur_med_us": round(float(np.median([x[1] for x in v])), 1),
                        "dur_max_us": round(float(max(x[1] for x in v)), 1)}
               for k, v in sorted(by_len.items(), reverse=True)[:6]}
    res[f"tpb{tpb}"] = {"kernel_us": round(float(end.max()), 1),
                        "distinct_cus": len(set(key)),
                        "long_waves_per_cu_max": max(per_cu.values()),
                        "long_cus": len(per_cu),
                        "long_waves_per_simd_max": max(per_simd.values()),
                        "by_len": summary}
print(json.dumps(res))

# slow long waves: who shared their CU / SIMD, and when
long_w = [w for w in range(nw) if wave_len[w] >= (1 << 20)]
durs = sorted(dur[w] for w in long_w)
detail = {"long_dur_us_quantiles": [round(float(np.quantile(durs, q)), 1) for q in (0, .1, .5, .9, .95, 1)]}
slow = sorted(long_w, key=lambda w: -dur[w])[:6]
fast = sorted(long_w, key=lambda w: dur[w])[:3]
def neighbours(w):
    same_cu = [v for v in range(nw) if v != w and key[v] == key[w]]
    same_simd = [v for v in same_cu if simd[v] == simd[w]]
    busy = lambda vs: round(float(sum(dur[v] for v in vs)) / 1000.0, 2)   # ms of co-resident wave time
    return {"xcc": key[w][0], "se": key[w][1], "cu": key[w][3], "simd": int(simd[w]),
            "dur_us": round(float(dur[w]), 1), "cu_waves": len(same_cu), "cu_busy_ms": busy(same_cu),
            "simd_waves": len(same_simd), "simd_busy_ms": busy(same_simd)}
detail["slowest"] = [neighbours(w) for w in slow]
detail["fastest"] = [neighbours(w) for w in fast]
print(json.dumps(detail))
