#!/usr/bin/env python3
"""fastcrc=128 (crc32_fast_pipe) over 1, 2 and 4 M blocks of 16 KiB at the C2
stride: ms per launch from 20 back-to-back launches between two hipEvents
(no per-launch event), G blocks/s and the window bytes' rate against 8 TB/s.
usage: fastcrc_batch.py [--out F]"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out")
    a = ap.parse_args()
    import torch
    from sproxy_amd import md5 as m
    L, F, K = 16384, 128, 20
    res = {}
    for n in (1 << 20, 2 << 20, 4 << 20):
        buf = m.arena_empty(n * L)
        m.fill_synthetic(buf, seed=7)
        for _ in range(5):
            m.crc32_fixed(buf, n, L, L, fastcrc=F)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(K):
            m.crc32_fixed(buf, n, L, L, fastcrc=F)
        e1.record()
        e1.synchronize()
        ms = e0.elapsed_time(e1) / K
        frac = 2 * F * n / ms / 1e6 / 8000.0     # window bytes per ms -> GB/s, over 8 TB/s
        res[str(n)] = {"ms_per_launch": round(ms, 4), "g_blocks_s": round(n / ms / 1e6, 2), "frac_of_8tbs": round(frac, 4)}
        print(n, res[str(n)], flush=True)
        del buf
        torch.cuda.empty_cache()
    rec = {"probe": "fastcrc_batch", "fastcrc": F, "block_bytes": L, "launches_timed": K, "results": res}
    print(json.dumps(rec))
    if a.out:
        open(a.out, "w").write(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    main()
