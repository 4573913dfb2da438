#!/usr/bin/env python3
"""Is fastcrc=128 (blk_make_crc's head ^ tail windows, blk_io.c:408-424)
bound by where its windows fall in HBM?  The same kernel (crc32_fast_pipe)
over 1,048,576 blocks of 16 KiB laid at the C2 stride (16 KiB: every head
window 16 KiB from the next) and at padded strides that move consecutive
windows onto other address bits; ms per launch (hipEvent, median of 15
after 5 warm-up launches), G blocks/s.  Also fastcrc=64 and the full CRC.
usage: fastcrc_stride.py [--out F]"""
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
    n, L = 1 << 20, 16384
    res = {}
    for pad in (0, 128, 256, 4096):
        stride = L + pad
        buf = m.arena_empty(n * stride)
        m.fill_synthetic(buf, seed=7)
        for F in (128, 64):
            for _ in range(5):
                m.crc32_fixed(buf, n, L, stride, fastcrc=F)
            torch.cuda.synchronize()
            t = []
            for _ in range(15):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                m.crc32_fixed(buf, n, L, stride, fastcrc=F)
                e1.record()
                e1.synchronize()
                t.append(e0.elapsed_time(e1))
            t.sort()
            ms = t[len(t) // 2]
            res[f"stride{stride}_f{F}"] = {"ms": round(ms, 4), "g_blocks_s": round(n / ms / 1e6, 2),
                                           "window_bytes_tb_s": round(2 * F * n / ms / 1e9, 3)}
            print(f"stride {stride} F {F}: {ms:.4f} ms, {n / ms / 1e6:.2f} G blocks/s", flush=True)
        del buf
        torch.cuda.empty_cache()
    rec = {"probe": "fastcrc_stride", "blocks": n, "block_bytes": L, "results": res}
    print(json.dumps(rec))
    if a.out:
        open(a.out, "w").write(json.dumps(rec, indent=1) + "\n")


if __name__ == "__main__":
    main()
