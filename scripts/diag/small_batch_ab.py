#!/usr/bin/env python3
"""Which descriptor kernel is fastest for a SMALL batch -- the netcache call
site's vector of 16-1,024 blocks, where a launch is one to a few waves and its
time is one chunk's serial chain?  For n x L device-resident
chunks (contiguous, 16-B aligned, identity order) the four descriptor kernels
(XDMA, LANE, HYBRID, BALANCED) are launched back to back, each timed per
launch with HIP events (after 20 untimed launches of its own), in interleaved
rounds; digests must equal XDMA's.  Prints one JSON object.
With --crc: the product's CRC-32 kernels on the same batches instead
(crc32hip_desc_variant through the descriptors, crc32hip_fixed_variant on the
contiguous layout; XDMA16 streaming against SPLIT, one wave per chunk),
CRCs checked equal to each other.
With --fed: also the diagnostic library's fed pairs for every group
(md5diag_variant_desc 9: a feeder wave forms M + K for the chain wave, 4 VALU
per step on the chain instead of 5), and the same with each pair
padded to a whole CU's LDS (md5diag_fed_split_excl 2).
usage: small_batch_ab.py [--sizes 16,64,256,1024,4096] [--len 16384] [--iters 100] [--crc] [--fed]"""
import argparse
import ctypes
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

VARIANTS = {"xdma": 4, "lane": 1, "hybrid": 3, "balanced": 5, "fed": 6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="16,64,256,1024,4096")
    ap.add_argument("--len", type=int, default=16384)
    ap.add_argument("--iters", type=int, default=100)
    ap.add_argument("--rounds", type=int, default=2)
    ap.add_argument("--crc", action="store_true")
    ap.add_argument("--fed", action="store_true")
    ap.add_argument("--fastcrc", type=int, default=0, help="with --crc: blk_make_crc's window size")
    a = ap.parse_args()
    import torch
    from sproxy_amd._lib import lib
    L = lib()
    D = None
    if a.fed:
        D = ctypes.CDLL(os.path.join(REPO, "build", "diag", "libmd5hip_diag.so"), mode=ctypes.RTLD_LOCAL)
        vp = ctypes.c_void_p
        D.md5diag_variant_desc.argtypes = [ctypes.c_int, vp, vp, vp, vp, ctypes.c_uint64, vp, vp]
        D.md5diag_fed_split_excl.argtypes = [ctypes.c_int, ctypes.c_uint64, vp, vp, vp, vp,
                                             ctypes.c_uint64, vp, vp]
    stream = torch.cuda.Stream()
    sp = ctypes.c_void_p(stream.cuda_stream)
    out = {"len": a.len, "iters": a.iters, "fastcrc": a.fastcrc, "sizes": {}}
    nmax = max(int(x) for x in a.sizes.split(","))
    data = torch.empty(nmax * a.len, dtype=torch.uint8, device="cuda")
    rc = L.md5hip_fill_synthetic(ctypes.c_void_p(data.data_ptr()), data.numel(), 12345, sp)
    assert rc == 0, rc
    for n in (int(x) for x in a.sizes.split(",")):
        offs = torch.arange(n, dtype=torch.int64, device="cuda") * a.len
        lens = torch.full((n,), a.len, dtype=torch.int32, device="cuda")
        variants = ({"crc_desc_xdma16": 6, "crc_desc_split": 7, "crc_fixed_xdma16": 106,
                     "crc_fixed_split": 107} if a.crc else dict(VARIANTS))
        if D is not None and not a.crc:
            variants["fed_diag"] = -9
            variants["fed_excl"] = -1002
        dsz = 4 if a.crc else 16
        dig = {v: torch.zeros((n, dsz), dtype=torch.uint8, device="cuda") for v in variants}
        res = {v: [] for v in variants}
        for r in range(a.rounds):
            for v, code in variants.items():
                def launch():
                    d, o, ln = (ctypes.c_void_p(t.data_ptr()) for t in (data, offs, lens))
                    out_p = ctypes.c_void_p(dig[v].data_ptr())
                    if a.crc and code < 100:
                        return L.crc32hip_desc_variant(d, o, ln, None, n, a.fastcrc, out_p, sp, code)
                    if a.crc:
                        return L.crc32hip_fixed_variant(d, n, a.len, a.len, a.fastcrc, out_p, sp, code - 100)
                    if code <= -1000:
                        return D.md5diag_fed_split_excl(-code - 1000, 0, d, o, ln, None, n, out_p, sp)
                    if code < 0:
                        return D.md5diag_variant_desc(-code, d, o, ln, None, n, out_p, sp)
                    return L.md5hip_digest_desc_variant(d, o, ln, None, n, out_p, sp, code)
                with torch.cuda.stream(stream):
                    for _ in range(20):
                        assert launch() == 0
                    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2 * a.iters)]
                    for k in range(a.iters):
                        ev[2 * k].record(stream)
                        launch()
                        ev[2 * k + 1].record(stream)
                stream.synchronize()
                res[v] += [ev[2 * k].elapsed_time(ev[2 * k + 1]) * 1e3 for k in range(a.iters)]
        ref = dig["crc_desc_xdma16" if a.crc else "xdma"].cpu()
        row = {}
        for v in variants:
            t = sorted(res[v])
            row[v] = {"median_us": round(t[len(t) // 2], 1), "p10_us": round(t[len(t) // 10], 1),
                      "p90_us": round(t[9 * len(t) // 10], 1), "digests_equal": bool(torch.equal(dig[v].cpu(), ref))}
        out["sizes"][str(n)] = row
        print(n, json.dumps(row), file=sys.stderr, flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
