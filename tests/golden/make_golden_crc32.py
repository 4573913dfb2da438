#!/usr/bin/env python3
"""Regenerate tests/golden/crc32_golden.json from the REFERENCE netcache CRC32
(/root/reference/netcache/netcache/crc32.c, built in place by oracle/Makefile
into oracle/_ref/crc32_ref_tool).  Every value is cross-checked with Python's
zlib.crc32 (same polynomial, crc32.c:22) before it is written.  Run in the
build container only; the GPU box reads the committed JSON."""
import json
import os
import struct
import subprocess
import sys
import zlib

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
import gen  # noqa: E402

TOOL = os.path.join(REPO, "oracle", "_ref", "crc32_ref_tool")


def ref(records):
    """records: list of (bytes, fastcrc) -> list of (crc8, crcbit, blkcrc) ints."""
    blob = b"".join(struct.pack("<II", len(d), f) + d for d, f in records)
    out = subprocess.run([TOOL], input=blob, capture_output=True, check=True).stdout.decode()
    return [tuple(int(x, 16) for x in ln.split()) for ln in out.splitlines()]


def blk_py(d, f):
    if f == 0 or len(d) <= f:
        return zlib.crc32(d)
    return zlib.crc32(d[:f]) ^ zlib.crc32(d[max(0, len(d) - f):])


def main():
    out = {"generated_by": "tests/golden/make_golden_crc32.py from /root/reference/netcache/netcache/crc32.c"}
    kat = [b"", b"a", b"abc", b"123456789", b"message digest", b"abcdefghijklmnopqrstuvwxyz",
           b"The quick brown fox jumps over the lazy dog", bytes(range(256)), b"\xff" * 100]
    r = ref([(k, 0) for k in kat])
    assert r[3][0] == 0xCBF43926                   # the CRC-32 check value
    for k, (c8, cb, _) in zip(kat, r):
        assert c8 == cb == zlib.crc32(k)
    out["kat"] = [{"hex": k.hex(), "crc": "%08x" % c[0]} for k, c in zip(kat, r)]
    big = gen.mul_pattern(1 << 20)
    lens = [0, 1, 3, 4, 7, 8, 9, 15, 16, 17, 63, 64, 65, 127, 128, 1000, 4095, 4096, 16383, 16384,
            16385, 65536, 131072, 1 << 20]
    r = ref([(big[:L], 0) for L in lens])
    for L, c in zip(lens, r):
        assert c[0] == c[1] == zlib.crc32(big[:L])
    out["edge"] = {"generator": "mul_pattern", "lengths": lens, "crc": ["%08x" % c[0] for c in r]}
    # fastcrc (blk_make_crc head ^ tail), fastcrc a multiple of 4 (cfs_apix.c:2222-2236)
    fcases = []
    for f in (4, 64, 128, 1000, 4096):
        for L in (0, 1, f - 1, f, f + 1, 2 * f - 1, 2 * f, 2 * f + 3, 16384, 100000):
            if L >= 0:
                fcases.append((L, f))
    data = gen.xorshift_bytes(100000, seed=0xC5C5)
    r = ref([(data[:L], f) for L, f in fcases])
    for (L, f), c in zip(fcases, r):
        assert c[2] == blk_py(data[:L], f), (L, f)
    out["fastcrc"] = {"generator": "xorshift_bytes(seed=0xC5C5)", "cases": [[L, f] for L, f in fcases],
                      "crc": ["%08x" % c[2] for c in r]}
    batches = []
    for n, L, keep in [(256, 16384, True), (4096, 16384, False), (1000, 4096, True), (77, 1000, True)]:
        buf = gen.xorshift_bytes(n * L)
        rr = ref([(buf[i * L:(i + 1) * L], 0) for i in range(n)])
        crcs = [c[0] for c in rr]
        assert crcs == [zlib.crc32(buf[i * L:(i + 1) * L]) for i in range(n)]
        e = {"n": n, "len": L, "seed": "0x9E3779B97F4A7C15",
             "fold": "%08x" % gen.fold(b"".join(struct.pack("<I", c) for c in crcs))}
        if keep:
            e["crc"] = ["%08x" % c for c in crcs]
        batches.append(e)
    out["batches"] = batches
    # on-disk header CRC (diskcache.c:1391-1393 write, :3660-3690 verify): CRC-32 over
    # header_size bytes with disk_header_size (4..8), flag (12..16), crc (16..20) as zero
    hdrs = []
    for k, hs in enumerate([20, 21, 27, 100, 1000, 4096, 70001]):
        body = gen.xorshift_bytes(hs, seed=0x4EAD + k)
        dhs, flag = (hs // 3, 0x10000000) if k % 2 else (0, 0)
        zeroed = struct.pack("<IiiII", 0x30334253, 0, hs, 0, 0) + body[20:]
        crc = ref([(zeroed, 0)])[0][0]
        assert crc == zlib.crc32(zeroed)
        hdrs.append({"header_size": hs, "body_seed": 0x4EAD + k, "disk_header_size": dhs,
                     "flag": flag, "crc": "%08x" % crc})
    out["headers"] = {"magic": "%08x" % 0x30334253, "cases": hdrs,
                      "layout": "<I magic, i disk_header_size, i header_size, I flag, I crc, then "
                                "xorshift_bytes(header_size, body_seed)[20:]"}
    path = os.path.join(HERE, "crc32_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main()
