#!/usr/bin/env python3
"""tests/golden/ncmd5_golden.json from the REFERENCE nc_MD5
(/root/reference/netcache/netcache/md5.c built in place into
oracle/_ref/libncmd5_ref.so).  Inputs: the RFC 1321 suite strings the
reference itself lists (netcache/netcache/md5.c:498-512), cache-key-like
strings, and generated lengths 0..300 plus a few long ones."""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
import gen  # noqa: E402

L = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libncmd5_ref.so"))


def ref(data: bytes, splits=()):
    ctx = ctypes.create_string_buffer(128)
    L.nc_MD5Init(ctx)
    prev = 0
    for s in list(splits) + [len(data)]:
        part = data[prev:s]
        L.nc_MD5Update(ctx, ctypes.c_char_p(part), ctypes.c_uint(len(part)))
        prev = s
    L.nc_MD5Final(ctx)
    return ctx.raw[112:128].hex()


def main():
    msgs = [b"", b"a", b"abc", b"message digest", b"abcdefghijklmnopqrstuvwxyz",
            b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
            b"1234567890" * 8,
            b"http://origin.example.com/vod/movie.mp4?start=10", b"/volume1/obj/abc.ts#gzip",
            b"10.0.0.17:8080"]
    big = gen.mul_pattern(70000)
    lens = list(range(0, 300)) + [511, 512, 513, 4096, 65536, 70000]
    out = {"generated_by": "tests/golden/make_golden_ncmd5.py from netcache/netcache/md5.c",
           "strings": [{"hex": m.hex(), "md5": ref(m)} for m in msgs],
           "lengths": lens, "mul_pattern_md5": [ref(big[:n]) for n in lens]}
    assert out["strings"][0]["md5"] == "e4c23762ed2823a27e62a64b95c024e7"
    assert out["strings"][2]["md5"] == "7999dc75e8da648c6727e137c5b77803"
    for n in (0, 1, 63, 64, 65, 299, 4096):                                 # split invariance
        assert ref(big[:n], [n // 3]) == out["mul_pattern_md5"][lens.index(n)]
    path = os.path.join(HERE, "ncmd5_golden.json")
    json.dump(out, open(path, "w"), indent=0)
    print("wrote", path, os.path.getsize(path))


if __name__ == "__main__":
    main()
