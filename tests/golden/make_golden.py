#!/usr/bin/env python3
"""Regenerate tests/golden/md5_golden.json from the REFERENCE md5.c.

Run in the build container only (needs /root/reference, compiled in place by
``make -C oracle ref`` into oracle/_ref/libmd5_ref.so).  The GPU box never runs
this script; it only reads the committed JSON.

Inputs are data, not reference source:
  * RFC 1321 appendix A.5 test suite strings (also listed, as dead code, in
    /root/reference/netcache/netcache/md5.c:498-512);
  * the MHD unit vectors, /root/reference/MHD/0.9.73/src/microhttpd/test_md5.c
    :48-65 (strings) and :81-210 (binary), with their published digests;
  * curl tests/unit/unit1601.c ("1", "hello-you-fool");
  * generated buffers (edge lengths, random lengths, batches) whose digests
    come from the reference md5.c itself.
Each published digest is asserted against the reference build before writing.
"""
import ctypes
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(REPO, "tests"))
import gen  # noqa: E402  (shared deterministic generators)


class MD5Context(ctypes.Structure):  # md5.h:33-38
    _fields_ = [("buf", ctypes.c_uint32 * 4), ("bits", ctypes.c_uint32 * 2),
                ("in_", ctypes.c_ubyte * 64)]


def load_ref():
    path = os.path.join(REPO, "oracle", "_ref", "libmd5_ref.so")
    lib = ctypes.CDLL(path)
    lib.MD5Init.argtypes = [ctypes.POINTER(MD5Context)]
    lib.MD5Update.argtypes = [ctypes.POINTER(MD5Context), ctypes.c_void_p, ctypes.c_uint]
    lib.MD5Final.argtypes = [ctypes.c_void_p, ctypes.POINTER(MD5Context)]
    return lib


def ref_md5(lib, data: bytes, splits=()) -> str:
    ctx = MD5Context()
    lib.MD5Init(ctypes.byref(ctx))
    buf = ctypes.create_string_buffer(bytes(data), len(data) or 1)
    prev = 0
    for s in list(splits) + [len(data)]:
        lib.MD5Update(ctypes.byref(ctx), ctypes.addressof(buf) + prev, s - prev)
        prev = s
    out = (ctypes.c_ubyte * 16)()
    lib.MD5Final(out, ctypes.byref(ctx))
    return bytes(out).hex()


RFC = [b"", b"a", b"abc", b"message digest", b"abcdefghijklmnopqrstuvwxyz",
       b"ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz0123456789",
       b"1234567890" * 8]
RFC_MD5 = ["d41d8cd98f00b204e9800998ecf8427e", "0cc175b9c0f1b6a831c399e269772661",
           "900150983cd24fb0d6963f7d28e17f72", "f96b697d7cb7938d525a2f31aaf161d0",
           "c3fcd3d76192e4007dfb496cca67e13b", "d174ab98d277d9f5a5611c2c9f419d9f",
           "57edf4a22be3c955ac49da2e2107b67a"]

_MHD_RAND = bytes([
    41, 35, 190, 132, 225, 108, 214, 174, 82, 144, 73, 241, 241, 187, 233, 235, 179, 166,
    219, 60, 135, 12, 62, 153, 36, 94, 13, 28, 6, 183, 71, 222, 179, 18, 77, 200, 67, 187,
    139, 166, 31, 3, 90, 125, 9, 56, 37, 31, 93, 212, 203, 252, 150, 245, 69, 59, 19, 13,
    137, 10, 28, 219, 174, 50, 32, 154, 80, 238, 64, 120, 54, 253, 18, 73, 50, 246, 158,
    125, 73, 220, 173, 79, 20, 242, 68, 64, 102, 208, 107, 196, 48, 183, 50, 59, 161, 34,
    246, 34, 145, 157, 225, 139, 31, 218, 176, 202, 153, 2, 185, 114, 157, 73, 44, 128,
    126, 197, 153, 213, 233, 128, 178, 234, 201, 204, 83, 191, 103, 214, 191, 20, 214, 126,
    45, 220, 142, 102, 131, 239, 87, 73, 97, 255, 105, 143, 97, 205, 209, 30, 157, 156, 22,
    114, 114, 230, 29, 240, 132, 79, 74, 119, 2, 215, 232, 57, 44, 83, 203, 201, 18, 30, 51,
    116, 158, 12, 244, 213, 212, 159, 212, 164, 89, 126, 53, 207, 50, 34, 244, 204, 207,
    211, 144, 45, 72, 211, 143, 117, 230, 217, 29, 42, 229, 192, 247, 43, 120, 129, 135, 68,
    14, 95, 80, 0, 212, 97, 141, 190, 123, 5, 21, 7, 59, 51, 130, 31, 24, 112, 146, 218,
    100, 84, 206, 177, 133, 62, 105, 21, 248, 70, 106, 4, 150, 115, 14, 217, 22, 47, 103,
    104, 212, 247, 74, 74, 208, 87, 104])

# (name, input, published digest) -- test_md5.c:48-65 and :81-210
MHD = [
    ("mhd_str1", b"1234567890!@~%&$@#{}[]\\/!?`.", "1c68c2e51f63c95f17ab1f208b863957"),
    ("mhd_str2", b"Simple string.", "f12b7cada041fede4e681663b4605d78"),
    ("mhd_str3", b"abcdefghijklmnopqrstuvwxyz", "c3fcd3d76192e4007dfb496cca67e13b"),
    ("mhd_str4", b"zyxwvutsrqponMLKJIHGFEDCBA", "05613a6bde753a4591a881b0a7e2e20e"),
    ("mhd_str5", b"abcdefghijklmnopqrstuvwxyzzyxwvutsrqponMLKJIHGFEDCBA" * 2,
     "afabc7e9e717bed6c00f788cdedd11d1"),
    ("mhd_bin1", bytes(range(97, 123)), "c3fcd3d76192e4007dfb496cca67e13b"),
    ("mhd_bin2", b"A" * 72, "24a5ef3682803a062feaadad76dabda8"),
    ("mhd_bin3", bytes(range(19, 74)), "6d2e6ede5d646a17f1092cac1910e3d6"),
    ("mhd_bin4", bytes(range(7, 70)), "8813484773aa92f2c9dd69b3acf4ba6e"),
    ("mhd_bin5", bytes(range(38, 93)), "80f0057ea2f7c84312d3b161ab523baf"),
    ("mhd_bin6", bytes(range(1, 73)), "c328c5adc926a999954a5e2550345173"),
    ("mhd_bin7", bytes(range(0, 256)), "e2c865db4162bed963bfaa9ef6ac18f0"),
    ("mhd_bin8", bytes(range(199, 138, -1)), "bb3fdb4a9603363738785e44bf3a8551"),
    ("mhd_bin9", bytes(range(255, 0, -1)), "5221a5834f387c73ba1822b1f97eae8b"),
    ("mhd_bin10", _MHD_RAND, "55612ceb29eea8b2f6107bc15b0f0195"),
]
CURL = [("curl_1", b"1", "c4ca4238a0b923820dcc509a6f75849b"),
        ("curl_hello", b"hello-you-fool", "88670b6d5d742fada5cdf9b682875f22")]

EDGE_LENGTHS = [0, 1, 2, 3, 4, 5, 7, 8, 15, 16, 31, 32, 33, 47, 48, 54, 55, 56, 57, 58, 62, 63,
                64, 65, 66, 100, 111, 112, 118, 119, 120, 121, 127, 128, 129, 191, 192, 255,
                256, 257, 1000, 1023, 1024, 4095, 4096, 4097, 8192, 16320, 16376, 16383, 16384,
                16385, 16440, 32768, 65535, 65536, 131072, 262144, 524288, 1048575, 1048576]


def main():
    lib = load_ref()
    out = {"generated_by": "tests/golden/make_golden.py from /root/reference/md5.c "
                           "(compiled in place by oracle/Makefile)",
           "kat": [], "edge": {}, "random_lengths": {}, "batches": [], "mixed": {}}
    for i, (m, d) in enumerate(zip(RFC, RFC_MD5)):
        got = ref_md5(lib, m)
        assert got == d, (m, got, d)
        out["kat"].append({"name": f"rfc1321_{i}", "source": "RFC 1321 A.5", "hex": m.hex(), "md5": d})
    for name, m, d in MHD:
        got = ref_md5(lib, m)
        assert got == d, (name, got, d)
        # MHD's split-update variants (test_md5.c:280-371): len/4 for strings, 2len/3 for bins
        cut = len(m) // 4 if "str" in name else len(m) * 2 // 3
        assert ref_md5(lib, m, [cut]) == d
        out["kat"].append({"name": name, "source": "MHD test_md5.c", "hex": m.hex(), "md5": d})
    for name, m, d in CURL:
        assert ref_md5(lib, m) == d
        out["kat"].append({"name": name, "source": "curl unit1601.c", "hex": m.hex(), "md5": d})

    # Edge lengths over the SURVEY §8(c) multiplicative generator.
    big = gen.mul_pattern(max(EDGE_LENGTHS))
    out["edge"] = {"generator": "mul_pattern: buf[i] = (u8)((u32)(i*2654435761) >> 24)",
                   "lengths": EDGE_LENGTHS,
                   "md5": [ref_md5(lib, big[:L]) for L in EDGE_LENGTHS]}
    # spot-check the survey's published edge values
    survey = {0: "d41d8cd98f00b204e9800998ecf8427e", 55: "1eec39e439a0686e0f16143c93e65544",
              16384: "2f2217e5c573a65adc70089d702e1c74", 1048576: "900fad0e36be8d5ba0cb1653208c9f07"}
    for L, d in survey.items():
        assert out["edge"]["md5"][EDGE_LENGTHS.index(L)] == d, L

    # Random lengths 0..4999 over xorshift64 data, with random two-way splits.
    rng = np.random.default_rng(1321)
    lens = [int(x) for x in rng.integers(0, 5000, size=200)]
    data = gen.xorshift_bytes(max(lens), seed=0x243F6A8885A308D3)
    splits = [int(rng.integers(0, L + 1)) for L in lens]
    out["random_lengths"] = {"generator": "xorshift_bytes(seed=0x243F6A8885A308D3)[:len]",
                             "lengths": lens, "splits": splits,
                             "md5": [ref_md5(lib, data[:L]) for L in lens]}
    for L, s, d in zip(lens, splits, out["random_lengths"]["md5"]):
        assert ref_md5(lib, data[:L], [s]) == d

    # Fixed-length batches (contiguous chunks of one xorshift64 stream).
    for n, L, keep in [(256, 16384, True), (1024, 4096, True), (64, 65536, True),
                       (65536, 16384, False), (4096, 16384, False), (333, 1000, True),
                       (100, 1, True), (50, 0, True)]:
        buf = gen.xorshift_bytes(n * L)
        digs = [ref_md5(lib, buf[i * L:(i + 1) * L]) for i in range(n)]
        raw = b"".join(bytes.fromhex(d) for d in digs)
        entry = {"n": n, "len": L, "seed": "0x9E3779B97F4A7C15", "fold": "%08x" % gen.fold(raw)}
        if keep:
            entry["md5"] = digs
        out["batches"].append(entry)
    assert out["batches"][3]["fold"] == "53a0a616"

    # Mixed-length batch (C3 shape, small n), packed contiguously at 64-byte alignment.
    lens = gen.mixed_lengths(96, seed=7, max_len=262144)
    offs, total = gen.pack_offsets(lens, align=64)
    buf = gen.xorshift_bytes(total, seed=0x13198A2E03707344)
    out["mixed"] = {"seed": 7, "max_len": 262144, "data_seed": "0x13198A2E03707344",
                    "align": 64, "lengths": lens, "offsets": offs,
                    "md5": [ref_md5(lib, buf[o:o + L]) for o, L in zip(offs, lens)]}

    path = os.path.join(HERE, "md5_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=0)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
