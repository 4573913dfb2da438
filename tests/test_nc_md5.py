"""netcache nc_MD5 (LP64 semantics) -- host path of libmd5hip.so vs the
vectors from the reference build (tests/golden/ncmd5_golden.json) and the
pure-Python restatement (oracle/nc_md5_oracle.py)."""
import ctypes
import hashlib
import json
import os
import sys

import numpy as np

import gen
from sproxy_amd import _lib

sys.path.insert(0, os.path.join(gen.REPO, "oracle"))
import nc_md5_oracle  # noqa: E402

GOLD = json.load(open(os.path.join(gen.REPO, "tests", "golden", "ncmd5_golden.json")))


def product(data: bytes, splits=()):
    L = _lib.lib()
    ctx = ctypes.create_string_buffer(128)
    L.nc_MD5Init(ctx)
    prev = 0
    for s in list(splits) + [len(data)]:
        part = data[prev:s]
        L.nc_MD5Update(ctx, ctypes.c_char_p(part), ctypes.c_uint(len(part)))
        prev = s
    L.nc_MD5Final(ctx)
    return ctx.raw[112:128].hex()


def test_strings():
    for v in GOLD["strings"]:
        m = bytes.fromhex(v["hex"])
        assert product(m) == v["md5"]
        assert nc_md5_oracle.nc_md5(m).hex() == v["md5"]


def test_lengths_and_splits():
    big = gen.mul_pattern(max(GOLD["lengths"]))
    rng = np.random.default_rng(4)
    for n, d in zip(GOLD["lengths"], GOLD["mul_pattern_md5"]):
        cuts = sorted(int(x) for x in rng.integers(0, n + 1, 2))
        assert product(big[:n], cuts) == d, n
        if n <= 4096:
            assert nc_md5_oracle.nc_md5(big[:n]).hex() == d, n


def test_not_rfc_md5():
    assert product(b"") != hashlib.md5(b"").hexdigest()
