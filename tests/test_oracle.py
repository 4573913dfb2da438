"""The oracle (oracle/md5_oracle.c) pinned against the golden vectors.

Golden vectors come from the REFERENCE md5.c compiled in place
(tests/golden/make_golden.py): RFC 1321 A.5, MHD test_md5.c (:48-65, :81-210,
whole and split as :280-371 does), curl unit1601.c, edge lengths 0..1 MiB,
random lengths with random split points, and fixed-length batches (the C1
65,536 x 16 KiB fold 53a0a616 of SURVEY.md §8(c)).
"""
import ctypes
import hashlib
import os

import numpy as np
import pytest

import gen

REF_LIB = os.path.join(gen.REPO, "oracle", "_ref", "libmd5_ref.so")


def oracle_md5(data: bytes, splits=()) -> str:
    lib = gen.oracle_lib()
    ctx = ctypes.create_string_buffer(lib.oracle_md5_ctx_size())
    lib.oracle_md5_init(ctx)
    buf = ctypes.create_string_buffer(bytes(data), max(len(data), 1))
    prev = 0
    for s in list(splits) + [len(data)]:
        lib.oracle_md5_update(ctx, ctypes.c_void_p(ctypes.addressof(buf) + prev), ctypes.c_uint(s - prev))
        prev = s
    out = (ctypes.c_ubyte * 16)()
    lib.oracle_md5_final(out, ctx)
    assert ctx.raw == b"\0" * len(ctx.raw), "MD5Final must zero the context (md5.c:264)"
    return bytes(out).hex()


def test_ctx_layout():
    assert gen.oracle_lib().oracle_md5_ctx_size() == 88   # md5.h:33-38


def test_kat(golden):
    assert len(golden["kat"]) == 7 + 15 + 2
    for v in golden["kat"]:
        m = bytes.fromhex(v["hex"])
        assert oracle_md5(m) == v["md5"], v["name"]
        # split updates at every kind of boundary (MHD test2_*: len/4, 2len/3)
        for cut in {0, len(m) // 4, len(m) * 2 // 3, len(m)}:
            assert oracle_md5(m, [cut]) == v["md5"], (v["name"], cut)


def test_edge_lengths(golden):
    e = golden["edge"]
    big = gen.mul_pattern(max(e["lengths"]))
    for L, d in zip(e["lengths"], e["md5"]):
        assert oracle_md5(big[:L]) == d, L
        assert hashlib.md5(big[:L]).hexdigest() == d, L


def test_random_lengths_with_splits(golden):
    r = golden["random_lengths"]
    data = gen.xorshift_bytes(max(r["lengths"]), seed=0x243F6A8885A308D3)
    for L, s, d in zip(r["lengths"], r["splits"], r["md5"]):
        assert oracle_md5(data[:L], [s]) == d
        assert oracle_md5(data[:L], [s // 2, s]) == d


def test_fixed_batches(golden):
    for b in golden["batches"]:
        n, L = b["n"], b["len"]
        if n * L > (64 << 20):
            continue            # the 1 GiB fold is checked in test_c1_fold
        buf = gen.xorshift_array(n * L)
        dig = gen.oracle_digests_fixed(buf, n, L)
        assert "%08x" % gen.fold(dig.tobytes()) == b["fold"], (n, L)
        if "md5" in b:
            assert [bytes(x).hex() for x in dig] == b["md5"]


def test_c1_fold():
    """65,536 x 16 KiB xorshift64 -> fold 53a0a616 (1 GiB)."""
    n, L = 65536, 16384
    buf = gen.xorshift_array(n * L)
    dig = gen.oracle_digests_fixed(buf, n, L)
    assert "%08x" % gen.fold(dig.tobytes()) == "53a0a616"


def test_mixed_batch(golden):
    mx = golden["mixed"]
    lens, offs = mx["lengths"], mx["offsets"]
    assert gen.mixed_lengths(len(lens), seed=mx["seed"], max_len=mx["max_len"]) == lens
    assert gen.pack_offsets(lens, align=mx["align"])[0] == offs
    total = gen.pack_offsets(lens, align=mx["align"])[1]
    buf = gen.xorshift_array(total, seed=int(mx["data_seed"], 16))
    dig = gen.oracle_digests(buf, offs, lens)
    assert [bytes(x).hex() for x in dig] == mx["md5"]


def test_fold_matches_python_loop():
    raw = np.random.default_rng(0).integers(0, 256, 1000, dtype=np.uint8).tobytes()
    f = 0
    for b in raw:
        f = (f * 31 + b) & 0xFFFFFFFF
    assert gen.fold(raw) == f


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="oracle/_ref not built (no /root/reference)")
def test_oracle_equals_reference_build():
    """Where the reference md5.c build is present, it and the oracle agree on
    random inputs with random split points."""
    lib = ctypes.CDLL(REF_LIB)
    rng = np.random.default_rng(99)
    for _ in range(300):
        L = int(rng.integers(0, 3000))
        data = rng.integers(0, 256, L, dtype=np.uint8).tobytes()
        cuts = sorted(int(x) for x in rng.integers(0, L + 1, 3))
        ctx = ctypes.create_string_buffer(88)
        lib.MD5Init(ctx)
        buf = ctypes.create_string_buffer(data, max(L, 1))
        prev = 0
        for s in cuts + [L]:
            lib.MD5Update(ctx, ctypes.c_void_p(ctypes.addressof(buf) + prev), ctypes.c_uint(s - prev))
            prev = s
        out = (ctypes.c_ubyte * 16)()
        lib.MD5Final(out, ctx)
        assert bytes(out).hex() == oracle_md5(data, cuts)
