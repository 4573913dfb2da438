"""The host MD5Update of libmd5hip.so (sproxy_amd/csrc/md5_stream.c) leaves
all 88 bytes of struct MD5Context as the reference md5.c does, call by call.

md5.c:204-210 copies each whole block into ctx->in before transforming it, so
after an update in[] holds the last whole block with the tail copied over its
first bytes (md5.c:214); a partial fill that does not complete a block leaves
the stale bytes past it alone (md5.c:192-194).  The digest does not depend on
those bytes, the context does.  The checker is the reference md5.c compiled
where it lies (oracle/_ref/libmd5_ref.so, oracle/Makefile); both libraries are
driven on separate copies of the same contexts, stale in[] bytes preset."""
import ctypes
import os

import numpy as np
import pytest

import gen
from sproxy_amd import _lib

REF = os.path.join(gen.REPO, "oracle", "_ref", "libmd5_ref.so")


@pytest.fixture(scope="module")
def libs():
    if not os.path.exists(REF):
        pytest.skip("oracle/_ref/libmd5_ref.so not built (make -C oracle ref)")
    ref = ctypes.CDLL(REF)
    prod = _lib.lib()
    for L in (ref, prod):
        L.MD5Init.argtypes = [ctypes.c_void_p]
        L.MD5Update.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint]
        L.MD5Final.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.MD5Init.restype = L.MD5Update.restype = L.MD5Final.restype = None
    return ref, prod


class Pair:
    """One context driven through both libraries."""

    def __init__(self, libs, stale: np.ndarray):
        self.ref, self.prod = libs
        self.a = np.zeros(88, np.uint8)
        self.b = np.zeros(88, np.uint8)
        self.ref.MD5Init(self.a.ctypes.data)
        self.prod.MD5Init(self.b.ctypes.data)
        self.a[24:] = stale                      # MD5Init leaves in[] untouched (md5.c:153-163)
        self.b[24:] = stale
        assert np.array_equal(self.a, self.b)

    def update(self, data: np.ndarray, off: int, n: int):
        p = data.ctypes.data + off
        self.ref.MD5Update(self.a.ctypes.data, p, n)
        self.prod.MD5Update(self.b.ctypes.data, p, n)
        return np.array_equal(self.a, self.b)

    def final(self):
        da, db = np.zeros(16, np.uint8), np.zeros(16, np.uint8)
        self.ref.MD5Final(da.ctypes.data, self.a.ctypes.data)
        self.prod.MD5Final(db.ctypes.data, self.b.ctypes.data)
        return np.array_equal(da, db) and np.array_equal(self.a, self.b) and not self.b.any()


def test_single_update_every_length_below_300(libs):
    """one update of each length in [0, 300) from a fresh
    context with stale in[]; 236 of these differed before the fix."""
    rng = np.random.default_rng(11)
    data = rng.integers(0, 256, 300 + 64, dtype=np.uint8)
    for L in range(300):
        p = Pair(libs, rng.integers(0, 256, 64, dtype=np.uint8))
        assert p.update(data, int(rng.integers(0, 64)), L), L
        assert p.final(), L


def test_golden_random_lengths_splits(libs, golden):
    """tests/golden random_lengths: update data[:split] then data[split:len]."""
    g = golden["random_lengths"]
    lens, splits = g["lengths"], g["splits"]
    data = gen.xorshift_array(max(lens) + 64, seed=0x243F6A8885A308D3)
    rng = np.random.default_rng(12)
    for L, s, want in zip(lens, splits, g["md5"]):
        p = Pair(libs, rng.integers(0, 256, 64, dtype=np.uint8))
        assert p.update(data, 0, s) and p.update(data, s, L - s), (L, s)
        d = np.zeros(16, np.uint8)
        libs[1].MD5Final(d.ctypes.data, p.b.ctypes.data)
        assert d.tobytes().hex() == want
        assert not p.b.any()


def test_random_multi_call_sequences(libs):
    """Random sequences of 1..12 updates with lengths from 0 to 300 K (sub-block,
    straddling, exact-fill, multi-block), any source alignment, every context
    byte compared after every call."""
    rng = np.random.default_rng(13)
    data = rng.integers(0, 256, (300 << 10) + 4096, dtype=np.uint8)
    kinds = [lambda: int(rng.integers(0, 64)), lambda: int(rng.integers(64, 200)),
             lambda: 64 * int(rng.integers(1, 5)), lambda: int(rng.integers(200, 20000)),
             lambda: int(rng.integers(0, 300 << 10))]
    for seq in range(300):
        p = Pair(libs, rng.integers(0, 256, 64, dtype=np.uint8))
        for call in range(int(rng.integers(1, 13))):
            used = (int(p.a[16:20].view("<u4")[0]) >> 3) & 63
            if used and rng.random() < 0.3:
                n = 64 - used                     # exactly completes the pending block
            else:
                n = kinds[int(rng.integers(0, len(kinds)))]()
            off = int(rng.integers(0, data.size - n + 1))
            assert p.update(data, off, n), (seq, call, n)
        assert p.final(), seq


def test_bitcount_carry_context_bytes(libs):
    """bits[] with carry (md5.c:179-182) and in[] agree around 2^32 bits."""
    rng = np.random.default_rng(14)
    data = rng.integers(0, 256, 1 << 16, dtype=np.uint8)
    for low in (0xFFFFFFF8, 0xFFFFFE00, 0xFFFFFC08):
        p = Pair(libs, rng.integers(0, 256, 64, dtype=np.uint8))
        for arr in (p.a, p.b):
            arr[16:20].view("<u4")[0] = low
        for n in (3, 61, 64, 1000, 40000):
            assert p.update(data, int(rng.integers(0, 100)), n), (hex(low), n)
        assert p.final()
