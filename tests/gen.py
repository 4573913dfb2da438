"""Deterministic test-data generators shared by the tests, the golden-fixture
script and bench.py's cpu_baseline leg.  Test infrastructure: the product never
imports this module."""
import ctypes
import os

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C1_SEED = 0x9E3779B97F4A7C15
SIZE_CLASSES = [4096 << k for k in range(9)]   # 4 KiB .. 1 MiB (httpd.c:7968 range)

_oracle = None


def oracle_lib():
    """ctypes handle on oracle/_build/libmd5_oracle.so (the checker)."""
    global _oracle
    if _oracle is None:
        path = os.path.join(REPO, "oracle", "_build", "libmd5_oracle.so")
        lib = ctypes.CDLL(path)
        lib.oracle_md5.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        lib.oracle_md5_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint64, ctypes.c_void_p]
        lib.oracle_md5_batch_fixed.argtypes = [ctypes.c_void_p, ctypes.c_uint64,
                                               ctypes.c_uint32, ctypes.c_void_p]
        lib.oracle_xorshift_fill.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64]
        lib.oracle_md5_ctx_size.restype = ctypes.c_size_t
        _oracle = lib
    return _oracle


def mul_pattern(n: int) -> bytes:
    """buf[i] = (u8)((u32)(i * 2654435761) >> 24)  (SURVEY.md §8(c) edge goldens)."""
    i = np.arange(n, dtype=np.uint64)
    return (((i * np.uint64(2654435761)) & np.uint64(0xFFFFFFFF)) >> np.uint64(24)).astype(np.uint8).tobytes()


def xorshift_array(nbytes: int, seed: int = C1_SEED) -> np.ndarray:
    """xorshift64 13/7/17 stream, u64 stored little-endian."""
    out = np.empty(max(nbytes, 1), dtype=np.uint8)
    oracle_lib().oracle_xorshift_fill(out.ctypes.data, nbytes, seed)
    return out[:nbytes]


def xorshift_bytes(nbytes: int, seed: int = C1_SEED) -> bytes:
    return xorshift_array(nbytes, seed).tobytes()


def fold(raw) -> int:
    """fold = fold*31 + byte (u32) over a byte string."""
    b = np.frombuffer(bytes(raw), dtype=np.uint8).astype(np.uint64)
    n = b.size
    if n == 0:
        return 0
    p = np.full(n, 31, dtype=np.uint64)
    p[0] = 1
    p = np.cumprod(p, dtype=np.uint64)[::-1] & np.uint64(0xFFFFFFFF)   # 31^(n-1-i) mod 2^32
    # wraps mod 2^64 are harmless: 2^32 divides 2^64
    return int(np.sum(b * p, dtype=np.uint64) & np.uint64(0xFFFFFFFF))


def mixed_lengths(n: int, seed: int, max_len: int = 1 << 20, tail_every: int = 8):
    """C3 chunk lengths: classes 4 KiB..max_len, 1-in-`tail_every` a tail chunk of
    random length in [1, class) like the last block of an object (blk_io.c:377)."""
    rng = np.random.default_rng(seed)
    classes = [c for c in SIZE_CLASSES if c <= max_len]
    out = []
    for _ in range(n):
        c = int(classes[int(rng.integers(0, len(classes)))])
        if int(rng.integers(0, tail_every)) == 0:
            c = int(rng.integers(1, c))
        out.append(c)
    return out


def pack_offsets(lens, align: int = 64):
    offs, cur = [], 0
    for L in lens:
        offs.append(cur)
        cur += (L + align - 1) // align * align
    return offs, cur


def oracle_digests_fixed(buf: np.ndarray, n: int, length: int) -> np.ndarray:
    out = np.empty((max(n, 1), 16), dtype=np.uint8)
    oracle_lib().oracle_md5_batch_fixed(buf.ctypes.data, n, length, out.ctypes.data)
    return out[:n]


def oracle_digests(buf: np.ndarray, offs, lens) -> np.ndarray:
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    n = offs.size
    out = np.empty((max(n, 1), 16), dtype=np.uint8)
    oracle_lib().oracle_md5_batch(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, n,
                                  out.ctypes.data)
    return out[:n]


def synthetic_bytes(nbytes: int, seed: int) -> np.ndarray:
    """numpy mirror of the device generator md5hip_fill_synthetic: u32 word i =
    splitmix64-finaliser(seed + (i+1)*0x9E3779B97F4A7C15), little-endian."""
    with np.errstate(over="ignore"):
        i = np.arange(nbytes // 4, dtype=np.uint64)
        z = np.uint64(seed & (2**64 - 1)) + (i + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return (z & np.uint64(0xFFFFFFFF)).astype("<u4").view(np.uint8)


def oracle_crc32_batch(buf: np.ndarray, offs, lens, fastcrc: int = 0) -> np.ndarray:
    """netcache block CRC-32 per chunk (oracle/crc32_oracle.c)."""
    L = oracle_lib()
    L.oracle_crc32_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
    offs = np.ascontiguousarray(offs, dtype=np.uint64)
    lens = np.ascontiguousarray(lens, dtype=np.uint32)
    out = np.empty(max(offs.size, 1), dtype=np.uint32)
    L.oracle_crc32_batch(buf.ctypes.data, offs.ctypes.data, lens.ctypes.data, offs.size, fastcrc,
                         out.ctypes.data)
    return out[:offs.size]
