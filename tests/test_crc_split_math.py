"""CPU restatement of crc32_split's arithmetic (md5_kernels.h, hashers.h
CrcShift), pinned to zlib's CRC-32 (the crc32.c polynomial, crc32.c:22):
the register is linear in its start value and in the data, so a message cut
into 256-B segments counted from its end (the first holding the L mod 256
leftover bytes, or 256) is the XOR of each segment's register -- the first
from ~0, the others from 0 -- advanced through the bytes after it by the
zero-byte operators built by repeated squaring, combined in a 6-level tree
over 64 lanes and pass after pass through 16 KiB, exactly as the kernel
does.  Test infrastructure only (numpy + zlib)."""
import zlib

import numpy as np

POLY = 0xEDB88320


def _zero_byte_op():
    cols = []
    for i in range(32):
        c = 1 << i
        for _ in range(8):
            c = (c >> 1) ^ POLY if c & 1 else c >> 1
        cols.append(c)
    return cols


def _apply(op, v):
    r = 0
    for i in range(32):
        if (v >> i) & 1:
            r ^= op[i]
    return r


def _shift_ops():
    """m[l] = operator for 256 * 2^l zero bytes, l = 0..6 (hashers.h CrcShift)."""
    cur, out = _zero_byte_op(), []
    for sq in range(14):
        cur = [_apply(cur, cur[i]) for i in range(32)]
        if sq >= 7:
            out.append(cur)
    return out


OPS = _shift_ops()


def _reg(data: bytes, start: int) -> int:
    """The raw register after `data` from `start` (no final complement)."""
    return zlib.crc32(data, start ^ 0xFFFFFFFF) ^ 0xFFFFFFFF


def split_crc(msg: bytes) -> int:
    L = len(msg)
    if L == 0:
        return 0
    nseg = (L + 255) >> 8
    r0 = L - ((nseg - 1) << 8)
    npass = (nseg + 63) >> 6
    acc = 0
    for p in range(npass):
        regs = []
        for lane in range(64):
            s = nseg - 64 * (npass - p) + lane
            if s < 0:
                regs.append(0)
                continue
            start = 0 if s == 0 else r0 + ((s - 1) << 8)
            ln = r0 if s == 0 else 256
            regs.append(_reg(msg[start:start + ln], 0xFFFFFFFF if s == 0 else 0))
        for l in range(6):                       # the tree over __shfl_up
            d = 1 << l
            new = list(regs)
            for j in range(64):
                if (j & (2 * d - 1)) == 2 * d - 1:
                    new[j] = regs[j] ^ _apply(OPS[l], regs[j - d])
            regs = new
        acc = _apply(OPS[6], acc) ^ regs[63]
    return acc ^ 0xFFFFFFFF


def test_zero_byte_operators_match_zlib():
    rng = np.random.default_rng(1)
    for l in range(7):
        for _ in range(3):
            v = int(rng.integers(0, 1 << 32))
            n = 256 << l
            assert _apply(OPS[l], v) == _reg(bytes(n), v), l


def test_split_equals_crc32_at_segment_and_pass_boundaries():
    rng = np.random.default_rng(2)
    data = rng.integers(0, 256, (1 << 17) + 300, dtype=np.uint8).tobytes()
    for L in (1, 2, 3, 4, 5, 63, 64, 255, 256, 257, 511, 512, 513, 16383, 16384, 16385,
              16384 + 256, 32767, 32768, 32769, (1 << 17) + 13):
        assert split_crc(data[:L]) == zlib.crc32(data[:L]), L
    assert split_crc(b"") == zlib.crc32(b"") == 0
