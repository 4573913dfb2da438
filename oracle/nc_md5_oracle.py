"""oracle/nc_md5_oracle.py -- TEST INFRASTRUCTURE ONLY.

Pure-Python restatement of netcache's nc_MD5 on an LP64 host
(/root/reference/netcache/netcache/md5.c with UINT4 = unsigned long = 64 bits,
netcache/include/md5.h:40): 64-bit adds and round functions (md5.c:116-119),
ROTATE_LEFT(x, n) = (x << n) | (x >> (32 - n)) in 64 bits (md5.c:122), bit
counters kept as md5.c:180-183, length words stored whole (md5.c:211-212),
digest = low 32 bits of each state word (md5.c:232-238).  Small inputs only.
Pinned by tests/test_nc_md5.py against vectors from the reference build."""
M64 = (1 << 64) - 1
K = [0xd76aa478, 0xe8c7b756, 0x242070db, 0xc1bdceee, 0xf57c0faf, 0x4787c62a, 0xa8304613,
     0xfd469501, 0x698098d8, 0x8b44f7af, 0xffff5bb1, 0x895cd7be, 0x6b901122, 0xfd987193,
     0xa679438e, 0x49b40821, 0xf61e2562, 0xc040b340, 0x265e5a51, 0xe9b6c7aa, 0xd62f105d,
     0x02441453, 0xd8a1e681, 0xe7d3fbc8, 0x21e1cde6, 0xc33707d6, 0xf4d50d87, 0x455a14ed,
     0xa9e3e905, 0xfcefa3f8, 0x676f02d9, 0x8d2a4c8a, 0xfffa3942, 0x8771f681, 0x6d9d6122,
     0xfde5380c, 0xa4beea44, 0x4bdecfa9, 0xf6bb4b60, 0xbebfbc70, 0x289b7ec6, 0xeaa127fa,
     0xd4ef3085, 0x04881d05, 0xd9d4d039, 0xe6db99e5, 0x1fa27cf8, 0xc4ac5665, 0xf4292244,
     0x432aff97, 0xab9423a7, 0xfc93a039, 0x655b59c3, 0x8f0ccc92, 0xffeff47d, 0x85845dd1,
     0x6fa87e4f, 0xfe2ce6e0, 0xa3014314, 0x4e0811a1, 0xf7537e82, 0xbd3af235, 0x2ad7d2bb,
     0xeb86d391]
S = [(7, 12, 17, 22), (5, 9, 14, 20), (4, 11, 16, 23), (6, 10, 15, 21)]


def _transform(st, m):
    v = list(st)
    for j in range(64):
        r, i = j >> 4, j & 15
        w = (4 - (j & 3)) & 3
        x, y, z = v[(w + 1) & 3], v[(w + 2) & 3], v[(w + 3) & 3]
        nx, nz = ~x & M64, ~z & M64
        if r == 0:
            f, g = (x & y) | (nx & z), i
        elif r == 1:
            f, g = (x & z) | (y & nz), (5 * i + 1) & 15
        elif r == 2:
            f, g = x ^ y ^ z, (3 * i + 5) & 15
        else:
            f, g = y ^ (x | nz), (7 * i) & 15
        a = (v[w] + f + m[g] + K[j]) & M64
        s = S[r][j & 3]
        a = ((a << s) | (a >> (32 - s))) & M64
        v[w] = (a + x) & M64
    return [(st[k] + v[k]) & M64 for k in range(4)]


def nc_md5(data: bytes) -> bytes:
    st = [0x67452301, 0xefcdab89, 0x98badcfe, 0x10325476]
    n = len(data)
    i0 = (n << 3) & M64                      # single Update of n bytes from zero
    i1 = n >> 29
    if n << 3 > M64:
        i1 += 1
    msg = bytes(data)
    fill = n & 63
    pad = (56 - fill) if fill < 56 else (120 - fill)
    body = msg + b"\x80" + b"\0" * (pad - 1)
    words = lambda blk, k: [int.from_bytes(blk[4 * t:4 * t + 4], "little") for t in range(k)]  # noqa: E731
    for off in range(0, len(body) - 56, 64):
        st = _transform(st, words(body[off:off + 64], 16))
    last = body[len(body) - 56:]
    st = _transform(st, words(last, 14) + [i0, i1])
    return b"".join((w & 0xFFFFFFFF).to_bytes(4, "little") for w in st)
