"""On-disk digest formats around the block checksum:
chunk #5 of netcache's object header (the blkno-indexed digest array,
netcache.h:408-410 / :879) and the header CRC (diskcache.c:1391-1393 write,
:3660-3690 verify).

The reference code for these lives inside diskcache.c, which needs the whole of
netcache to build, so it is unbuildable here; the CRC itself is pinned by the
reference crc32.c (tests/golden/crc32_golden.json "headers", produced by
oracle/_ref/crc32_ref_tool over the zeroed header bytes), and the field-zeroing
rule and array bounds are restated from the cited lines."""
import errno
import json
import os
import struct

import numpy as np
import pytest

import gen
from sproxy_amd import md5 as m
from sproxy_amd import nc_digest as nd

GOLD = json.load(open(os.path.join(gen.REPO, "tests", "golden", "crc32_golden.json")))


def _oracle_crc(b: bytes) -> int:
    a = np.frombuffer(b + b"\0", dtype=np.uint8)
    return int(gen.oracle_crc32_batch(a, [0], [len(b)])[0])


def _golden_headers():
    out = []
    for c in GOLD["headers"]["cases"]:
        hs = c["header_size"]
        body = gen.xorshift_bytes(hs, seed=c["body_seed"])
        h = bytearray(struct.pack("<IiiII", int(GOLD["headers"]["magic"], 16), c["disk_header_size"],
                                  hs, c["flag"], int(c["crc"], 16)) + body[20:])
        out.append((h, int(c["crc"], 16)))
    return out


def test_header_crc_golden():
    for h, crc in _golden_headers():
        zeroed = bytes(h[:4]) + bytes(4) + bytes(h[8:12]) + bytes(8) + bytes(h[20:])
        assert _oracle_crc(zeroed) == crc                     # oracle pinned to the reference
        assert nd.header_crc(h) == crc                        # product host path
        assert nd.header_verify(h)
        g = bytearray(h)
        g[16:20] = b"\0\0\0\0"
        nd.header_seal(g)
        assert g == h                                         # seal writes the same crc


def test_header_verify_rules():
    h, _ = _golden_headers()[3]
    g = bytearray(h)
    g[4:8] = struct.pack("<i", 12345)                         # disk_header_size: ignored
    g[12:16] = struct.pack("<I", 0x10000000)                  # flag (COMPRESSED): ignored
    assert nd.header_verify(g)
    for pos in (0, 20, len(h) - 1):                           # anything else is covered
        g = bytearray(h)
        g[pos] ^= 0x40
        assert not nd.header_verify(g), pos
    g = bytearray(h)
    struct.pack_into("<i", g, 8, len(h) - 1)                  # header_size covered too
    assert not nd.header_verify(g)
    g[9] ^= 0x40                                              # a size past the buffer: refused
    with pytest.raises(ValueError):                           # before C reads past it
        nd.header_verify(g)
    g = bytearray(h)
    g[16] ^= 1                                                # stored crc itself
    assert not nd.header_verify(g)
    assert nd.header_crc(bytearray(h) + b"trailing") == nd.header_crc(h)   # only header_size bytes


def _small_header(hs, seed=5):
    """A V30 header whose header_size field reads hs, with random other
    fields and a body after the fixed part."""
    rng = np.random.default_rng(seed + (hs & 0xFFFF))
    return bytearray(struct.pack("<IiiII", nd.NC_MAGIC_V30, int(rng.integers(0, 1 << 30)), hs,
                                 int(rng.integers(0, 2)) << 28, int(rng.integers(0, 1 << 32)))
                     + gen.xorshift_bytes(64, seed=seed))


def test_header_size_below_fixed_part_follows_the_reference():
    """dm_verify_header (diskcache.c:3676-3686) CRCs header_size bytes with no
    lower bound: for 0 <= header_size < 20 the CRC covers only the first
    header_size bytes of the fixed part, with disk_header_size, flag and crc
    zeroed wherever they fall inside them (header_size 0: crc32_8bytes of
    nothing, 0 -- so a header with a zero crc field verifies).  The CRC of
    those bytes is the oracle's (pinned to crc32.c); the zeroing rule itself
    is restated from diskcache.c, which cannot be built here (it needs
    autoconf's generated config.h): parity unpinned for that rule.  Only a
    negative header_size is refused -- the reference would hand it to
    crc32_8bytes as a huge size_t and read far past the header."""
    for hs in (19, 18, 17, 16, 13, 12, 11, 9, 8, 5, 4, 3, 1, 0):
        g = _small_header(hs)
        z = bytearray(g[:20])
        z[4:8] = bytes(4)
        z[12:20] = bytes(8)
        want = _oracle_crc(bytes(z[:hs]))
        assert nd.header_crc(g) == want, hs
        assert nd.header_verify(g) == (want == struct.unpack_from("<I", g, 16)[0]), hs
        nd.header_seal(g)
        assert struct.unpack_from("<I", g, 16)[0] == want and nd.header_verify(g), hs
        g[24] ^= 0x55                                          # past header_size: not covered
        assert nd.header_verify(g), hs
        for pos in (0, 3):                                     # magic: dm_check_magic fails first
            b = bytearray(g)
            b[pos] ^= 0x01
            assert not nd.header_verify(b), (hs, pos)
        if hs > 8:                                             # header_size's own bytes are covered
            b = bytearray(g)
            b[8] ^= 0x01                                       # hs +- 1: other bytes, other CRC
            assert not nd.header_verify(b), hs
        for pos in [p for p in (4, 7, 12, 15) if p < 20]:      # zeroed fields: never covered
            b = bytearray(g)
            b[pos] ^= 0x80
            assert nd.header_verify(b), (hs, pos)
    z = _small_header(0)
    z[16:20] = bytes(4)
    assert nd.header_crc(z) == 0 and nd.header_verify(z)        # crc field 0 == CRC of nothing
    for hs in (-1, -20, -(1 << 31)):
        g = _small_header(hs)
        assert not nd.header_verify(g) and nd.header_crc(g) == 0, hs
        with pytest.raises(m.MD5HipError):
            nd.header_seal(g)
    with pytest.raises(ValueError):
        nd.header_verify(bytes(19))                            # the fixed part is 20 B
    with pytest.raises(ValueError):
        nd.header_verify(_small_header(200))                   # header_size past the buffer


def test_host_crc32_matches_reference_vectors():
    for k in GOLD["kat"]:
        assert "%08x" % nd.crc32(bytes.fromhex(k["hex"])) == k["crc"]
    big = gen.mul_pattern(1 << 20)
    for L, c in zip(GOLD["edge"]["lengths"], GOLD["edge"]["crc"]):
        assert "%08x" % nd.crc32(big[:L]) == c


def test_digest_array_bounds_and_layout():
    for bl in (0, 1, 2, 3, 255, 65535):
        assert nd.canned_digest_size(bl, 4) == (bl * 4 + 7) // 8 * 8     # NC_CANNED_CRC_SIZE
        assert nd.canned_digest_size(bl, 16) == bl * 16
    a = nd.DigestArray(5, dsz=4)
    assert a.buf.size == 24
    for b in range(5):
        assert a.update(b, struct.pack("<I", 0xA0 + b), mapped=5) == 0
    assert a.update(5, b"\1\2\3\4", mapped=5) == -errno.ERANGE           # extent check
    assert a.update(5, b"\1\2\3\4", mapped=6) == 0                       # slack of align8
    assert a.update(6, b"\1\2\3\4", mapped=9) == -errno.E2BIG            # crcsize check
    assert list(np.frombuffer(a.buf[:20].tobytes(), "<u4")) == [0xA0, 0xA1, 0xA2, 0xA3, 0xA4]
    assert a.verify(2, struct.pack("<I", 0xA2)) == 1
    assert a.verify(2, struct.pack("<I", 0xA3)) == 0
    assert a.verify(6, b"\0\0\0\0") == -errno.ERANGE
    md = nd.DigestArray(3, dsz=16)
    assert md.update(2, bytes(range(16)), mapped=3) == 0 and md.buf[32:48].tolist() == list(range(16))
    assert md.update(3, bytes(16), mapped=4) == -errno.E2BIG


def test_digest_array_batched():
    rng = np.random.default_rng(3)
    n = 1000
    arr = nd.DigestArray(n, dsz=16)
    dig = rng.integers(0, 256, (n, 16), dtype=np.uint8)
    perm = rng.permutation(n).astype(np.uint64)
    assert arr.scatter(perm, dig[perm], mapped=n) == 0
    assert np.array_equal(arr.buf.reshape(n, 16), dig)
    bad = dig.copy()
    bad[[1, 500]] ^= 0x80
    ok, nbad = arr.compare(np.arange(n), bad)
    assert nbad == 2 and not ok[1] and not ok[500]
    assert arr.scatter(np.array([n - 1, n, n + 5]), dig[:3], mapped=n + 1) == 2   # n: E2BIG, n+5: ERANGE


@pytest.mark.gpu
def test_gpu_batch_verify_headers(cuda):
    """dm_verify_header for a batch of headers through a batcher (CRC-32 over
    the gathered, field-zeroed header bytes on the GPU), with corrupted,
    wrong-magic, negative-size and 0..20-byte header_size headers (the
    reference's partial-fixed-part rule) mixed in; the batcher keeps its mode."""
    rng = np.random.default_rng(8)
    heads = [bytearray(h) for h, _ in _golden_headers()]
    for k in range(300):
        hs = int(rng.integers(20, 300000)) if k % 10 else int(rng.integers(20, 64))
        h = bytearray(struct.pack("<IiiII", nd.NC_MAGIC_V30, int(rng.integers(0, 1 << 30)), hs,
                                  int(rng.integers(0, 2)) << 28, 0) + gen.xorshift_bytes(hs - 20, seed=k))
        nd.header_seal(h)
        h[4:8] = struct.pack("<i", hs // 2)                 # written after the crc, as on disk
        heads.append(h)
    want = np.ones(len(heads), bool)
    for i in (9, 40, 77):
        heads[i][int(rng.integers(20, len(heads[i])))] ^= 0x01; want[i] = False
    heads[100][0] ^= 0xFF; want[100] = False                # bad magic
    heads[150][8:12] = struct.pack("<i", 3); want[150] = False   # CRC of 3 bytes != the stored one
    for hs in (0, 1, 4, 5, 12, 13, 19, 20):                 # the reference's small-size rule, sealed
        h = _small_header(hs, seed=9)
        nd.header_seal(h)
        h[4:8] = struct.pack("<i", 77)
        heads.append(h)
        want = np.append(want, True)
    heads.append(_small_header(-5)); want = np.append(want, False)
    assert [nd.header_verify(h) for h in heads] == want.tolist()
    with m.Batcher(device=0, slice_bytes=2 << 20, nslots=3) as b:
        ok, nbad = nd.verify_headers(b, heads)
        assert nbad == (~want).sum() and np.array_equal(ok, want)
        bufs = [bytes(h) for h in heads[:20]]              # still MD5 afterwards
        blob = b"".join(bufs) + b"\0"
        lens = [len(x) for x in bufs]
        want_md5 = gen.oracle_digests(np.frombuffer(blob, np.uint8), np.cumsum([0] + lens[:-1]), lens)
        assert np.array_equal(b.submit(bufs), want_md5)


def test_header_layout_against_reference_probe():
    """include/nc_digest.h's header offsets, magic and canned-array size
    against the reference netcache.h compiled as is
    (oracle/nc_header_probe.c with the image's libuuid 1.0.3 header;
    tests/golden/make_nc_layout.py wrote the fixture).  When the probe builds
    here, its live output must equal the committed fixture too."""
    import re
    lay = json.load(open(os.path.join(gen.REPO, "tests", "golden", "nc_header_layout.json")))
    live = os.path.join(gen.REPO, "oracle", "_ref", "nc_header_layout.json")
    if os.path.exists(live):
        got = json.load(open(live))
        assert all(lay[k] == v for k, v in got.items()), got
    hdr = open(os.path.join(gen.REPO, "include", "nc_digest.h")).read()
    off = {k: int(v) for k, v in re.findall(r"#define NC_HDR_OFF_(\w+) (\d+)", hdr)}
    assert off["MAGIC"] == lay["magic"] and off["DISK_HEADER_SIZE"] == lay["disk_header_size"]
    assert off["HEADER_SIZE"] == lay["header_size"] and off["FLAG"] == lay["flag"]
    assert off["CRC"] == lay["crc"] and lay["sizeof_nc_crc_t"] == 4
    assert lay["sizeof_fc_common_header_t"] == 16 and lay["block_size"] == off["CRC"] + 4
    assert nd.HDR_MIN_SIZE == lay["crc"] + lay["sizeof_nc_crc_t"]
    assert nd.NC_MAGIC_V30 == lay["NC_MAGIC_V30"]
    for bl, size in lay["NC_CANNED_CRC_SIZE"]:
        assert nd.canned_digest_size(bl, 4) == size, bl
