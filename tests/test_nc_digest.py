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
    for pos in (0, 9, 20, len(h) - 1):                        # anything else is covered
        g = bytearray(h)
        g[pos] ^= 0x40
        assert not nd.header_verify(g), pos
    g = bytearray(h)
    g[16] ^= 1                                                # stored crc itself
    assert not nd.header_verify(g)
    assert nd.header_crc(bytearray(h) + b"trailing") == nd.header_crc(h)   # only header_size bytes


def test_header_size_below_fixed_part_is_a_deliberate_divergence():
    """DELIBERATE DIVERGENCE from the reference (DESIGN.md
    §9): dm_verify_header (diskcache.c:3676-3689) CRCs header_size bytes with
    no lower bound -- for 0 <= header_size < 20 a CRC over only part of the
    fixed header (the zeroed crc / disk_header_size / flag fields partly
    outside it), and for a negative header_size a length the reference never
    guards.  Here a header whose header_size is below the 20-byte fixed part
    (or negative) is rejected: header_verify false, header_crc 0, seal
    -EINVAL.  Not parity: a corrupt size field is refused, not hashed."""
    h, _ = _golden_headers()[3]
    for hs in (19, 4, 0, -1, -(1 << 31)):
        g = bytearray(h)
        g[8:12] = struct.pack("<i", hs)
        assert not nd.header_verify(g) and nd.header_crc(g) == 0, hs


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
    wrong-magic and undersized headers mixed in; the batcher keeps its mode."""
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
    heads[150][8:12] = struct.pack("<i", 3); want[150] = False
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
