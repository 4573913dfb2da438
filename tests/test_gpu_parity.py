"""GPU parity: the HIP kernels of libmd5hip.so against the oracle and the
golden vectors (produced by the reference md5.c).  Bit-exact, every case.

Small sizes are compared digest by digest; at BASELINE.json's full size
(1,048,576 x 16 KiB, 16 GiB) the properties are (a) a sampled subset of
>= 4096 chunks, first and last included, re-digested by the oracle and
(b) every kernel variant producing the identical 16 MiB digest array
(checksum of checksums).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

import gen
from sproxy_amd import md5 as m

pytestmark = pytest.mark.gpu

FIXED_VARIANTS = [v for v in m.VARIANTS if v != "auto"]


def _dev(a, cuda):
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


@pytest.mark.parametrize("variant", FIXED_VARIANTS)
def test_fixed_golden_batches(golden, cuda, variant):
    for b in golden["batches"]:
        n, L = b["n"], b["len"]
        host = gen.xorshift_array(max(n * L, 16))
        d = _dev(host, cuda)
        got = m.digest_fixed(d, n, L, variant=variant).cpu().numpy()
        assert "%08x" % gen.fold(got.tobytes()) == b["fold"], (variant, n, L)
        if "md5" in b:
            assert [bytes(x).hex() for x in got] == b["md5"], (variant, n, L)


@pytest.mark.parametrize("variant", FIXED_VARIANTS)
def test_fixed_edge_lengths(golden, cuda, variant):
    """Every golden edge length as a fixed-length batch of the same message
    repeated at a 16-B-aligned stride (ragged tails, 55/56/63/64-byte
    padding boundaries, 1 MiB -- every variant, the product C2 kernel
    xdma1nt included)."""
    e = golden["edge"]
    big = np.frombuffer(gen.mul_pattern(max(e["lengths"])), dtype=np.uint8)
    assert max(e["lengths"]) >= 1 << 20
    for L, want in zip(e["lengths"], e["md5"]):
        stride = max(16, (L + 15) // 16 * 16)
        n = 130                                  # > 2 waves, ragged last wave
        host = np.zeros(n * stride, dtype=np.uint8)
        for i in range(n):
            host[i * stride:i * stride + L] = big[:L]
        got = m.digest_fixed(_dev(host, cuda), n, L, stride, variant=variant).cpu().numpy()
        assert all(bytes(x).hex() == want for x in got), (variant, L)


DESC = [v for v in m.DESC_VARIANTS if v != "auto"]


@pytest.mark.parametrize("dv", DESC)
def test_kat_through_desc(golden, cuda, dv):
    """All KAT messages packed at odd offsets into one descriptor batch."""
    msgs = [bytes.fromhex(v["hex"]) for v in golden["kat"]]
    offs, cur, parts = [], 3, [b"\xAA" * 3]
    for msg in msgs:
        offs.append(cur)
        parts.append(msg + b"\x55" * 5)
        cur += len(msg) + 5
    buf = np.frombuffer(b"".join(parts) + b"\0" * 64, dtype=np.uint8)
    lens = [len(x) for x in msgs]
    got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                        torch.tensor(lens, dtype=torch.int32, device=cuda), variant=dv).cpu().numpy()
    assert [bytes(x).hex() for x in got] == [v["md5"] for v in golden["kat"]]


@pytest.mark.parametrize("dv", DESC)
def test_mixed_golden(golden, cuda, dv):
    mx = golden["mixed"]
    lens, offs = mx["lengths"], mx["offsets"]
    total = gen.pack_offsets(lens, align=mx["align"])[1]
    buf = gen.xorshift_array(total, seed=int(mx["data_seed"], 16))
    order = m.plan_order(lens).astype(np.int32)
    for o in (None, _dev(order, cuda)):
        got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                            torch.tensor(lens, dtype=torch.int32, device=cuda), o,
                            variant=dv).cpu().numpy()
        assert [bytes(x).hex() for x in got] == mx["md5"]


@pytest.mark.parametrize("dv", DESC)
@pytest.mark.parametrize("align", [1, 4, 16])
def test_desc_random_vs_oracle(cuda, align, dv):
    lens = gen.mixed_lengths(700, seed=11 + align, max_len=1 << 17)
    lens += [0, 1, 55, 56, 63, 64, 65, 119, 120, 127, 128]
    offs, total = gen.pack_offsets(lens, align=align)
    buf = gen.xorshift_array(total + 64, seed=77)
    want = gen.oracle_digests(buf, offs, lens)
    order = m.plan_order(lens).astype(np.int32)
    got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                        torch.tensor(lens, dtype=torch.int32, device=cuda),
                        _dev(order, cuda), variant=dv).cpu().numpy()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("dv", DESC)
def test_desc_netcache_blocks(cuda, dv):
    """The netcache shape the xpose descriptor kernel is built for: mostly
    full chunk_size blocks plus ragged last blocks, 16-B aligned, packed in an
    arena, ordered longest-first or not at all; plus waves whose chunks are
    all shorter than one 128-B stage, a ragged last wave, and one unaligned
    chunk that sends its wave down the lane-direct path."""
    rng = np.random.default_rng(4242)
    for S in (4096, 65536):
        n = 1000
        lens = np.full(n, S, dtype=np.int64)
        tail = rng.integers(0, 8, n) == 0
        lens[tail] = rng.integers(0, S, int(tail.sum()))
        lens[-70:] = rng.integers(0, 128, 70)          # a whole wave without any stage
        lens = [int(x) for x in lens]
        for align in (16, 4):
            offs, total = gen.pack_offsets(lens, align=align)
            if align == 4:                             # only chunk 500 unaligned
                offs = list(gen.pack_offsets(lens, align=16)[0])
                offs[500] += 4
                total = offs[-1] + lens[-1] + 64
            buf = gen.xorshift_array(total + 64, seed=S + align)
            want = gen.oracle_digests(buf, offs, lens)
            for order in (m.plan_order(lens).astype(np.int32), None):
                got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                                    torch.tensor(lens, dtype=torch.int32, device=cuda),
                                    None if order is None else _dev(order, cuda), variant=dv).cpu().numpy()
                assert np.array_equal(got, want), (S, align, order is None)


@pytest.mark.parametrize("dv", DESC)
def test_desc_long_and_short_waves(cuda, dv):
    """Waves whose longest chunk is >= 256 KiB (HYBRID sends the first of
    them lane-direct) beside short-chunk waves, longest-first and unordered."""
    rng = np.random.default_rng(99)
    lens = ([1 << 20] * 70 + [256 << 10] * 40 + [int(x) for x in rng.integers(1, 1 << 19, 30)]
            + [int(x) for x in rng.integers(0, 8192, 200)])
    offs, total = gen.pack_offsets(lens, align=16)
    buf = gen.xorshift_array(total + 64, seed=991)
    want = gen.oracle_digests(buf, offs, lens)
    for order in (m.plan_order(lens).astype(np.int32), None):
        got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                            torch.tensor(lens, dtype=torch.int32, device=cuda),
                            None if order is None else _dev(order, cuda), variant=dv).cpu().numpy()
        assert np.array_equal(got, want), order is None


def test_balanced_guard_free_stage_edges(cuda):
    """BALANCED's guard-free stages (md5_kernels.h, desc_xpose_group NB = 2:
    stages every live lane holds whole and no row clamps, four per loop test)
    hand over to the guarded stage at every boundary: 64-chunk groups of one
    length with 1..21 whole 128-B stages and each of 0 / 64 / 100 B more; the
    same groups with one lane of no stage, one lane a stage short, one lane
    much longer; 16-B-aligned (off-line) and line-aligned packing; a ragged
    last group.  Longest-first and unordered, against the oracle."""
    rng = np.random.default_rng(5150)
    lens = []
    for k in range(1, 22):
        for extra in (0, 64, 100):
            g = [128 * k + extra] * 64
            lens += g
            h = list(g)
            h[int(rng.integers(0, 64))] = int(rng.integers(0, 128))        # a lane with no stage
            lens += h
            h = list(g)
            h[int(rng.integers(0, 64))] = max(0, 128 * (k - 1) + extra)   # a stage short
            lens += h
            h = list(g)
            h[int(rng.integers(0, 64))] = 128 * (k + 9) + 17               # one much longer
            lens += h
    lens += [128 * 7 + 3] * 37                                            # ragged last group
    for align in (16, 128):
        offs, total = gen.pack_offsets(lens, align=align)
        buf = gen.xorshift_array(total + 64, seed=align + 5150)
        want = gen.oracle_digests(buf, offs, lens)
        for order in (None, m.plan_order(lens).astype(np.int32)):
            got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                                torch.tensor(lens, dtype=torch.int32, device=cuda),
                                None if order is None else _dev(order, cuda), variant="balanced").cpu().numpy()
            assert np.array_equal(got, want), (align, order is None)


def test_hybrid_long_group_edges(cuda):
    """HYBRID's long groups (longest chunk >= 256 KiB, one per CU, run
    lane-direct): long chunks at every residue mod 64 and 128 beside lanes
    with no whole block, a lone partial group, twenty full long groups, and a
    group with one unaligned start."""
    rng = np.random.default_rng(4242)
    K = 4096 * 64                                       # 256 KiB: HYBRID's long threshold
    cases = {
        "residues": [K + r for r in (0, 1, 55, 56, 63, 64, 65, 127, 128, 129)] +
                    [int(x) for x in rng.integers(K, 3 * K, 40)] + [0, 1, 63, 64, 100, 4096] +
                    [int(x) for x in rng.integers(0, 64, 8)],
        "lone_partial": [K + 77] * 3 + [5, 0],
        "twenty_groups": [int(x) for x in rng.integers(K, K + 4000, 64 * 20)],
    }
    for name, lens in cases.items():
        offs, total = gen.pack_offsets(lens, align=16)
        buf = gen.xorshift_array(total + 64, seed=len(lens))
        want = gen.oracle_digests(buf, offs, lens)
        order = m.plan_order(lens).astype(np.int32)
        got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                            torch.tensor(lens, dtype=torch.int32, device=cuda), _dev(order, cuda),
                            variant="hybrid").cpu().numpy()
        assert np.array_equal(got, want), name
    # one chunk start off 16 B inside the first (long) group
    lens = [K + 5] * 20 + [300] * 30
    offs, total = gen.pack_offsets(lens, align=16)
    offs = list(offs)
    offs[3] += 4
    buf = gen.xorshift_array(total + 64, seed=77)
    want = gen.oracle_digests(buf, offs, lens)
    got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                        torch.tensor(lens, dtype=torch.int32, device=cuda),
                        _dev(m.plan_order(lens).astype(np.int32), cuda), variant="hybrid").cpu().numpy()
    assert np.array_equal(got, want)


def test_fed_group_edges(cuda):
    """FED (chain wave + feeder wave per group, md5_desc_fed): groups whose
    lanes end at every residue mod 64 around the longest chunk (lanes past
    their own last block discard the feeder's clamped addends), lanes with no
    whole block, exactly two blocks (the smallest fed group), a ragged last
    group, a group of chunks under 128 B (LANE fallback), one unaligned start
    (LANE fallback for its group only), ordered and unordered, and the
    planner's own choice for a netcache vector."""
    rng = np.random.default_rng(606)
    cases = {
        "residues": [16384 + r for r in (0, 1, 55, 56, 63, 64, 65, 127, 128, 129)] +
                    [int(x) for x in rng.integers(1, 40000, 50)] + [0, 1, 63, 64, 100, 128],
        "two_blocks": [128] * 10 + [127, 64, 0, 5],
        "ragged": [int(x) for x in rng.integers(0, 70000, 64 * 5 + 7)],
        "short_group": [int(x) for x in rng.integers(0, 128, 64)] + [4096] * 64,
        "long": [(1 << 20) + 13] * 3 + [int(x) for x in rng.integers(0, 1 << 18, 100)],
    }
    for name, lens in cases.items():
        offs, total = gen.pack_offsets(lens, align=16)
        buf = gen.xorshift_array(total + 64, seed=len(lens) + 7)
        want = gen.oracle_digests(buf, offs, lens)
        for order in (m.plan_order(lens).astype(np.int32), None):
            got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                                torch.tensor(lens, dtype=torch.int32, device=cuda),
                                None if order is None else _dev(order, cuda), variant="fed").cpu().numpy()
            assert np.array_equal(got, want), (name, order is None)
    # one start off 16 B: its group goes LANE, the other groups stay fed
    lens = [16384] * 200
    offs = list(gen.pack_offsets(lens, align=16)[0])
    offs[70] += 4
    buf = gen.xorshift_array(offs[-1] + 16384 + 64, seed=70)
    want = gen.oracle_digests(buf, offs, lens)
    got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                        torch.tensor(lens, dtype=torch.int32, device=cuda), variant="fed").cpu().numpy()
    assert np.array_equal(got, want)
    # the planner's choice for a netcache vector is FED, through the default entry
    order, v = m.plan_desc(np.asarray(lens, np.uint32))
    assert v == "fed"
    got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                        torch.tensor(lens, dtype=torch.int32, device=cuda),
                        _dev(order.astype(np.int32), cuda), variant=v).cpu().numpy()
    assert np.array_equal(got, want)


@pytest.mark.parametrize("dv", DESC)
def test_desc_offsets_beyond_4gib(cuda, dv):
    """Descriptor offsets past 2^32 (64-bit row pointers): chunks scattered
    over a 5 GiB arena, half of them above 4 GiB, one wave straddling."""
    arena = torch.empty(5 << 30, dtype=torch.uint8, device=cuda)
    m.fill_synthetic(arena, seed=0x4646)
    rng = np.random.default_rng(46)
    n = 200
    lens = [int(x) for x in rng.integers(0, 70000, n)]
    lo = rng.integers(0, (4 << 30) // 16 - 8192, n // 2) * 16
    hi = rng.integers((4 << 30) // 16, (5 << 30) // 16 - 8192, n - n // 2) * 16
    offs = np.concatenate([lo, hi]).astype(np.int64)
    rng.shuffle(offs)
    want = np.empty((n, 16), dtype=np.uint8)
    for i in range(n):
        chunk = arena[int(offs[i]):int(offs[i]) + lens[i]].cpu().numpy()
        want[i] = gen.oracle_digests(chunk, [0], [lens[i]])[0] if lens[i] else \
            np.frombuffer(bytes.fromhex("d41d8cd98f00b204e9800998ecf8427e"), dtype=np.uint8)
    order = m.plan_order(lens).astype(np.int32)
    got = m.digest_desc(arena, torch.from_numpy(offs).to(cuda),
                        torch.tensor(lens, dtype=torch.int32, device=cuda), _dev(order, cuda),
                        variant=dv).cpu().numpy()
    assert np.array_equal(got, want)
    del arena
    torch.cuda.empty_cache()


def test_unaligned_fixed_falls_back_bit_exact(cuda):
    n, L = 300, 1000
    host = gen.xorshift_array(n * L + 8, seed=9)
    d = _dev(host, cuda)
    want = gen.oracle_digests_fixed(host[3:], n, L)
    got = m.digest_fixed(d[3:], n, L).cpu().numpy()        # base 3 bytes off alignment
    assert np.array_equal(got, want)
    want2 = gen.oracle_digests(host, [i * 1001 for i in range(n - 1)], [L] * (n - 1))
    got2 = m.digest_fixed(d, n - 1, L, 1001).cpu().numpy()  # odd stride
    assert np.array_equal(got2, want2)


def test_c1_fold_on_gpu(cuda):
    """The 1 GiB C1 set (65,536 x 16 KiB xorshift64) -> fold 53a0a616."""
    n, L = 65536, 16384
    d = _dev(gen.xorshift_array(n * L), cuda)
    for v in FIXED_VARIANTS:
        got = m.digest_fixed(d, n, L, variant=v).cpu().numpy()
        assert "%08x" % gen.fold(got.tobytes()) == "53a0a616", v
    del d
    torch.cuda.empty_cache()


def test_full_size_c2(cuda):
    """BASELINE config: 1,048,576 x 16 KiB = 16 GiB device-resident."""
    n, L = 1 << 20, 16384
    d = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    m.fill_synthetic(d, seed=0xC2)
    ref = m.digest_fixed(d, n, L, variant="direct2")
    for v in FIXED_VARIANTS[1:]:
        assert torch.equal(m.digest_fixed(d, n, L, variant=v), ref), v
    rng = np.random.default_rng(2)
    idx = np.unique(np.concatenate([[0, 1, n - 2, n - 1], rng.integers(0, n, 4096)]))
    rows = d.view(n, L)[torch.from_numpy(idx).to(cuda)].cpu().numpy()
    want = gen.oracle_digests_fixed(rows, idx.size, L)
    assert np.array_equal(ref[torch.from_numpy(idx).to(cuda)].cpu().numpy(), want)
    del d
    torch.cuda.empty_cache()


def test_c4_shard_shape(cuda):
    """BASELINE config 4 on one device: 16,777,216 x 16 KiB split over 8 GPUs
    is 2,097,152 chunks (32 GiB) per rank (sproxy_amd.shard.shard_range).
    The last rank's shard, generated with bench.py's per-rank seed, hashed by
    the default kernel: sampled chunks against the oracle, and the digest of a
    chunk independent of where its shard starts (hash of a sub-batch = the
    same rows of the whole)."""
    from sproxy_amd.shard import shard_range
    lo, hi = shard_range(16 << 20, 7, 8)
    n, L = hi - lo, 16384
    assert n == 2 << 20
    d = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    m.fill_synthetic(d, seed=0x5EED0000 + 7)
    got = m.digest_fixed(d, n, L)
    rng = np.random.default_rng(4)
    idx = np.unique(np.concatenate([[0, n // 2, n - 1], rng.integers(0, n, 2048)]))
    rows = d.view(n, L)[torch.from_numpy(idx).to(cuda)].cpu().numpy()
    assert np.array_equal(got[torch.from_numpy(idx).to(cuda)].cpu().numpy(),
                          gen.oracle_digests_fixed(rows, idx.size, L))
    part = m.digest_fixed(d[(n // 2) * L:], n // 2, L)
    assert torch.equal(part, got[n // 2:])
    del d
    torch.cuda.empty_cache()


def test_fill_synthetic_matches_numpy_mirror(cuda):
    t = torch.empty(4096, dtype=torch.uint8, device=cuda)
    m.fill_synthetic(t, seed=123)
    assert np.array_equal(t.cpu().numpy(), gen.synthetic_bytes(4096, 123))


def test_streams_and_async(cuda):
    """Launch on a side stream; results visible after that stream syncs."""
    n, L = 2048, 4096
    host = gen.xorshift_array(n * L, seed=4)
    d = _dev(host, cuda)
    s = torch.cuda.Stream()
    out = torch.empty((n, 16), dtype=torch.uint8, device=cuda)
    with torch.cuda.stream(s):
        m.digest_fixed(d, n, L, out=out)
    s.synchronize()
    assert np.array_equal(out.cpu().numpy(), gen.oracle_digests_fixed(host, n, L))


def test_batcher_submit(cuda):
    lens = gen.mixed_lengths(500, seed=21, max_len=1 << 18) + [0, 1, 64]
    blob = gen.xorshift_bytes(sum(lens) + 1, seed=33)
    bufs, cur = [], 0
    for L in lens:
        bufs.append(blob[cur:cur + L])
        cur += L
    with m.Batcher(device=0, slice_bytes=4 << 20, nslots=3) as b:
        got = b.submit(bufs)
    offs = np.cumsum([0] + lens[:-1])
    want = gen.oracle_digests(np.frombuffer(blob, dtype=np.uint8), offs, lens)
    assert np.array_equal(got, want)


def test_batcher_async_pipeline(cuda):
    """md5_batch_submit_async / md5_batch_wait / md5_batch_poll: several
    submissions in flight on one batcher (more slices than slots, so later
    submits deliver earlier ones while reusing their slots), waited on out of
    order, mixed with synchronous calls and iov submissions; every digest
    array equals the oracle."""
    rng = np.random.default_rng(5150)
    batches = []
    for k in range(6):
        lens = [int(x) for x in rng.integers(0, 300000, 40)]
        blob = gen.xorshift_bytes(sum(lens) + 1, seed=600 + k)
        bufs, cur = [], 0
        for L in lens:
            bufs.append(blob[cur:cur + L])
            cur += L
        offs = np.cumsum([0] + lens[:-1])
        batches.append((bufs, gen.oracle_digests(np.frombuffer(blob, dtype=np.uint8), offs, lens)))
    with m.Batcher(device=0, slice_bytes=2 << 20, nslots=3) as b:
        pend = [b.submit_async(bufs) for bufs, _ in batches[:4]]
        assert np.array_equal(b.submit(batches[4][0]), batches[4][1])     # sync in between
        pend.append(b.submit_iov_async([[x[:7], x[7:]] for x in batches[5][0]]))
        for j in (2, 0, 5, 1, 3, 4):                                      # out of order
            if j == 4:
                continue
            p = pend[j if j < 4 else 4]
            got = p.wait()
            assert np.array_equal(got, batches[j][1]), j
        assert all(p.poll() for p in pend)
        empty = b.submit_async([])
        assert empty.poll() and empty.wait().shape[0] == 0


def test_batcher_host_fixed(cuda):
    n, L = 5000, 16384
    host = gen.xorshift_array(n * L, seed=8)
    with m.Batcher(device=0, slice_bytes=16 << 20, nslots=3) as b:
        got = b.host_fixed(host, n, L)
    assert np.array_equal(got, gen.oracle_digests_fixed(host, n, L))


def test_batcher_submit_iov_pages(cuda):
    """netcache-style blocks: each block a list of 16 KiB pages plus a ragged
    last page (blk->pages[i]->memory, block.h:143-146); digests over the
    concatenated bytes, compared with the oracle on the joined buffer."""
    rng = np.random.default_rng(12)
    page = 16384
    blocks, joined = [], []
    for b in range(40):
        npages = int(rng.integers(1, 9))
        tail = int(rng.integers(0, page + 1))
        pages = [gen.xorshift_bytes(page, seed=1000 * b + p) for p in range(npages - 1)]
        pages.append(gen.xorshift_bytes(tail, seed=1000 * b + 999))
        blocks.append(pages)
        joined.append(b"".join(pages))
    blocks.append([])                       # empty block
    joined.append(b"")
    with m.Batcher(device=0, slice_bytes=1 << 20, nslots=2) as bt:
        got = bt.submit_iov(blocks)
    blob = b"".join(joined)
    offs = np.cumsum([0] + [len(j) for j in joined[:-1]])
    want = gen.oracle_digests(np.frombuffer(blob + b"\0", dtype=np.uint8), offs, [len(j) for j in joined])
    assert np.array_equal(got, want)


def test_batcher_threaded_host_gather(cuda):
    """Slices of >= 8 MiB are gathered into pinned staging on several threads
    (MD5HIP_GATHER_THREADS, default 4), each copying a byte range of the
    slice's chunks: page-list blocks of mixed sizes (ragged last pages, empty
    blocks) and flat buffers over 24 MiB slices, MD5 and CRC-32, against the
    oracle."""
    rng = np.random.default_rng(31)
    page = 16384
    heap = gen.xorshift_array(6000 * page, seed=4242)
    perm = rng.permutation(6000)
    blocks, joined, k = [], [], 0
    while k < 5800:
        npages = int(rng.integers(1, 65))
        tail = int(rng.integers(0, page + 1)) if rng.integers(0, 4) == 0 else page
        ids = perm[k:k + npages]
        k += npages
        pages = [heap[i * page:(i + 1) * page] for i in ids[:-1]]
        pages.append(heap[ids[-1] * page:ids[-1] * page + tail])
        if rng.integers(0, 50) == 0:
            pages = []
        blocks.append(pages)
        joined.append(b"".join(p.tobytes() for p in pages))
    blob = b"".join(joined) + b"\0"
    offs = np.cumsum([0] + [len(j) for j in joined[:-1]])
    lens = [len(j) for j in joined]
    want = gen.oracle_digests(np.frombuffer(blob, dtype=np.uint8), offs, lens)
    with m.Batcher(device=0, slice_bytes=24 << 20, nslots=3) as bt:
        assert np.array_equal(bt.submit_iov(blocks), want)
        assert np.array_equal(bt.submit(joined), want)
        bt.set_digest(m.Batcher.CRC32, 0)
        crcs = bt.submit(joined).view("<u4").ravel()
    want_crc = gen.oracle_crc32_batch(np.frombuffer(blob, dtype=np.uint8), offs, lens)
    assert np.array_equal(crcs, want_crc)


def test_batcher_crc32_and_verify(cuda):
    """The block-checksum call site end to end: a batcher in netcache CRC-32
    mode (fastcrc window) and the batched verify with a corrupted block."""
    rng = np.random.default_rng(77)
    page = 16384
    blocks, joined = [], []
    for b in range(30):
        pages = [gen.xorshift_bytes(page, seed=500 + 10 * b + p) for p in range(int(rng.integers(1, 5)))]
        pages[-1] = pages[-1][:int(rng.integers(1, page + 1))]
        blocks.append(pages)
        joined.append(b"".join(pages))
    blob = b"".join(joined)
    offs = np.cumsum([0] + [len(j) for j in joined[:-1]])
    lens = [len(j) for j in joined]
    arena = np.frombuffer(blob + b"\0", dtype=np.uint8)
    for fast in (0, 128):
        with m.Batcher(device=0, slice_bytes=1 << 20, nslots=2, kind=m.Batcher.CRC32, fastcrc=fast) as bt:
            got = bt.submit_iov(blocks)
            assert np.array_equal(got, gen.oracle_crc32_batch(arena, offs, lens, fast))
            ok, bad = bt.verify_iov(blocks, got)
            assert bad == 0 and ok.all()
            exp = got.copy()
            exp[7] ^= 1
            ok, bad = bt.verify_iov(blocks, exp)
            assert bad == 1 and not ok[7] and ok.sum() == len(blocks) - 1
    with m.Batcher(device=0, slice_bytes=1 << 20, nslots=2) as bt:       # MD5 verify
        dig = bt.submit_iov(blocks)
        assert np.array_equal(dig, gen.oracle_digests(arena, offs, lens))
        dig[3, 0] ^= 0xFF
        ok, bad = bt.verify_iov(blocks, dig)
        assert bad == 1 and not ok[3]


@pytest.mark.gpu
def test_pool_matches_oracle(cuda):
    """Multi-GPU host pool (§8e) on the one device of the box, listed 1-3
    times: each entry is a separate batcher driven by its own host thread, so
    the split, per-thread device binding and digest placement are exercised."""
    lens = gen.mixed_lengths(700, seed=91, max_len=1 << 18) + [0, 1, 64, 16384]
    blob = gen.xorshift_bytes(sum(lens) + 1, seed=92)
    bufs, cur = [], 0
    for L in lens:
        bufs.append(blob[cur:cur + L])
        cur += L
    arena = np.frombuffer(blob, dtype=np.uint8)
    offs = np.cumsum([0] + lens[:-1])
    want = gen.oracle_digests(arena, offs, lens)
    n, L = 3000, 16384
    host = gen.xorshift_array(n * L, seed=93)
    want_fixed = gen.oracle_digests_fixed(host, n, L)
    pages = [[bufs[i][:7000], bufs[i][7000:]] for i in range(len(bufs))]
    for devs in ((0,), (0, 0), (0, 0, 0)):
        with m.Pool(devs, slice_bytes=2 << 20, nslots=2) as p:
            assert p.ndev == len(devs)
            assert np.array_equal(p.submit(bufs), want)
            assert np.array_equal(p.submit_iov(pages), want)
            assert np.array_equal(p.host_fixed(host, n, L), want_fixed)
            bad = want.copy()
            bad[[5, 600]] ^= 1
            ok, nbad = p.verify_iov(pages, bad)
            assert nbad == 2 and not ok[5] and not ok[600]
            p.set_digest(m.Pool.CRC32, 64)
            assert np.array_equal(p.submit(bufs), gen.oracle_crc32_batch(arena, offs, lens, 64))


@pytest.mark.parametrize("variant", FIXED_VARIANTS)
def test_fixed_ragged_counts_and_empty_chunks(cuda, variant):
    """n not a multiple of the wave (64) or workgroup (256), n = 1, and
    zero-length chunks (digest of the empty message, md5.c:221-265)."""
    L = 4160                                       # 65 blocks: odd block count, no tail
    host = gen.xorshift_array(4100 * L, seed=61)
    d = _dev(host, cuda)
    for n in (1, 63, 65, 255, 257, 4097):
        got = m.digest_fixed(d, n, L, variant=variant).cpu().numpy()
        assert np.array_equal(got, gen.oracle_digests_fixed(host, n, L)), (variant, n)
    got = m.digest_fixed(d, 100, 0, 16, variant=variant).cpu().numpy()
    assert all(bytes(x).hex() == "d41d8cd98f00b204e9800998ecf8427e" for x in got)


def test_huge_stride_and_large_chunks(cuda):
    """A stride past the 32-bit buffer-offset range of the xpose/lds loaders
    (they fall back to the lane-direct kernel), and long chunks: 16 MiB each
    through the fixed entry and one 64 MiB chunk among small ones through the
    descriptor entry (MD5 and CRC-32)."""
    L, stride, n = 16384, 40 << 20, 5              # 40 MiB > 2^31 / 64
    host = np.zeros(n * stride, dtype=np.uint8)
    for i in range(n):
        host[i * stride:i * stride + L] = np.frombuffer(gen.xorshift_bytes(L, seed=70 + i), np.uint8)
    d = _dev(host, cuda)
    want = gen.oracle_digests(host, np.arange(n, dtype=np.uint64) * stride, [L] * n)
    for v in FIXED_VARIANTS:
        assert np.array_equal(m.digest_fixed(d, n, L, stride, variant=v).cpu().numpy(), want), v
    crc_want = gen.oracle_crc32_batch(host, np.arange(n, dtype=np.uint64) * stride, [L] * n)
    for v in m.CRC_VARIANTS:
        got = m.crc32_fixed(d, n, L, stride, variant=v).cpu().numpy().view(np.uint32)
        assert np.array_equal(got, crc_want), v
    del d
    nb, Lb = 4, 16 << 20
    big = gen.xorshift_array(nb * Lb, seed=71)
    db = _dev(big, cuda)
    assert np.array_equal(m.digest_fixed(db, nb, Lb).cpu().numpy(), gen.oracle_digests_fixed(big, nb, Lb))
    lens = [3, 64 << 20, 100, 0, 4097]
    offs, total = gen.pack_offsets(lens, align=16)
    arena = gen.xorshift_array(total + 64, seed=72)
    da = _dev(arena, cuda)
    t_off = torch.tensor(offs, dtype=torch.int64, device=cuda)
    t_len = torch.tensor(lens, dtype=torch.int32, device=cuda)
    for dv in DESC:
        got = m.digest_desc(da, t_off, t_len, variant=dv).cpu().numpy()
        assert np.array_equal(got, gen.oracle_digests(arena, offs, lens)), dv
    got = m.crc32_desc(da, t_off, t_len).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, gen.oracle_crc32_batch(arena, offs, lens))


def test_chunk_past_512mib_bit_count_high_word(cuda):
    """A chunk of 2^29 + 123 bytes: its bit count no longer fits 32 bits, so
    the length words of the final block carry bits[1] = 1 (md5.c:179-182,
    :258-259).  One lane hashes it as one 8.4 M-compression chain (~5 s),
    through the fixed entry (a stride this large takes the lane-direct
    kernel) and the descriptor entry at an odd offset."""
    L = (1 << 29) + 123
    buf = gen.xorshift_array(L + 64, seed=4099)
    want = gen.oracle_digests(buf, [0], [L])
    d = _dev(buf, cuda)
    assert np.array_equal(m.digest_fixed(d, 1, L, (L + 15) // 16 * 16).cpu().numpy(), want)
    want_odd = gen.oracle_digests(buf, [7], [L - 7])
    got = m.digest_desc(d, torch.tensor([7], dtype=torch.int64, device=cuda),
                        torch.tensor([L - 7], dtype=torch.int32, device=cuda)).cpu().numpy()
    assert np.array_equal(got, want_odd)


REF_LIB = os.path.join(gen.REPO, "oracle", "_ref", "libmd5_ref.so")


@pytest.mark.skipif(not os.path.exists(REF_LIB), reason="oracle/_ref not built")
def test_gpu_equals_reference_md5c_build(cuda):
    """North-star check without the restatement in between: the reference
    md5.c itself (compiled where it lies, oracle/_ref/libmd5_ref.so; it travels
    with the tree) digests the same inputs as the product kernels -- 1,000
    random-length chunks at random 16-B offsets (descriptor kernel) and 4,096
    x 16 KiB (fixed kernel, the C2 shape)."""
    ref = ctypes.CDLL(REF_LIB)
    rng = np.random.default_rng(20261016)

    def md5c(view):
        ctx = ctypes.create_string_buffer(88)
        ref.MD5Init(ctx)
        ref.MD5Update(ctx, ctypes.c_void_p(view.ctypes.data), ctypes.c_uint(view.size))
        out = (ctypes.c_ubyte * 16)()
        ref.MD5Final(out, ctx)
        return bytes(out)

    lens = [int(x) for x in rng.integers(0, 200000, 1000)]
    offs, total = gen.pack_offsets(lens, align=16)
    buf = gen.xorshift_array(total + 64, seed=606)
    want = [md5c(buf[o:o + L]) for o, L in zip(offs, lens)]
    got = m.digest_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                        torch.tensor(lens, dtype=torch.int32, device=cuda),
                        _dev(m.plan_order(lens).astype(np.int32), cuda)).cpu().numpy()
    assert [bytes(x) for x in got] == want
    n, L = 4096, 16384
    fx = gen.xorshift_array(n * L, seed=607)
    got = m.digest_fixed(_dev(fx, cuda), n, L).cpu().numpy()
    assert [bytes(x) for x in got] == [md5c(fx[i * L:(i + 1) * L]) for i in range(n)]


def test_arena_batches(cuda):
    """md5hip_arena_alloc: a 1 GiB-aligned device arena wrapped as a torch
    tensor (no copy); fixed, descriptor (every variant) and CRC batches over it
    equal the oracle; free / double free behave."""
    t = m.arena_empty(3 << 30)
    assert t.is_cuda and t.numel() == 3 << 30 and t.data_ptr() % (1 << 30) == 0
    m.fill_synthetic(t, seed=0xA7E)
    n, L = 4096, 65536
    host = t[:n * L].cpu().numpy()
    want = gen.oracle_digests_fixed(host, n, L)
    assert np.array_equal(m.digest_fixed(t, n, L).cpu().numpy(), want)
    lens = [int(x) for x in np.random.default_rng(3).integers(0, 1 << 21, 600)]
    offs, total = gen.pack_offsets(lens, align=16)
    arena = t[:total + 64].cpu().numpy()
    want = gen.oracle_digests(arena, offs, lens)
    order, v = m.plan_desc(lens)
    d_off = torch.tensor(offs, dtype=torch.int64, device=cuda)
    d_len = torch.tensor(lens, dtype=torch.int32, device=cuda)
    d_ord = _dev(order.astype(np.int32), cuda)
    for dv in DESC + [v]:
        assert np.array_equal(m.digest_desc(t, d_off, d_len, d_ord, variant=dv).cpu().numpy(), want), dv
    crc = m.crc32_desc(t, d_off, d_len, d_ord).cpu().numpy().view(np.uint32)
    assert np.array_equal(crc, gen.oracle_crc32_batch(arena, offs, lens))
    owner = t._md5hip_arena
    p = owner.ptr
    del t
    torch.cuda.synchronize()
    from sproxy_amd._lib import lib
    assert owner.ptr is not None                   # still referenced here: not yet freed
    owner.__del__()
    assert lib().md5hip_arena_free(ctypes.c_void_p(p)) == -2          # -ENOENT: already freed


def test_zero_copy_gather_modes(cuda):
    """Registered host memory (md5hip_host_register) pulled by the device
    gather kernel or per-segment DMA instead of the host memcpy: same digests
    as the oracle for page-list blocks with ragged, unaligned segment sizes,
    empty blocks and CRC-32 mode; a call touching unregistered memory takes
    the host gather; unregister works and double registration is refused."""
    rng = np.random.default_rng(404)
    heap = np.frombuffer(gen.xorshift_bytes(8 << 20, seed=405), np.uint8).copy()   # the "page heap"
    other = np.frombuffer(gen.xorshift_bytes(1 << 20, seed=406), np.uint8).copy()  # not registered
    page = 16384
    blocks, joined = [], []
    for b in range(60):
        segs = []
        for p in range(int(rng.integers(0, 6))):
            start = int(rng.integers(0, heap.size // page)) * page
            ln = page if rng.integers(0, 3) else int(rng.integers(1, page))     # ragged -> unaligned dst
            segs.append(heap[start:start + ln])
        blocks.append(segs)
        joined.append(b"".join(x.tobytes() for x in segs))
    lens = [len(j) for j in joined]
    arena = np.frombuffer(b"".join(joined) + b"\0", np.uint8)
    offs = np.cumsum([0] + lens[:-1])
    want = gen.oracle_digests(arena, offs, lens)
    want_crc = gen.oracle_crc32_batch(arena, offs, lens)
    m.register_host(heap)
    try:
        with pytest.raises(m.MD5HipError):
            m.register_host(heap[4096:8192])                 # overlaps
        with m.Batcher(device=0, slice_bytes=1 << 20, nslots=2) as b:
            for mode in (b.GATHER_HOST, b.GATHER_DEVICE, b.GATHER_DMA, b.GATHER_AUTO):
                b.set_gather(mode)
                b.set_digest(b.MD5)
                assert np.array_equal(b.submit_iov(blocks), want), mode
                flat = [x for segs in blocks for x in segs]
                fj = [x.tobytes() for x in flat]
                fa = np.frombuffer(b"".join(fj) + b"\0", np.uint8)
                fo = np.cumsum([0] + [len(x) for x in fj[:-1]])
                assert np.array_equal(b.submit(flat), gen.oracle_digests(fa, fo, [len(x) for x in fj]))
                b.set_digest(b.CRC32)
                assert np.array_equal(b.submit_iov(blocks), want_crc), mode
            b.set_gather(b.GATHER_DEVICE)
            b.set_digest(b.MD5)
            mixed = blocks[:5] + [[other[:5000]]]            # one unregistered segment
            got = b.submit_iov(mixed)
            assert np.array_equal(got[:5], want[:5])
            assert bytes(got[5]).hex() == bytes(gen.oracle_digests(other, [0], [5000])[0]).hex()
        with m.Pool((0, 0), slice_bytes=1 << 20, nslots=2) as p:
            p.set_gather(p.GATHER_DEVICE)
            assert np.array_equal(p.submit_iov(blocks), want)
    finally:
        m.unregister_host(heap)
    with pytest.raises(m.MD5HipError):
        m.unregister_host(heap)


@pytest.mark.gpu
def test_order_device_is_a_longest_first_permutation(cuda):
    """md5hip_plan_hist + md5hip_order_device (the batcher's planner): the
    device-built order is a permutation, keys non-increasing along it, bucket
    by bucket where md5hip_plan_hist put them; a descriptor launch with it
    gives the oracle digests."""
    import ctypes
    import torch
    from sproxy_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(2024)
    for n in (1, 63, 64, 1000, 200003, 100001):
        lens = rng.integers(0, 300000, n).astype(np.uint32)
        lens[rng.integers(0, n, max(1, n // 10))] = 16384          # a popular key
        if n == 100001:                                             # two keys, interleaved:
            lens = np.where(rng.integers(0, 2, n) == 1, 4096, 65536).astype(np.uint32)   # one add per key per wave
        keys = (lens >> 6) + 1
        kmax = int(keys.max())
        hist = np.bincount(keys, minlength=kmax + 1).astype(np.uint32)
        start = np.zeros(kmax + 1, np.uint32)
        v = L.md5hip_plan_hist(hist.ctypes.data, kmax, n, start.ctypes.data)
        assert v >= 0
        d_len = torch.from_numpy(lens.view(np.int32)).to(cuda)
        d_next = torch.from_numpy(start.view(np.int32)).to(cuda)
        d_ord = torch.full((n,), -1, dtype=torch.int32, device=cuda)
        s = torch.cuda.current_stream().cuda_stream
        assert L.md5hip_order_device(d_len.data_ptr(), n, kmax, d_next.data_ptr(), d_ord.data_ptr(), s) == 0
        order = d_ord.cpu().numpy().view(np.uint32)
        assert np.array_equal(np.sort(order), np.arange(n, dtype=np.uint32)), n
        assert np.all(np.diff(keys[order].astype(np.int64)) <= 0), n
        if n <= 1000:
            offs, total = gen.pack_offsets([int(x) for x in lens], align=16)
            host = gen.xorshift_array(total + 64, seed=n)
            dev = torch.from_numpy(host).to(cuda)
            got = m.digest_desc(dev, torch.tensor(offs, dtype=torch.int64, device=cuda), d_len, d_ord,
                                variant=v)
            assert np.array_equal(got.cpu().numpy(), gen.oracle_digests(host, offs, [int(x) for x in lens]))


def test_order_device_stable_equals_host_order(cuda):
    """md5hip_order_device_stable (ABI 5, the batcher's order for large
    slots): exactly md5hip_plan_desc's host order -- longest key first, equal
    keys in chunk-index order -- for random, single-key, two-key and
    C3-shaped lengths; a chunk past kmax goes last; scratch too small is
    -ENOSPC; a BALANCED launch with it gives the oracle digests."""
    import errno
    import torch
    from sproxy_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(2025)
    cases = [rng.integers(0, 300000, 200003).astype(np.uint32),
             np.full(70000, 16384, np.uint32),
             np.where(rng.integers(0, 2, 100001) == 1, 4096, 65536).astype(np.uint32),
             np.asarray(gen.mixed_lengths(150000, seed=9), np.uint32),
             rng.integers(0, 1 << 20, 5000).astype(np.uint32)]
    s = torch.cuda.current_stream().cuda_stream
    for lens in cases:
        n = lens.size
        kmax = int(((lens >> 6) + 1).max())
        need = L.md5hip_order_stable_scratch(n, kmax)
        assert need > 0 and L.md5hip_order_stable_scratch(n, 0) >= need
        scratch = torch.empty(need, dtype=torch.uint8, device=cuda)
        d_len = torch.from_numpy(lens.view(np.int32)).to(cuda)
        d_ord = torch.full((n,), -1, dtype=torch.int32, device=cuda)
        assert L.md5hip_order_device_stable(d_len.data_ptr(), n, kmax, scratch.data_ptr(), need,
                                            d_ord.data_ptr(), s) == 0
        host, _ = m.plan_desc(lens)
        assert np.array_equal(d_ord.cpu().numpy().view(np.uint32), host), n
        assert L.md5hip_order_device_stable(d_len.data_ptr(), n, kmax, scratch.data_ptr(), need - 1,
                                            d_ord.data_ptr(), s) == -errno.ENOSPC
    # a key past kmax: after every bucket, not dropped
    lens = np.array([100, 5000, 70000, 64, 5000], np.uint32)
    kmax = int(((np.array([100, 5000, 64, 5000]) >> 6) + 1).max())
    need = L.md5hip_order_stable_scratch(lens.size, kmax)
    scratch = torch.empty(need, dtype=torch.uint8, device=cuda)
    d_len = torch.from_numpy(lens.view(np.int32)).to(cuda)
    d_ord = torch.full((lens.size,), -1, dtype=torch.int32, device=cuda)
    assert L.md5hip_order_device_stable(d_len.data_ptr(), lens.size, kmax, scratch.data_ptr(), need,
                                        d_ord.data_ptr(), s) == 0
    assert d_ord.cpu().numpy().tolist() == [1, 4, 0, 3, 2]
    # a BALANCED launch in that order
    lens = np.asarray(gen.mixed_lengths(40000, seed=10, max_len=1 << 18), np.uint32)
    offs, total = gen.pack_offsets([int(x) for x in lens], align=16)
    host = gen.xorshift_array(total + 64, seed=11)
    kmax = int(((lens >> 6) + 1).max())
    need = L.md5hip_order_stable_scratch(lens.size, kmax)
    scratch = torch.empty(need, dtype=torch.uint8, device=cuda)
    d_len = torch.from_numpy(lens.view(np.int32)).to(cuda)
    d_ord = torch.empty(lens.size, dtype=torch.int32, device=cuda)
    assert L.md5hip_order_device_stable(d_len.data_ptr(), lens.size, kmax, scratch.data_ptr(), need,
                                        d_ord.data_ptr(), s) == 0
    got = m.digest_desc(torch.from_numpy(host).to(cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                        d_len, d_ord, variant="balanced")
    assert np.array_equal(got.cpu().numpy(), gen.oracle_digests(host, offs, [int(x) for x in lens]))


def test_fixed_auto_small_batches_run_fed(golden, cuda):
    """md5hip_digest_fixed's AUTO launch sends a batch of at most one 64-chunk
    group per CU to fed pairs (md5_desc_fed, implicit layout) when its chunks
    have two whole blocks: every golden edge length, a ragged last group,
    unaligned strides (the lane-direct kernel), against md5.c's digests."""
    e = golden["edge"]
    big = np.frombuffer(gen.mul_pattern(max(e["lengths"])), dtype=np.uint8)
    for L, want in zip(e["lengths"], e["md5"]):
        if L > (1 << 17):
            continue
        for stride in (max(16, (L + 15) // 16 * 16), L + 4):
            n = 130
            host = np.zeros(n * stride + 16, dtype=np.uint8)
            for i in range(n):
                host[i * stride:i * stride + L] = big[:L]
            got = m.digest_fixed(_dev(host, cuda), n, L, stride).cpu().numpy()
            assert all(bytes(x).hex() == want for x in got), (L, stride)
    n, L = 4000, 16384                                   # 63 groups: FED
    host = gen.xorshift_array(n * L, seed=4000)
    got = m.digest_fixed(_dev(host, cuda), n, L).cpu().numpy()
    assert np.array_equal(got, gen.oracle_digests_fixed(host, n, L))
