"""CRC-32 block checksums (netcache crc32.c + blk_make_crc fastcrc mode).

CPU: the oracle (oracle/crc32_oracle.c) pinned to tests/golden/crc32_golden.json,
which the reference crc32.c built in place produced (cross-checked with zlib).
GPU (-m gpu): crc32hip_fixed / crc32hip_desc bit-exact against the goldens and
the oracle, fastcrc head^tail included."""
import ctypes
import errno
import json
import os
import struct
import zlib

import numpy as np
import pytest

import gen
from sproxy_amd import _lib
from sproxy_amd import md5 as m

GOLD = json.load(open(os.path.join(gen.REPO, "tests", "golden", "crc32_golden.json")))


def _crc(b: bytes, fast=0) -> int:
    a = np.frombuffer(b + b"\0", dtype=np.uint8)
    return int(gen.oracle_crc32_batch(a, [0], [len(b)], fast)[0])


def test_oracle_kat_and_edges():
    for k in GOLD["kat"]:
        assert "%08x" % _crc(bytes.fromhex(k["hex"])) == k["crc"]
    big = gen.mul_pattern(1 << 20)
    for L, c in zip(GOLD["edge"]["lengths"], GOLD["edge"]["crc"]):
        assert "%08x" % _crc(big[:L]) == c
        assert "%08x" % zlib.crc32(big[:L]) == c


def test_oracle_fastcrc():
    data = gen.xorshift_bytes(100000, seed=0xC5C5)
    for (L, f), c in zip(GOLD["fastcrc"]["cases"], GOLD["fastcrc"]["crc"]):
        assert "%08x" % _crc(data[:L], f) == c, (L, f)


def test_oracle_batches():
    for b in GOLD["batches"]:
        n, L = b["n"], b["len"]
        buf = gen.xorshift_array(n * L)
        crcs = gen.oracle_crc32_batch(buf, np.arange(n, dtype=np.uint64) * L, [L] * n)
        assert "%08x" % gen.fold(b"".join(struct.pack("<I", int(c)) for c in crcs)) == b["fold"]
        if "crc" in b:
            assert ["%08x" % c for c in crcs] == b["crc"]


def test_crc_abi_errors():
    L = _lib.lib()
    E = -errno.EINVAL
    assert L.crc32hip_fixed(None, 0, 16, 16, 0, None, None) == 0
    assert L.crc32hip_fixed(None, 4, 16, 16, 0, None, None) == E
    assert L.crc32hip_fixed(ctypes.c_void_p(16), 4, 16, 16, 6, ctypes.c_void_p(16), None) == E
    assert L.crc32hip_desc(None, None, None, None, 2, 0, None, None) == E


# ----------------------------------------------------------------- GPU parity
def _dev(a, cuda):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(cuda)


CRC_VARIANTS = list(m.CRC_VARIANTS)


@pytest.mark.gpu
@pytest.mark.parametrize("variant", CRC_VARIANTS)
def test_gpu_crc_batches(cuda, variant):
    for b in GOLD["batches"]:
        n, L = b["n"], b["len"]
        host = gen.xorshift_array(n * L)
        got = m.crc32_fixed(_dev(host, cuda), n, L, variant=variant).cpu().numpy().view(np.uint32)
        assert "%08x" % gen.fold(b"".join(struct.pack("<I", int(c)) for c in got)) == b["fold"], (n, L)
        if "crc" in b:
            assert ["%08x" % c for c in got] == b["crc"]


@pytest.mark.gpu
@pytest.mark.parametrize("variant", CRC_VARIANTS)
def test_gpu_crc_edges_fixed_and_unaligned(cuda, variant):
    big = np.frombuffer(gen.mul_pattern(1 << 20), dtype=np.uint8)
    for L, want in zip(GOLD["edge"]["lengths"], GOLD["edge"]["crc"]):
        if L > (1 << 17):
            continue
        for stride in ((L + 15) // 16 * 16 or 16, L + 3):
            n = 70
            host = np.zeros(n * stride + 16, dtype=np.uint8)
            for i in range(n):
                host[i * stride:i * stride + L] = big[:L]
            got = m.crc32_fixed(_dev(host, cuda), n, L, stride, variant=variant).cpu().numpy().view(np.uint32)
            assert all("%08x" % c == want for c in got), (L, stride)


@pytest.mark.gpu
@pytest.mark.parametrize("fast", [0, 4, 64, 128, 4096])
def test_gpu_crc_desc_fastcrc(cuda, fast):
    import torch
    lens = gen.mixed_lengths(300, seed=31, max_len=1 << 17) + [0, 1, 4, 127, 128, 129, 4095, 4097]
    offs, total = gen.pack_offsets(lens, align=4)
    buf = gen.xorshift_array(total + 64, seed=88)
    want = gen.oracle_crc32_batch(buf, offs, lens, fast)
    got = m.crc32_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                       torch.tensor(lens, dtype=torch.int32, device=cuda),
                       fastcrc=fast).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)
    # the fixed entry with fastcrc (every chunk longer than fastcrc)
    if fast:
        n, L = 100, 16384
        host = gen.xorshift_array(n * L, seed=89)
        got = m.crc32_fixed(_dev(host, cuda), n, L, fastcrc=fast).cpu().numpy().view(np.uint32)
        want = gen.oracle_crc32_batch(host, np.arange(n, dtype=np.uint64) * L, [L] * n, fast)
        assert np.array_equal(got, want)


@pytest.mark.gpu
def test_gpu_crc_variants_grid_stride(cuda):
    """More chunks than one grid of the lane-table kernels covers (grid-stride
    loop), ragged n, every variant equal to the oracle."""
    n, L = 300000, 1040
    host = gen.xorshift_array(n * L, seed=515)
    want = gen.oracle_crc32_batch(host, np.arange(n, dtype=np.uint64) * L, [L] * n)
    d = _dev(host, cuda)
    for v in CRC_VARIANTS:
        got = m.crc32_fixed(d, n, L, variant=v).cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want), v


@pytest.mark.gpu
def test_gpu_crc_full_size(cuda):
    import torch
    n, L = 1 << 20, 16384
    d = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    m.fill_synthetic(d, seed=0xCC)
    got = m.crc32_fixed(d, n, L)
    for v in CRC_VARIANTS[1:]:
        assert torch.equal(m.crc32_fixed(d, n, L, variant=v), got), v
    idx = np.unique(np.concatenate([[0, n - 1], np.random.default_rng(3).integers(0, n, 4096)]))
    rows = d.view(n, L)[torch.from_numpy(idx).to(cuda)].cpu().numpy()
    want = gen.oracle_crc32_batch(rows.reshape(-1), np.arange(idx.size, dtype=np.uint64) * L,
                                  [L] * idx.size)
    assert np.array_equal(got[torch.from_numpy(idx).to(cuda)].cpu().numpy().view(np.uint32), want)
    del d
    torch.cuda.empty_cache()


@pytest.mark.gpu
def test_gpu_crc_desc_netcache_blocks(cuda):
    """crc32hip_desc on the netcache shape (full blocks + ragged last blocks,
    a wave without any 128-B stage, one unaligned chunk, > one grid of
    64-chunk groups), ordered longest-first and unordered: the XPERM16
    descriptor kernel and its lane-direct fallback against crc32.c."""
    import torch
    rng = np.random.default_rng(777)
    for S, n in ((4096, 40000), (65536, 700)):
        lens = np.full(n, S, dtype=np.int64)
        tail = rng.integers(0, 8, n) == 0
        lens[tail] = rng.integers(0, S, int(tail.sum()))
        lens[-70:] = rng.integers(0, 128, 70)
        lens = [int(x) for x in lens]
        offs = list(gen.pack_offsets(lens, align=16)[0])
        offs[n // 2] += 4                              # one unaligned chunk
        total = offs[-1] + lens[-1] + 64
        buf = gen.xorshift_array(total + 64, seed=S)
        want = gen.oracle_crc32_batch(buf, offs, lens)
        d = _dev(buf, cuda)
        t_off = torch.tensor(offs, dtype=torch.int64, device=cuda)
        t_len = torch.tensor(lens, dtype=torch.int32, device=cuda)
        for order in (m.plan_order(lens).astype(np.int32), None):
            got = m.crc32_desc(d, t_off, t_len, None if order is None else _dev(order, cuda))
            assert np.array_equal(got.cpu().numpy().view(np.uint32), want), (S, order is None)


@pytest.mark.gpu
@pytest.mark.parametrize("fast", [4, 64, 100, 128, 1000, 16368])
def test_gpu_fastcrc_xdma_windows(cuda, fast):
    """fastcrc through the LDS-DMA loader (crc32_fast_xdma16) and, for 64 and
    128, the pipelined lane-load kernel (crc32_fast_pipe, whose ragged and
    unaligned groups fall back to lane_range): head and tail windows as row
    pairs, more 32-chunk groups than one grid holds, fixed
    16 KiB blocks and 16-B packed ragged blocks (windows of every alignment,
    blocks shorter than the window, empty blocks), against crc32.c's
    blk_make_crc combination (blk_io.c:408-424) in the oracle."""
    import torch
    n, L = 40000, 16384
    d = torch.empty(n * L, dtype=torch.uint8, device=cuda)
    m.fill_synthetic(d, seed=0xFA57 + fast)
    got = m.crc32_fixed(d, n, L, fastcrc=fast).cpu().numpy().view(np.uint32)
    host = gen.synthetic_bytes(n * L, 0xFA57 + fast)
    want = gen.oracle_crc32_batch(host, np.arange(n, dtype=np.uint64) * L, [L] * n, fast)
    assert np.array_equal(got, want)
    del d, host
    rng = np.random.default_rng(fast)
    lens = [int(x) for x in rng.integers(0, 40000, 5000)] + [0, 1, fast - 1, fast, fast + 1]
    offs, total = gen.pack_offsets(lens, align=16)
    buf = gen.xorshift_array(total + 64, seed=fast)
    want = gen.oracle_crc32_batch(buf, offs, lens, fast)
    got = m.crc32_desc(_dev(buf, cuda), torch.tensor(offs, dtype=torch.int64, device=cuda),
                       torch.tensor(lens, dtype=torch.int32, device=cuda),
                       fastcrc=fast).cpu().numpy().view(np.uint32)
    assert np.array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("align", [16, 4, 1])
def test_gpu_crc_split_desc(cuda, align):
    """CRCSPLIT (crc32_split: one wave per chunk, 256-B segments combined with
    crc32_combine's zero-byte operators) against crc32.c: every length around
    the segment (256 B) and pass (16 KiB) boundaries, chunks of several passes
    (up to 1 MiB + 13), empty and 1-3 byte chunks, starts at any alignment,
    ordered and unordered; and AUTO's choice for a netcache-size vector."""
    import torch
    rng = np.random.default_rng(4000 + align)
    edges = [0, 1, 2, 3, 4, 5, 63, 64, 65, 255, 256, 257, 511, 512, 513, 16383, 16384, 16385,
             16384 + 256, 32767, 32768, 32769, 65536 + 100, (1 << 20) + 13]
    lens = edges + [int(x) for x in rng.integers(0, 70000, 200)]
    offs, total = gen.pack_offsets(lens, align=align)
    buf = gen.xorshift_array(total + 64, seed=align)
    want = gen.oracle_crc32_batch(buf, offs, lens)
    d = _dev(buf, cuda)
    t_off = torch.tensor(offs, dtype=torch.int64, device=cuda)
    t_len = torch.tensor(lens, dtype=torch.int32, device=cuda)
    for order in (m.plan_order(lens).astype(np.int32), None):
        o = None if order is None else _dev(order, cuda)
        for v in ("split", "auto", "xdma16"):
            got = m.crc32_desc(d, t_off, t_len, o, variant=v).cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want), (v, order is None)
    # fastcrc windows (head ^ tail, blk_io.c:408-424) split as two messages
    for fast in (4, 100, 1000, 4096, 16368):
        want_f = gen.oracle_crc32_batch(buf, offs, lens, fast)
        for v in ("split", "auto"):
            got = m.crc32_desc(d, t_off, t_len, fastcrc=fast, variant=v).cpu().numpy().view(np.uint32)
            assert np.array_equal(got, want_f), (fast, v)
    # a netcache vector: 64 x 16 KiB pages; AUTO splits it (<= 4 chunks per CU)
    n, L = 64, 16384
    host = gen.xorshift_array(n * L, seed=64)
    want = gen.oracle_crc32_batch(host, np.arange(n, dtype=np.uint64) * L, [L] * n)
    for v in ("auto", "split"):
        got = m.crc32_fixed(_dev(host, cuda), n, L, variant=v).cpu().numpy().view(np.uint32)
        assert np.array_equal(got, want), v


@pytest.mark.gpu
def test_gpu_crc_queue_long_blocks_split(cuda):
    """The queue's CRC-32 launch picks the split kernel from the slot's mean
    chunk length (md5hip_crc_desc_choice): long blocks (netcache chunk_size
    up to MiBs: 1 MiB + ragged, 256 KiB) split at any count it allows, short
    ones (< 2 KiB) only in small batches, and every CRC equals crc32.c's."""
    import torch
    q = m.Queue(device=torch.cuda.current_device())
    q.set_digest(m.Batcher.CRC32)
    rng = np.random.default_rng(2024)
    for lens in ([(1 << 20) + 13] * 5 + [1 << 20] * 40 + [5, 0],
                 [256 << 10] * 300 + [int(x) for x in rng.integers(0, 256 << 10, 50)],
                 [int(x) for x in rng.integers(0, 2048, 5000)]):
        offs, total = gen.pack_offsets(lens, align=16)
        buf = gen.xorshift_array(total + 64, seed=len(lens))
        want = gen.oracle_crc32_batch(buf, offs, lens)
        d = _dev(buf, cuda)
        ptrs = np.asarray(offs, dtype=np.uint64) + np.uint64(d.data_ptr())
        got = q.submit_device(ptrs, np.asarray(lens, dtype=np.uint32))
        got = np.asarray(got).view(np.uint32).reshape(-1)
        assert np.array_equal(got, want), len(lens)
    q.close()


@pytest.mark.gpu
@pytest.mark.parametrize("registered", [False, True])
def test_gpu_fastcrc_host_blocks_stage_only_windows(cuda, registered):
    """A CRC-32 batcher with a fastcrc window F stages (or maps, zero-copy)
    only the first and last F bytes of each host block over 2F bytes (shorter
    ones whole; md5_submit.c staged_len): lengths around F and 2F, empty blocks, and page lists cut
    inside either window.  Every CRC equals crc32.c's blk_make_crc rule
    (blk_io.c:408-424), and the bytes staged are the windows' (stats)."""
    F = 128
    rng = np.random.default_rng(128 + registered)
    lens = [0, 1, F - 1, F, F + 1, 2 * F - 1, 2 * F, 2 * F + 1, 16384, 65536] + \
        [int(x) for x in rng.integers(0, 70000, 200)]
    offs, total = gen.pack_offsets(lens, align=16)
    buf = gen.xorshift_array(total + 4096, seed=777)
    want = gen.oracle_crc32_batch(buf, offs, lens, F)
    if registered:
        m.register_host(buf)
    try:
        chunks = []
        for o, L in zip(offs, lens):
            cut = int(rng.integers(0, L + 1)) if L else 0
            cut2 = int(rng.integers(cut, L + 1)) if L else 0
            mv = memoryview(buf)[o:o + L]
            chunks.append([mv[:cut], mv[cut:cut2], mv[cut2:]])
        with m.Batcher(device=0, kind=m.Batcher.CRC32, fastcrc=F) as b:
            got = b.submit_iov(chunks)
            st = b.stats()
        assert np.array_equal(np.asarray(got).view(np.uint32).reshape(-1), want)
        staged = sum(((2 * F if L > 2 * F else L) + 127) & ~127 for L in lens)   # up to 2F: whole
        if not registered:
            assert st["bytes_staged"] == staged, (st["bytes_staged"], staged)
    finally:
        if registered:
            m.unregister_host(buf)



@pytest.mark.gpu
def test_gpu_fastcrc_window_over_half_the_slice(cuda):
    """A fastcrc window F over half the batcher's slice: a block between F
    and 2F bytes is staged whole (its two windows would not fit a slot), from
    pageable and registered memory; CRCs as blk_make_crc (blk_io.c:408-424)."""
    F = 600 << 10
    lens = [700 << 10, F + 4, (1 << 20) - 128]
    offs, total = gen.pack_offsets(lens, align=16)
    buf = gen.xorshift_array(total + 4096, seed=4242)
    want = gen.oracle_crc32_batch(buf, offs, lens, F)
    for registered in (False, True):
        if registered:
            m.register_host(buf)
        try:
            with m.Batcher(device=0, slice_bytes=1 << 20, kind=m.Batcher.CRC32, fastcrc=F) as b:
                got = b.submit([memoryview(buf)[o:o + n] for o, n in zip(offs, lens)])
            assert np.array_equal(np.asarray(got).reshape(-1), want), registered
        finally:
            if registered:
                m.unregister_host(buf)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["md5", "fastcrc"])
def test_gpu_fragmented_chunks_at_the_zero_copy_table_edge(cuda, kind):
    """Chunks of ~4,096 one-byte segments of registered memory (a 1 MiB
    slice's zero-copy table holds 4,096 entries): a chunk goes zero-copy only
    if its pieces fit an empty slot, else it is staged, and either way its
    digest is right (md5_submit.c zc_pieces)."""
    F = 100
    buf = gen.xorshift_array(2 * 4200 + 64, seed=4096)
    m.register_host(buf)
    try:
        mk = dict(kind=m.Batcher.CRC32, fastcrc=F) if kind == "fastcrc" else {}
        with m.Batcher(device=0, slice_bytes=1 << 20, **mk) as b:
            for ns in (4093, 4094, 4095, 4096, 4097):
                segs = [memoryview(buf)[2 * k:2 * k + 1] for k in range(ns)]
                flat = np.ascontiguousarray(buf[0:2 * ns:2])
                got = np.asarray(b.submit_iov([segs])).reshape(-1)
                if kind == "fastcrc":
                    want = gen.oracle_crc32_batch(flat, [0], [ns], F)
                else:
                    want = gen.oracle_digests(flat, [0], [ns]).reshape(-1)
                assert np.array_equal(got, want), ns
    finally:
        m.unregister_host(buf)


@pytest.mark.gpu
@pytest.mark.parametrize("registered", [False, True])
def test_gpu_driver_test_shape(cuda, registered):
    """netcache's own stress configuration (driver_test.c:583-586:
    chunk_size 256 KiB, fastcrc 128) against its loopback origin, whose blocks
    begin with "0123456789ABCDEF" (NC_VALIDATE_ORIGIN_DATA, bc_mgr.c:1419-1456):
    vectors of 256 KiB blocks handed over as lists of 16 KiB pages, a short
    last block included.  Store (blk_make_crc, blk_io.c:851-863) and verify
    with one corrupted block (blk_io.c:665-704: only that block fails) through
    one CRC-32 batcher with fastcrc 128, and the same vectors' MD5."""
    F, B, P = 128, 256 << 10, 16 << 10
    lens = [B] * 7 + [B - 5000]
    offs = [k * B for k in range(len(lens))]
    buf = gen.xorshift_array(len(lens) * B + 4096, seed=583)
    for o in offs:
        buf[o:o + 16] = np.frombuffer(b"0123456789ABCDEF", np.uint8)
    if registered:
        m.register_host(buf)
    try:
        pages = [[memoryview(buf)[o + a:o + min(a + P, L)] for a in range(0, L, P)] for o, L in zip(offs, lens)]
        want = gen.oracle_crc32_batch(buf, offs, lens, F)
        with m.Batcher(device=0, kind=m.Batcher.CRC32, fastcrc=F) as b:
            got = np.asarray(b.submit_iov(pages)).reshape(-1)
            assert np.array_equal(got, want)
            bad = got.copy()
            bad[3] ^= 1
            ok, nbad = b.verify_iov(pages, bad)
            assert nbad == 1 and not ok[3] and ok.sum() == len(lens) - 1
        with m.Batcher(device=0) as b:
            assert np.array_equal(np.asarray(b.submit_iov(pages)), gen.oracle_digests(buf, offs, lens))
    finally:
        if registered:
            m.unregister_host(buf)
