"""The C-ABI boundary on CPU: libmd5hip.so loads, exports every symbol that
include/*.h declares, keeps md5.h's struct layout, the per-message
MD5Init/Update/Final entries (host path by design, include/md5.h) match the
golden vectors, and argument errors come back as -errno before any device
work is attempted."""
import ctypes
import errno
import os
import re
import subprocess

import numpy as np

import gen
from sproxy_amd import _lib
from sproxy_amd import md5 as m

INC = os.path.join(gen.REPO, "include")


def declared_functions():
    names = set()
    for h in ("md5.h", "md5hip.h", "nc_md5.h", "nc_digest.h"):
        text = open(os.path.join(INC, h)).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for mm in re.finditer(r"^\s*(?:const\s+)?[\w\s\*]+?\b(\w+)\s*\(", text, flags=re.M):
            name = mm.group(1)
            if name not in ("if", "sizeof", "defined"):
                names.add(name)
    return names


def test_exports_every_declared_symbol():
    decl = declared_functions()
    assert {"MD5Init", "MD5Update", "MD5Final", "md5hip_digest_fixed", "md5_batch_submit"} <= decl
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = {ln.split()[-1] for ln in out.splitlines() if " T " in ln}
    missing = decl - exported
    assert not missing, missing
    assert set(_lib.EXPORTS) == decl
    _lib.lib()   # binds every signature


def test_abi_version_and_names():
    L = _lib.lib()
    assert L.md5hip_abi_version() == 5
    assert [m.variant_name(v) for v in m.VARIANTS.values()] == list(m.VARIANTS)


def test_header_compiles_as_c_and_layout():
    src = r'''
    #include <stddef.h>
    #include "md5.h"
    #include "md5hip.h"
    _Static_assert(sizeof(struct MD5Context) == 88, "size");
    _Static_assert(offsetof(struct MD5Context, bits) == 16, "bits");
    _Static_assert(offsetof(struct MD5Context, in) == 24, "in");
    int main(void) { return MD5_DIGEST_SIZE == 16 ? 0 : 1; }
    '''
    exe = os.path.join(gen.REPO, "build", "hdrcheck")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", INC, "-x", "c", "-", "-o", exe],
                   input=src, text=True, check=True)
    assert subprocess.run([exe]).returncode == 0
    assert ctypes.sizeof(_lib.MD5Context) == 88


def test_streaming_api_matches_golden(golden):
    for v in golden["kat"]:
        msg = bytes.fromhex(v["hex"])
        ctx = m.MD5Context()
        m.MD5Init(ctx)
        cut = len(msg) // 3
        m.MD5Update(ctx, msg[:cut])
        m.MD5Update(ctx, msg[cut:])
        digest = bytearray(16)
        assert m.MD5Final(digest, ctx).hex() == v["md5"] == digest.hex()
        assert bytes(ctx) == b"\0" * 88          # md5.c:264
    e = golden["edge"]
    big = gen.mul_pattern(max(e["lengths"]))
    for L, d in zip(e["lengths"], e["md5"]):
        assert m.md5(big[:L]).hex() == d


def test_streaming_api_random_splits(golden):
    r = golden["random_lengths"]
    data = gen.xorshift_bytes(max(r["lengths"]), seed=0x243F6A8885A308D3)
    rng = np.random.default_rng(5)
    for L, d in zip(r["lengths"], r["md5"]):
        ctx = m.MD5Context()
        m.MD5Init(ctx)
        cuts = sorted(int(x) for x in rng.integers(0, L + 1, 4))
        prev = 0
        for c in cuts + [L]:
            m.MD5Update(ctx, data[prev:c])
            prev = c
        assert m.MD5Final(None, ctx).hex() == d


def test_bitcount_carry():
    """bits[0] wraps at 2^32 bits (512 MiB) and carries into bits[1] (md5.c:179-182)."""
    ctx = m.MD5Context()
    m.MD5Init(ctx)
    ctx.bits[0] = 0xFFFFFFF8
    m.MD5Update(ctx, b"abc")
    assert ctx.bits[0] == (0xFFFFFFF8 + 24) & 0xFFFFFFFF and ctx.bits[1] == 1


def test_argument_errors_before_device_work():
    L = _lib.lib()
    EINVAL = -errno.EINVAL
    assert L.md5hip_digest_fixed(None, 0, 16, 16, None, None) == 0          # empty batch: no-op
    assert L.md5hip_digest_fixed(None, 5, 16, 16, None, None) == EINVAL
    assert L.md5hip_digest_fixed(ctypes.c_void_p(16), 5, 32, 16, ctypes.c_void_p(16), None) == EINVAL
    assert L.md5hip_digest_fixed(ctypes.c_void_p(16), 5, 16, 16, ctypes.c_void_p(8), None) == EINVAL
    assert L.md5hip_digest_fixed_variant(ctypes.c_void_p(16), 5, 16, 16, ctypes.c_void_p(16), None, 99) == EINVAL
    assert L.md5hip_digest_desc(None, None, None, None, 0, None, None) == 0
    assert L.md5hip_digest_desc(None, None, None, None, 3, None, None) == EINVAL
    assert L.md5hip_digest_desc_variant(None, None, None, None, 0, None, None, 1) == 0
    assert L.md5hip_digest_desc_variant(ctypes.c_void_p(16), ctypes.c_void_p(16), ctypes.c_void_p(16),
                                        None, 3, ctypes.c_void_p(16), None, 8) == EINVAL   # 8 = MD5HIP_DESC_NUM_VARIANTS
    assert L.md5hip_fill_synthetic(ctypes.c_void_p(16), 15, 1, None) == EINVAL
    h = ctypes.c_void_p()
    assert L.md5hip_batcher_create(0, 1 << 20, 99, ctypes.byref(h)) == EINVAL
    assert L.md5_batch_submit(None, None, None, 1, None) == EINVAL
    t = ctypes.c_uint64()
    assert L.md5_batch_submit_async(None, None, None, 1, None, ctypes.byref(t)) == EINVAL
    assert L.md5_batch_submit_iov_async(None, None, None, 1, None, ctypes.byref(t)) == EINVAL
    assert L.md5_batch_wait(None, 0) == EINVAL
    assert L.md5_batch_poll(None, 0) == EINVAL
    p = ctypes.c_void_p()
    assert L.md5hip_arena_alloc(0, 0, ctypes.byref(p)) == EINVAL
    assert L.md5hip_arena_alloc(0, 1 << 20, None) == EINVAL
    assert L.md5hip_arena_free(None) == EINVAL
    assert L.md5hip_arena_free(ctypes.c_void_p(1 << 30)) == -errno.ENOENT     # not an arena
    assert L.md5hip_plan_desc(None, 5, None) == EINVAL
    # the pool router and the producer-ordered device submit (no pool / batcher)
    assert L.md5hip_pool_submit_async(None, None, None, 1, None, ctypes.byref(t)) == EINVAL
    assert L.md5hip_pool_submit_iov_async(None, None, None, 1, None, ctypes.byref(t)) == EINVAL
    assert L.md5hip_pool_wait(None, 1) == EINVAL and L.md5hip_pool_poll(None, 1) == EINVAL
    assert L.md5hip_pool_set_split(None, 1) == EINVAL
    assert L.md5hip_pool_get_stats(None, None) == EINVAL
    assert L.md5hip_pool_device_stats(None, 0, None) == EINVAL
    assert L.md5hip_pool_set_digest(None, 0, 0) == EINVAL
    assert L.md5_batch_submit_device_on(None, None, None, 1, None, 0, None, None) == EINVAL
    # set_chain: modes outside 0..2 are refused before the batcher is touched
    assert L.md5hip_batcher_set_chain(None, 1) == EINVAL
    assert L.md5hip_batcher_set_chain(ctypes.c_void_p(16), 3) == EINVAL
    assert L.md5hip_batcher_set_chain(ctypes.c_void_p(16), -1) == EINVAL
    # ABI 4 failure-policy entries
    assert L.md5hip_batcher_health(None) == EINVAL
    assert L.md5hip_batcher_inject_fault(None, 1) == EINVAL
    assert L.md5hip_pool_get_health(None, None) == EINVAL
    assert L.md5hip_pool_device_health(None, 0) == EINVAL
    assert L.md5hip_pool_inject_fault(None, 0, 1) == EINVAL


def test_producer_default_without_torch(monkeypatch):
    """Batcher.submit_device*(after='current') without torch orders on the
    null stream of the batcher's device (what a raw-HIP producer uses when
    it names no stream), instead of failing on its own default argument."""
    import types
    monkeypatch.setattr(m, "torch", None)
    b = types.SimpleNamespace(device=0)
    assert m.Batcher._producer(b, "current") == (None, 1)
    assert m.Batcher._producer(b, None) == (None, 0)
    assert m.Batcher._producer(b, 1234) == (1234, 1)


def test_device_fixed_explicit_stride_zero_is_kept():
    """submit_device_fixed_async(stride=0) passes stride 0 on as the C entry
    reads it (len 0 only), instead of turning it into stride = length:
    length 16 at stride 0 is refused before any device work."""
    import types
    b = types.SimpleNamespace(device=0)
    import pytest
    with pytest.raises(ValueError):
        m.Batcher.submit_device_fixed_async(b, 0x1000, 4, 16, stride=0)


def test_plan_order_longest_first():
    rng = np.random.default_rng(1)
    lens = rng.integers(0, 1 << 20, 5000).astype(np.uint32)
    order = m.plan_order(lens)
    assert sorted(order.tolist()) == list(range(5000))
    blocks = (lens[order] >> 6)
    assert np.all(np.diff(blocks.astype(np.int64)) <= 0)
    # stable within equal block counts
    for b in np.unique(blocks)[:50]:
        idx = order[blocks == b]
        assert np.all(np.diff(idx.astype(np.int64)) > 0)
    huge = np.array([0xFFFFFFFF, 5, 1 << 31, 64], dtype=np.uint32)   # comparison-sort path
    assert m.plan_order(huge).tolist() == [0, 2, 3, 1]
    assert m.plan_order(np.array([], dtype=np.uint32)).size == 0


def test_plan_desc_picks_hybrid_only_for_standout_long_chunks():
    """md5hip_plan_desc: the same order as md5hip_plan_order; FED for small
    batches of <= 1 group per CU with a chunk of >= 2 whole blocks, LANE for
    other small batches (<= 2 groups per CU -- 256 CUs when no device is
    visible); HYBRID
    only when the longest chunks (>= 256 KiB) stand out (the chunk two waves
    per CU deep is <= 1/4 as long)."""
    rng = np.random.default_rng(5)
    mixed = np.array([4096 << int(k) for k in rng.integers(0, 9, 80000)], dtype=np.uint32)
    order, v = m.plan_desc(mixed)
    assert np.array_equal(order, m.plan_order(mixed)) and v == "hybrid"           # C3 shape
    assert m.plan_desc(np.full(65536, 262144, np.uint32))[1] == "xdma"            # equal blocks
    ragged = np.full(65536, 262144, np.uint32)
    ragged[::8] = rng.integers(1, 262144, 8192)
    assert m.plan_desc(ragged)[1] == "xdma"                # probe 32,768 deep is still full size
    few = np.full(40000, 1 << 20, np.uint32)
    few[-1] = 100
    assert m.plan_desc(few)[1] == "xdma"                   # long, but all of equal length
    few[5000:] = 4096
    assert m.plan_desc(few)[1] == "hybrid"                 # long chunks stand out
    assert m.plan_desc(np.full(50000, 65536, np.uint32))[1] == "xdma"             # < 256 KiB
    # small batches (256 CUs without a device): FED up to one group per CU,
    # LANE up to two, and LANE when no chunk has two whole blocks
    for n in (1, 64, 1000, 16384):
        assert m.plan_desc(np.full(n, 16384, np.uint32))[1] == "fed", n
    for n in (16385, 32768):
        assert m.plan_desc(np.full(n, 16384, np.uint32))[1] == "lane", n
    for L in (0, 1, 64, 127):
        assert m.plan_desc(np.full(1000, L, np.uint32))[1] == "lane", L
    assert m.plan_desc(np.full(1000, 128, np.uint32))[1] == "fed"
    small_mixed = np.full(1000, 1 << 20, np.uint32)
    small_mixed[-1] = 100
    assert m.plan_desc(small_mixed)[1] == "fed"
    assert m.plan_desc(np.full(32769, 16384, np.uint32))[1] == "xdma"
    assert m.plan_desc(np.array([], np.uint32))[0].size == 0


def test_device_api_rejects_host_tensors():
    import pytest
    import torch
    with pytest.raises(ValueError):
        m.digest_fixed(torch.zeros((4, 64), dtype=torch.uint8))


def test_pool_plan_partitions_by_bytes():
    """md5hip_pool_plan (host logic of the multi-GPU pool, §8e): contiguous,
    covering, equal counts for fixed batches, near-equal weight for mixed."""
    for n in (0, 1, 7, 1000, 1 << 20):
        for G in (1, 2, 3, 8):
            f = m.pool_plan(n, G)
            assert list(f) == [n * g // G for g in range(G + 1)]
    rng = np.random.default_rng(5)
    for trial in range(20):
        n = int(rng.integers(0, 3000))
        lens = gen.mixed_lengths(n, seed=trial, max_len=1 << 20) if n else []
        w = np.asarray(lens, dtype=np.int64) + 64
        for G in (1, 2, 4, 8):
            f = m.pool_plan(lens, G).astype(np.int64)
            assert f[0] == 0 and f[-1] == n and np.all(np.diff(f) >= 0)
            parts = [w[f[g]:f[g + 1]].sum() for g in range(G)]
            slack = w.max() if n else 0
            assert max(parts) <= w.sum() / G + slack
    # one huge chunk among small ones: it lands alone-ish, nothing is lost
    f = m.pool_plan([16] * 10 + [1 << 30] + [16] * 10, 4)
    assert f[0] == 0 and f[-1] == 21
    L, EINVAL = _lib.lib(), -errno.EINVAL
    assert L.md5hip_pool_plan(None, 5, 0, (ctypes.c_uint64 * 2)()) == EINVAL
    h = ctypes.c_void_p()
    assert L.md5hip_pool_create(None, 0, 0, 0, ctypes.byref(h)) == EINVAL


def test_plan_desc_picks_balanced_for_coalesced_mixed_batches():
    """BALANCED (LPT over one wave per SIMD) for mixed batches holding several
    waves of work per SIMD -- coalesced C3 submissions -- but not for one C3
    batch (chain-bound: HYBRID) nor for equal-length netcache blocks (XDMA)."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    one = bench.c3_lens(16 << 30, 1000).astype(np.uint32)
    assert m.plan_desc(one)[1] == "hybrid"
    three = np.concatenate([bench.c3_lens(16 << 30, 3000 + 31 * j) for j in range(3)]).astype(np.uint32)
    order, v = m.plan_desc(three)
    assert v == "balanced" and np.array_equal(order, m.plan_order(three))
    five = np.concatenate([bench.c3_lens(16 << 30, 3000 + 31 * j) for j in range(5)]).astype(np.uint32)
    assert m.plan_desc(five)[1] == "balanced"
    big_uniform = np.full(1 << 20, 16384, np.uint32)
    big_uniform[::8] = 100
    assert m.plan_desc(big_uniform)[1] == "xdma"


def test_plan_order_stable_across_thread_split():
    """md5hip_plan_order: longest-first by 64-B block count, ties in index
    order (a stable counting sort), also where it splits the index range over
    several threads (>= 2^18 chunks) and for block counts past 2^20 (the
    comparison-sort fallback)."""
    for n, hi in ((0, 10), (1, 10), (1000, 1 << 21), (262143, 1 << 21), (262144, 1 << 21),
                  (1 << 20, 1 << 22), (300001, 1 << 16), (5000, 1 << 31)):
        x = np.random.default_rng(n + hi).integers(0, hi, n).astype(np.uint32)
        got = m.plan_order(x)
        want = np.argsort(-(x.astype(np.int64) >> 6), kind="stable")
        assert np.array_equal(got, want), (n, hi)


def test_plan_hist_matches_plan_desc():
    """md5hip_plan_hist (planning from a histogram of keys, as the batcher
    keeps while chunks arrive) makes md5hip_plan_desc's choice on the same
    batch, and its bucket starts are where each key begins in the
    longest-first order."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    L = _lib.lib()
    names = {v: k for k, v in m.DESC_VARIANTS.items()}
    rng = np.random.default_rng(8)
    cases = [bench.c3_lens(16 << 30, 1000),
             np.concatenate([bench.c3_lens(16 << 30, 3000 + 31 * j) for j in range(3)]),
             np.full(1 << 16, 16384), rng.integers(0, 1 << 20, 5000), rng.integers(0, 4096, 100),
             np.array([1 << 20] * 10 + [4096] * 100000)]
    for lens in cases:
        lens = lens.astype(np.uint32)
        keys = (lens >> 6) + 1
        kmax = int(keys.max())
        hist = np.bincount(keys, minlength=kmax + 1).astype(np.uint32)
        start = np.zeros(kmax + 1, np.uint32)
        v = L.md5hip_plan_hist(hist.ctypes.data, kmax, lens.size, start.ctypes.data)
        order, want = m.plan_desc(lens)
        assert names[v] == want, (names[v], want)
        sk = keys[order]                                   # keys in longest-first order
        for k in np.unique(keys):
            assert start[kmax - k] == np.argmax(sk == k), k
        assert start[kmax] == lens.size
    assert L.md5hip_plan_hist(None, 1, 1, None) == -errno.EINVAL
