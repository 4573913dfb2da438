"""The batcher as a coalescing, out-of-order submission queue (md5_submit.c):
device-resident chunks (md5_batch_submit_device*), host chunks, several
submitting threads, tickets completing independently.  Every digest array is
checked against the oracle (oracle/md5_oracle.c through tests/gen.py)."""
import threading

import numpy as np
import pytest
import torch

import gen
import sproxy_amd.md5 as m

pytestmark = pytest.mark.gpu


def _arena_batch(lens, seed, cuda, align=16):
    """A device buffer holding chunks of `lens` (packed at `align`), its host
    copy, the device addresses and the oracle digests."""
    offs, total = gen.pack_offsets(lens, align=align)
    host = gen.xorshift_array(total + 64, seed=seed)
    dev = torch.from_numpy(host.copy()).to(cuda)
    ptrs = np.asarray(offs, dtype=np.uint64) + np.uint64(dev.data_ptr())
    return dev, ptrs, np.asarray(lens, dtype=np.uint32), gen.oracle_digests(host, offs, lens)


def test_queue_device_chunks_host_and_device_digests(cuda):
    rng = np.random.default_rng(7)
    lens = [int(x) for x in rng.integers(0, 300000, 700)] + [0, 1, 55, 56, 63, 64, 65]
    dev, ptrs, L, want = _arena_batch(lens, 71, cuda, align=1)      # any alignment
    with m.Queue(device=0) as q:
        got_h = q.submit_device(ptrs, L)                              # digests to host
        out = torch.empty((len(lens), 16), dtype=torch.uint8, device=cuda)
        q.submit_device(ptrs, L, out=out)                             # digests stay on device
        torch.cuda.synchronize()
    assert np.array_equal(got_h, want)
    assert np.array_equal(out.cpu().numpy(), want)


def test_queue_device_digests_in_place_and_scattered(cuda):
    """Device-side digests: a slot holding one in-order submission is written
    in place by the kernel (16-B-aligned output, also slot by slot when the
    submission spans several slots); an unaligned output, or several
    submissions sharing a slot, go through the scatter kernel."""
    rng = np.random.default_rng(17)
    lens = [int(x) for x in rng.integers(0, 70000, 1000)] + [0, 1, 63, 64, 65]
    dev, ptrs, L, want = _arena_batch(lens, 171, cuda)
    n = len(lens)
    with m.Queue(device=0, max_chunks=256) as q:                      # 4+ slots' worth
        out = torch.empty((n, 16), dtype=torch.uint8, device=cuda)
        q.submit_device(ptrs, L, out=out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), want)
        raw = torch.zeros(n * 16 + 4, dtype=torch.uint8, device=cuda)
        odd = raw[4:].view(n, 16)                                     # not 16-B aligned
        q.submit_device(ptrs, L, out=odd)
        torch.cuda.synchronize()
        assert np.array_equal(odd.cpu().numpy(), want)
        halves = [torch.empty((k, 16), dtype=torch.uint8, device=cuda) for k in (100, 150)]
        p1 = q.submit_device_async(ptrs[:100], L[:100], out=halves[0])
        p2 = q.submit_device_async(ptrs[100:250], L[100:250], out=halves[1])
        p1.wait()
        p2.wait()
        torch.cuda.synchronize()
        assert np.array_equal(torch.cat(halves).cpu().numpy(), want[:250])


def test_queue_tickets_complete_out_of_order(cuda):
    """A submission of four 64 MiB chunks (each a ~0.6 s serial chain) and a
    later one of short chunks: the short ticket completes while the long one
    is still running -- completion does not follow submission order."""
    long_lens = [64 << 20] * 4
    dl, pl, Ll, wl = _arena_batch(long_lens, 5, cuda)
    short_lens = [4096] * 256
    ds, ps, Ls, ws = _arena_batch(short_lens, 6, cuda)
    with m.Queue(device=0, nslots=4) as q:
        q.set_inflight(2)
        a = q.submit_device_async(pl, Ll)
        b = q.submit_device_async(ps, Ls)
        assert np.array_equal(b.wait(), ws)
        assert not a.poll(), "the long ticket finished before the short one was delivered"
        assert np.array_equal(a.wait(), wl)
        assert a.poll() and b.poll()


def test_queue_coalesces_pending_submissions(cuda):
    """With one launch in flight (inflight target 1), everything submitted
    meanwhile goes out as ONE planned descriptor launch; each ticket still
    gets exactly its own digests."""
    dl, pl, Ll, wl = _arena_batch([32 << 20] * 2, 9, cuda)            # keeps the device busy
    rng = np.random.default_rng(11)
    small = []
    for k in range(12):
        lens = [int(x) for x in rng.integers(0, 70000, int(rng.integers(1, 200)))]
        small.append(_arena_batch(lens, 100 + k, cuda))
    with m.Queue(device=0, nslots=4) as q:
        q.set_inflight(1)
        pa = q.submit_device_async(pl, Ll)
        pend = [q.submit_device_async(p, L) for _, p, L, _ in small]
        outs = [p.wait() for p in reversed(pend)]
        assert np.array_equal(pa.wait(), wl)
        st = q.stats()
    for got, (_, _, _, want) in zip(reversed(outs), small):
        assert np.array_equal(got, want)
    assert st["submissions"] == 13
    assert st["launches"] == 2, st
    assert st["coalesced_launches"] == 1 and st["max_tickets_per_launch"] == 12, st


def test_queue_mixed_host_and_device_chunks(cuda):
    """Host-memory and device-resident submissions interleaved on one queue,
    MD5 and (per-call) CRC-32 verify."""
    rng = np.random.default_rng(13)
    lens = [int(x) for x in rng.integers(0, 100000, 300)]
    dev, ptrs, L, want = _arena_batch(lens, 131, cuda)
    blob = gen.xorshift_bytes(sum(lens) + 1, seed=132)
    bufs, cur = [], 0
    for x in lens:
        bufs.append(blob[cur:cur + x])
        cur += x
    want_h = gen.oracle_digests(np.frombuffer(blob, dtype=np.uint8), np.cumsum([0] + lens[:-1]), lens)
    with m.Queue(device=0, nslots=3) as q:
        p1 = q.submit_device_async(ptrs, L)
        p2 = q.submit_async(bufs)
        p3 = q.submit_device_async(ptrs[::-1].copy(), L[::-1].copy())
        assert np.array_equal(p2.wait(), want_h)
        assert np.array_equal(p3.wait(), want[::-1])
        assert np.array_equal(p1.wait(), want)
        ok, bad = q.verify_iov([[b] for b in bufs], want_h)
        assert bad == 0 and ok.all()


def test_batcher_shared_by_threads(cuda):
    """One batcher, four submitting threads (the netcache ASIO pool sharing
    one instance), async host submissions waited in reverse order."""
    res = {}
    errs = []

    with m.Batcher(device=0, slice_bytes=4 << 20, nslots=4) as b:
        def worker(k):
            try:
                rng = np.random.default_rng(500 + k)
                items = []
                for j in range(6):
                    lens = [int(x) for x in rng.integers(0, 200000, 30)]
                    blob = gen.xorshift_bytes(sum(lens) + 1, seed=10 * k + j)
                    bufs, cur = [], 0
                    for x in lens:
                        bufs.append(blob[cur:cur + x])
                        cur += x
                    want = gen.oracle_digests(np.frombuffer(blob, dtype=np.uint8),
                                              np.cumsum([0] + lens[:-1]), lens)
                    items.append((b.submit_async(bufs), want))
                res[k] = all(np.array_equal(p.wait(), w) for p, w in reversed(items))
            except Exception as e:  # pragma: no cover - surfaced below
                errs.append(repr(e))

        th = [threading.Thread(target=worker, args=(k,)) for k in range(4)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        st = b.stats()
    assert not errs, errs
    assert res == {0: True, 1: True, 2: True, 3: True}
    assert st["submissions"] == 24


def test_batcher_keeps_its_kind_during_header_verify(cuda):
    """md5hip_batch_verify_headers hashes CRC-32 for that call only: a
    concurrent MD5 submission on the same batcher still gets MD5."""
    import struct
    from sproxy_amd import nc_digest as ncd
    hdrs = []
    for k in range(50):
        hs = 20 + 977 * k
        h = bytearray(struct.pack("<IiiII", ncd.NC_MAGIC_V30, 0, hs, 0, 0) + gen.xorshift_bytes(hs - 20, seed=k))
        ncd.header_seal(h)
        hdrs.append(h)
    lens = [70000] * 40
    blob = gen.xorshift_bytes(sum(lens) + 1, seed=3)
    bufs = [blob[i * 70000:(i + 1) * 70000] for i in range(40)]
    want = gen.oracle_digests(np.frombuffer(blob, dtype=np.uint8), np.arange(40) * 70000, lens)
    with m.Batcher(device=0, slice_bytes=4 << 20, nslots=3) as b:
        p = b.submit_async(bufs)
        ok, bad = ncd.verify_headers(b, hdrs)
        assert bad == 0 and all(ok)
        assert np.array_equal(p.wait(), want)
        assert np.array_equal(b.submit(bufs), want)


def test_arena_freed_right_after_async_launch(cuda):
    """md5hip_arena_free synchronizes the device before unmapping: dropping an
    arena tensor right after an asynchronous launch is safe, and a later batch
    is still correct."""
    import gc
    n, L = 4096, 16384
    for k in range(3):
        a = m.arena_empty(n * L)
        m.fill_synthetic(a, seed=70 + k)
        out = m.digest_fixed(a, n, L)                # async on the current stream
        del a
        gc.collect()                                  # frees the arena while the kernel may run
        torch.cuda.synchronize()
        host = gen.synthetic_bytes(n * L, 70 + k)
        assert np.array_equal(out.cpu().numpy(), gen.oracle_digests_fixed(host, n, L)), k


def test_balanced_on_coalesced_mixed_batches(cuda):
    """BALANCED (LPT over one wave per SIMD) on three coalesced C3-shaped
    batches: digests equal the oracle on a sample and the other descriptor
    kernels on the whole batch; two launches back to back on one stream reuse
    the self-resetting group counter.  (The planner's choice of BALANCED at
    the bench's sizes is tests/test_abi.py::test_planner_choices.)"""
    import sys
    sys.path.insert(0, gen.REPO)
    import bench
    lk = [bench.c3_lens(2 << 30, 70 + j) for j in range(3)]
    L = np.concatenate(lk)
    offs = np.concatenate([[0], np.cumsum((L + 15) // 16 * 16)[:-1]])
    total = int(offs[-1] + L[-1] + 64)
    data = torch.empty(total, dtype=torch.uint8, device=cuda)
    m.fill_synthetic(data[: total // 16 * 16], seed=0xBA1)
    order, _ = m.plan_desc(L.astype(np.uint32))
    args = (data, torch.from_numpy(offs).to(cuda), torch.from_numpy(L.astype(np.int32)).to(cuda),
            torch.from_numpy(order.astype(np.int32)).to(cuda))
    a = m.digest_desc(*args, variant="balanced")
    b = m.digest_desc(*args, variant="balanced")
    for v in ("xdma", "hybrid", "lane", "fed"):
        assert torch.equal(m.digest_desc(*args, variant=v), a), v
    assert torch.equal(a, b)
    idx = np.unique(np.concatenate([order[:300], order[-300:],
                                    np.random.default_rng(4).integers(0, L.size, 600)]))
    host = data.cpu().numpy()
    want = gen.oracle_digests(host, offs[idx], L[idx])
    assert np.array_equal(a.cpu().numpy()[idx], want)


def test_zero_copy_adjacent_registrations(cuda):
    """Two adjacent host ranges registered separately (two pinned
    allocations) and blocks whose pages run across the boundary: the DMA
    gather list never merges a copy over two registrations, and
    every gather mode returns the oracle digests."""
    buf = np.frombuffer(gen.xorshift_bytes(4 << 20, seed=77), np.uint8).copy()
    base = buf.ctypes.data
    cut = ((base + (2 << 20) + 4095) & ~4095) - base          # page-aligned split point
    lo, hi = buf[:cut], buf[cut:]
    page = 16384
    blocks = []
    for k in range(24):                                        # pages straddling the boundary
        s0 = cut - (k + 1) * 4096
        blocks.append([buf[s0:s0 + page], buf[s0 + page:s0 + 2 * page]])
    joined = [b"".join(x.tobytes() for x in segs) for segs in blocks]
    arena = np.frombuffer(b"".join(joined) + b"\0", np.uint8)
    lens = [len(j) for j in joined]
    want = gen.oracle_digests(arena, np.cumsum([0] + lens[:-1]), lens)
    m.register_host(lo)
    m.register_host(hi)
    try:
        with m.Batcher(device=0, slice_bytes=1 << 20, nslots=2) as b:
            for mode in (b.GATHER_DMA, b.GATHER_DEVICE, b.GATHER_AUTO, b.GATHER_HOST):
                b.set_gather(mode)
                assert np.array_equal(b.submit_iov(blocks), want), mode
                flat = [buf[cut - 3 * page: cut + 3 * page]]     # one segment over both ranges
                got = b.submit(flat)
                assert bytes(got[0]) == bytes(gen.oracle_digests(buf, [cut - 3 * page], [6 * page])[0])
    finally:
        m.unregister_host(lo)
        m.unregister_host(hi)


def test_queue_linger_turns_a_burst_into_one_launch(cuda):
    """With nothing in flight, asynchronous submissions arriving back to back
    are held for up to 1/8 of the recent launches' wall time (capped by
    md5hip_batcher_set_linger) and go out as ONE launch; with linger 0 the
    first of them is launched at once.  Digests per ticket either way."""
    dl, pl, Ll, wl = _arena_batch([64 << 20] * 2, 21, cuda)      # ~0.6 s of serial chains
    rng = np.random.default_rng(23)
    small = [_arena_batch([int(x) for x in rng.integers(0, 70000, 100)], 300 + k, cuda) for k in range(5)]
    with m.Queue(device=0, nslots=4) as q:
        q.set_linger(200000)
        assert np.array_equal(q.submit_device(pl, Ll), wl)        # sets the launch-time average
        n0 = q.stats()["launches"]
        pend = [q.submit_device_async(p, L) for _, p, L, _ in small]
        for pn, (_, _, _, want) in zip(pend, small):
            assert np.array_equal(pn.wait(), want)
        n1 = q.stats()["launches"]
        assert n1 == n0 + 1, (n0, n1)
        q.set_linger(0)
        pend = [q.submit_device_async(p, L) for _, p, L, _ in small]
        for pn, (_, _, _, want) in zip(pend, small):
            assert np.array_equal(pn.wait(), want)
        assert q.stats()["launches"] >= n1 + 2


def test_queue_concurrency_stress(cuda):
    """Eight threads on one queue for a few seconds: device-resident and host
    submissions, synchronous and asynchronous, tickets waited / polled in
    random order, while another thread keeps changing the inflight target
    and the linger -- every ticket's digests equal the oracle and every
    ticket completes (the coalescing, linger, plan-ahead and wait paths of
    md5_submit.c under contention)."""
    import time
    rng0 = np.random.default_rng(99)
    pool = []
    for k in range(6):
        lens = [int(x) for x in rng0.integers(0, 150000, int(rng0.integers(1, 120)))]
        pool.append(_arena_batch(lens, 900 + k, cuda, align=int(rng0.choice([1, 16, 128]))))
    hosts = []
    for k in range(4):
        lens = [int(x) for x in rng0.integers(0, 90000, int(rng0.integers(1, 60)))]
        blob = gen.xorshift_bytes(sum(lens) + 1, seed=950 + k)
        bufs, cur = [], 0
        for x in lens:
            bufs.append(blob[cur:cur + x])
            cur += x
        want = gen.oracle_digests(np.frombuffer(blob, dtype=np.uint8), np.cumsum([0] + lens[:-1]), lens)
        hosts.append((bufs, want))
    errs, done = [], []
    stop = time.time() + 6.0
    with m.Queue(device=0, nslots=4) as q:
        def worker(seed):
            rng = np.random.default_rng(seed)
            try:
                while time.time() < stop:
                    held = []
                    for _ in range(int(rng.integers(1, 6))):
                        if rng.random() < 0.7:
                            _, p, L, want = pool[int(rng.integers(0, len(pool)))]
                            if rng.random() < 0.2:
                                assert np.array_equal(q.submit_device(p, L), want)
                                done.append(1)
                            else:
                                held.append((q.submit_device_async(p, L), want))
                        else:
                            bufs, want = hosts[int(rng.integers(0, len(hosts)))]
                            held.append((q.submit_async(bufs), want))
                    rng.shuffle(held)
                    for pn, want in held:
                        if rng.random() < 0.3:
                            while not pn.poll():
                                time.sleep(0.0002)
                        assert np.array_equal(pn.wait(), want)
                        done.append(1)
            except Exception as e:  # pragma: no cover - surfaced below
                errs.append(repr(e))

        def knobs():
            rng = np.random.default_rng(5)
            while time.time() < stop:
                q.set_inflight(int(rng.integers(1, 5)))
                q.set_linger(int(rng.choice([0, 200, 5000])))
                time.sleep(0.05)

        th = [threading.Thread(target=worker, args=(s,)) for s in range(8)] + [threading.Thread(target=knobs)]
        for t in th:
            t.start()
        for t in th:
            t.join(timeout=120)
        st = q.stats()
    assert not errs, errs[:3]
    assert len(done) > 50 and st["submissions"] >= len(done), (len(done), st)


@pytest.mark.parametrize("chain", [0, 1, 2])
def test_queue_pipelined_stream_every_chain_mode(cuda, chain):
    """The c3q stream in miniature under each chain mode
    (md5hip_batcher_set_chain: 0 off, 1 kernel queued behind the running
    launch's event, 2 the same but BALANCED launches overlapping their
    tails): 4 C3-shaped vectors of 8 GiB per step -- coalesced, BALANCED's
    size -- 5 steps, step k submitted before step k-1 is waited for, digests
    into two alternating sets of device tensors.  Every digest of every step
    equals a separate XDMA launch over the same vector, and a sample of the
    oracle's."""
    import sys
    sys.path.insert(0, gen.REPO)
    import bench
    K = 4
    lk = [bench.c3_lens(8 << 30, 90 + j) for j in range(K)]
    _, var = m.plan_desc(np.concatenate(lk).astype(np.uint32))
    assert var == "balanced", var                  # the launches chain mode 2 overlaps
    spans = [int(((L + 15) // 16 * 16).sum()) for L in lk]
    starts = np.concatenate([[0], np.cumsum(spans)[:-1]]).astype(np.int64)
    data = m.arena_empty(int(sum(spans)) + 64)
    m.fill_synthetic(data, seed=0xC4A1)
    torch.cuda.synchronize()
    ref, subs = [], []
    for j, L in enumerate(lk):
        offs = starts[j] + np.concatenate([[0], np.cumsum((L + 15) // 16 * 16)[:-1]])
        ref.append(m.digest_desc(data, torch.from_numpy(offs).to(cuda),
                                 torch.from_numpy(L.astype(np.int32)).to(cuda), variant="xdma"))
        subs.append(((np.uint64(data.data_ptr()) + offs.astype(np.uint64)), L.astype(np.uint32)))
    # the oracle on the chunks of vector 0's first 256 MiB
    offs0 = np.concatenate([[0], np.cumsum((lk[0] + 15) // 16 * 16)[:-1]])
    near = np.nonzero(offs0 + lk[0] <= (256 << 20))[0]
    idx = np.unique(np.concatenate([near[:64], np.random.default_rng(9).choice(near, 200)]))
    host = data[: 256 << 20].cpu().numpy()
    want = gen.oracle_digests(host, offs0[idx], lk[0][idx])
    assert np.array_equal(ref[0].cpu().numpy()[idx], want)
    q = m.Queue(device=0, nslots=4, inflight=1)
    q.set_chain(chain)
    outs = [[torch.empty((L.size, 16), dtype=torch.uint8, device=cuda) for L in lk] for _ in range(2)]
    prev = None
    for k in range(5):
        cur = [q.submit_device_async(p, L, o) for (p, L), o in zip(subs, outs[k & 1])]
        if prev is not None:
            for pn in prev:
                pn.wait()
            for j in range(K):
                assert torch.equal(outs[(k - 1) & 1][j], ref[j]), (chain, k - 1, j)
        prev = cur
    for pn in prev:
        pn.wait()
    for j in range(K):
        assert torch.equal(outs[0][j], ref[j]), (chain, 4, j)
    st = q.stats()
    assert st["submissions"] == 5 * K and st["launches"] < st["submissions"], st


def test_queue_device_fixed_md5_and_fastcrc(cuda):
    """md5_batch_submit_device_fixed (ABI 4): fixed-length device-resident
    runs read in place, no per-chunk descriptor.  MD5 with host digests,
    in-place device digests and unaligned (scattered) device digests, a run
    longer than one slot (several launches), a stride wider than the
    length, ordering after a producer stream; CRC-32 whole and fastcrc
    windows (blk_io.c:408-424).  Every digest against the oracle."""
    n, L, S = 3000, 5000, 5120
    host = gen.xorshift_array(n * S + 64, seed=4242)
    offs = [i * S for i in range(n)]
    want = gen.oracle_digests(host, offs, [L] * n)
    dev = torch.from_numpy(host.copy()).to(cuda)
    with m.Queue(device=0, max_chunks=1024) as q:                      # 3 slots' worth
        got = q.submit_device_fixed_async(dev, n, L, S, after=None).wait()
        assert np.array_equal(got, want)
        out = torch.empty((n, 16), dtype=torch.uint8, device=cuda)
        q.submit_device_fixed_async(dev, n, L, S, out=out).wait()      # ordered after torch's stream
        assert np.array_equal(out.cpu().numpy(), want)
        raw = torch.zeros(n * 16 + 4, dtype=torch.uint8, device=cuda)
        odd = raw[4:].view(n, 16)
        q.submit_device_fixed_async(dev, n, L, S, out=odd).wait()
        assert np.array_equal(odd.cpu().numpy(), want)
        # the producer's write lands before the kernel reads it
        s = torch.cuda.Stream()
        with torch.cuda.stream(s):
            dev2 = torch.empty_like(dev)
            dev2.copy_(dev)
            pend = q.submit_device_fixed_async(dev2, n, L, S, after=s)
        assert np.array_equal(pend.wait(), want)
        for F in (0, 128, 4096):
            q.set_digest(m.Batcher.CRC32, F)
            crc = q.submit_device_fixed_async(dev, n, L, S, after=None).wait()
            assert np.array_equal(crc, gen.oracle_crc32_batch(host, offs, [L] * n, fastcrc=F)), F
        st = q.stats()
        # a run whose chunks start off the 16-B grid (base + 3, stride 5,001):
        # the kernels' unaligned paths, MD5 and CRC-32 whole and windowed
        n2, S2 = 2000, 5001
        offs2 = [3 + i * S2 for i in range(n2)]
        for kind, F in ((m.Batcher.MD5, 0), (m.Batcher.CRC32, 0), (m.Batcher.CRC32, 128)):
            q.set_digest(kind, F)
            got = q.submit_device_fixed_async(dev[3:], n2, L, S2, after=None).wait()
            want2 = gen.oracle_digests(host, offs2, [L] * n2) if kind == m.Batcher.MD5 else \
                gen.oracle_crc32_batch(host, offs2, [L] * n2, fastcrc=F)
            assert np.array_equal(got, want2), (kind, F)
    assert st["launches"] >= 3 * 7


def test_batcher_failure_policy_with_an_injected_fault(cuda):
    """INTEGRATION.md §2j on the GPU: the launch that faults gives its
    ticket -EIO and writes no digest; the batcher is failed from then on
    (-ENODEV at once, nothing launched); a pool over device 0 listed three
    times moves a synchronous submission off its failed member and never
    uses it again."""
    import errno
    rng = np.random.default_rng(99)
    lens = [int(x) for x in rng.integers(1, 40000, 64)]
    dev, ptrs, L, want = _arena_batch(lens, 991, cuda)
    host = [bytes(dev[int(p - dev.data_ptr()):int(p - dev.data_ptr()) + int(n)].cpu().numpy())
            for p, n in zip(ptrs, L)]
    with m.Queue(device=0) as q:
        assert np.array_equal(q.submit_device(ptrs, L), want) and q.health() == 0
        q.inject_fault(1)
        out = np.full((len(lens), 16), 0x5A, dtype=np.uint8)
        with pytest.raises(m.MD5HipError) as e:
            q.submit_device(ptrs, L, out=out)
        assert e.value.rc == -errno.EIO and (out == 0x5A).all()
        assert q.health() == -errno.ENODEV
        launches = q.stats()["launches"]
        with pytest.raises(m.MD5HipError) as e:
            q.submit(host)
        assert e.value.rc == -errno.ENODEV and q.stats()["launches"] == launches
    with m.Pool(devices=(0, 0, 0)) as p:
        p.set_split(64 << 10)                                          # every member takes a part
        p.inject_fault(1, 1)
        assert np.array_equal(p.submit(host), want)
        h = p.health()
        assert h["nfailed"] == 1 and h["failed_mask"] == 2 and h["failovers"] == 1, h
        before = p.device_stats(1)["submissions"]
        for _ in range(3):
            assert np.array_equal(p.submit(host), want)
        assert p.device_stats(1)["submissions"] == before
