"""The multi-GPU pool as a router over per-device coalescing batchers
(md5_pool.c, include/md5hip.h md5hip_pool_*).  On a node with more than one
GPU every pool spans distinct devices (all of them for the 8-thread router
test); on a one-GPU box the device is listed several times (each entry is its
own batcher, so routing, split tickets and digest placement still run).

The reference calls its block checksum from every ASIO thread at once
(asio_mgr.c:205, :1050-1057) with one vector of blocks each: here 8 threads
submit netcache-sized vectors concurrently; every ticket is checked against
the oracle, vectors go whole to one device and coalesce there.  Also: split
tickets above the threshold, poll/wait in any order, CRC-32, error returns,
and device-resident submissions ordered after the producer's stream."""
import threading

import numpy as np
import pytest
import torch

import gen
import sproxy_amd.md5 as m

pytestmark = pytest.mark.gpu

MT_BIT = 1 << 63


def _devs(k=None):
    """k pool entries: distinct devices when more than one is visible (every
    device for k None), else device 0 listed k times (4 for k None)."""
    ndev = torch.cuda.device_count()
    if ndev > 1:
        return tuple(range(ndev)) if k is None else tuple(g % ndev for g in range(k))
    return (0,) * (4 if k is None else k)


def _vectors(k, seed):
    """k netcache-like vectors: 64-1,024 blocks of 16 KiB, some last-block tails."""
    rng = np.random.default_rng(seed)
    out = []
    for j in range(k):
        nb = int(rng.integers(64, 1025))
        lens = [16384] * nb
        if j % 3 == 0:
            lens[-1] = int(rng.integers(1, 16384))                # blk_io.c:377 tail
        out.append(lens)
    return out


def _bufs(lens, seed):
    blob = gen.xorshift_array(sum(lens) + 1, seed=seed)
    offs = np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
    bufs = [blob[o:o + L] for o, L in zip(offs, lens)]
    return bufs, gen.oracle_digests(blob, offs, lens), blob, offs


def test_pool_router_eight_threads(cuda):
    """8 threads x 6 async vectors each through a pool over every device (or
    (0,0,0,0) on one GPU), the
    blocks in a registered page heap (zero-copy, as INTEGRATION.md asks of
    netcache): every ticket equals the oracle, every vector went whole to one
    device, every device took work, and vectors arriving while launches run
    were coalesced."""
    # vectors of 1 MiB blocks (chunk_size up to 10 MiB, httpd.c:7968): a launch
    # is at least one block's ~9 ms chain, so vectors from the other threads
    # arrive while launches run -- what coalescing needs, whatever the
    # Python-side cost of a submission
    rng = np.random.default_rng(301)
    vecs = []
    for j in range(48):
        lens = [1 << 20] * int(rng.integers(2, 9))
        if j % 3 == 0:
            lens[-1] = int(rng.integers(1, 1 << 20))                  # last-block tail
        vecs.append(lens)
    sizes = [sum(v) for v in vecs]
    heap = gen.xorshift_array(sum(sizes) + 64, seed=302)
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]]).astype(np.int64)
    data = []
    for j, lens in enumerate(vecs):
        offs = starts[j] + np.concatenate([[0], np.cumsum(lens)[:-1]]).astype(np.int64)
        data.append(([heap[o:o + L] for o, L in zip(offs, lens)], gen.oracle_digests(heap, offs, lens)))
    errors, results = [], {}
    m.register_host(heap)
    try:
        devs = _devs()
        with m.Pool(devs) as p:
            start = threading.Barrier(8)

            def worker(t):
                try:
                    start.wait()
                    mine = list(range(t, 48, 8))
                    pend = [(j, p.submit_async(data[j][0])) for j in mine]
                    for j, pn in reversed(pend):                  # any order
                        results[j] = pn.wait()
                except Exception as e:                            # pragma: no cover
                    errors.append(repr(e))

            th = [threading.Thread(target=worker, args=(t,)) for t in range(8)]
            for x in th:
                x.start()
            for x in th:
                x.join()
            assert not errors, errors
            for j in range(48):
                assert np.array_equal(results[j], data[j][1]), j
            st = p.stats()
            assert st["submissions"] == 48 and st["routed_whole"] == 48 and st["split"] == 0
            dev = [p.device_stats(g) for g in range(len(devs))]
            assert sum(d["submissions"] for d in dev) == 48
            assert all(d["submissions"] > 0 for d in dev), dev        # load spread
            assert sum(d["launches"] for d in dev) < 48, dev          # vectors coalesced
            assert sum(d["coalesced_launches"] for d in dev) > 0, dev
    finally:
        m.unregister_host(heap)
    # netcache-sized vectors of 16 KiB blocks from pageable memory (host
    # gather): correct, and whole
    small = [_bufs(lens, 600 + j) for j, lens in enumerate(_vectors(8, seed=303))]
    with m.Pool(_devs(2)) as p:
        pend = [p.submit_async(d[0]) for d in small]
        for d, pn in zip(small, pend):
            assert np.array_equal(pn.wait(), d[1])
        assert p.stats()["routed_whole"] == 8


def test_pool_sync_submit_from_threads(cuda):
    """Synchronous submits from several threads at once (the old pool
    serialized them under one mutex)."""
    vecs = _vectors(16, seed=311)
    data = [_bufs(lens, 500 + j) for j, lens in enumerate(vecs)]
    got, errors = {}, []
    with m.Pool(_devs(2)) as p:
        def worker(t):
            try:
                for j in range(t, 16, 4):
                    got[j] = p.submit(data[j][0])
            except Exception as e:                                # pragma: no cover
                errors.append(repr(e))
        th = [threading.Thread(target=worker, args=(t,)) for t in range(4)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    assert not errors, errors
    for j in range(16):
        assert np.array_equal(got[j], data[j][1]), j


def test_pool_split_tickets(cuda):
    """Above the split threshold a submission is cut over devices: its ticket
    is a split ticket (bit 63), complete only when every part is; waits and
    polls in any order, repeated waits, iov and host_fixed forms."""
    lens = gen.mixed_lengths(600, seed=321, max_len=1 << 18) + [0, 1, 64, 16384]
    bufs, want, blob, offs = _bufs(lens, 322)
    pages = [[b[:5000], b[5000:]] for b in bufs]
    with m.Pool(_devs(3), slice_bytes=8 << 20, nslots=3) as p:
        p.set_split(1 << 20)
        a = p.submit_async(bufs)
        b = p.submit_iov_async(pages)
        small = p.submit_async(bufs[:3])                       # < threshold: whole
        assert a.ticket & MT_BIT and b.ticket & MT_BIT and not small.ticket & MT_BIT
        assert np.array_equal(b.wait(), want)
        assert np.array_equal(small.wait(), want[:3])
        while not a.poll():
            pass
        assert np.array_equal(a.wait(), want)
        assert a.poll() and a.wait() is not None                   # done stays done
        st = p.stats()
        assert st["split"] == 2 and st["routed_whole"] == 1 and st["parts"] >= 2 + 2 + 1
        n, L = 2000, 16384
        host = gen.xorshift_array(n * L, seed=323)
        assert np.array_equal(p.host_fixed(host, n, L), gen.oracle_digests_fixed(host, n, L))
        p.set_split(0)                                             # one slice (8 MiB)
        assert np.array_equal(p.submit(bufs), want)


def test_pool_crc32_and_verify(cuda):
    lens = gen.mixed_lengths(300, seed=331, max_len=1 << 17)
    bufs, want, blob, offs = _bufs(lens, 332)
    pages = [[b] for b in bufs]
    with m.Pool(_devs(2)) as p:
        p.set_digest(m.Pool.CRC32, 0)
        got = p.submit_async(bufs).wait()
        assert np.array_equal(got, gen.oracle_crc32_batch(blob, offs, lens, 0))
        p.set_digest(m.Pool.CRC32, 128)
        assert np.array_equal(p.submit(bufs), gen.oracle_crc32_batch(blob, offs, lens, 128))
        p.set_digest(m.Pool.MD5, 0)
        bad = want.copy()
        bad[7] ^= 1
        ok, nbad = p.verify_iov(pages, bad)
        assert nbad == 1 and not ok[7] and ok.sum() == len(lens) - 1


def test_pool_ticket_errors(cuda):
    import ctypes
    import errno
    from sproxy_amd._lib import lib
    with m.Pool(_devs(2)) as p:
        L = lib()
        assert L.md5hip_pool_wait(p._h, 0) == 0 and L.md5hip_pool_poll(p._h, 0) == 1
        assert L.md5hip_pool_wait(p._h, (12345 << 6) | 1) == -errno.EINVAL     # never issued
        assert L.md5hip_pool_wait(p._h, (5 << 6) | 9) == -errno.EINVAL         # no device 9
        assert L.md5hip_pool_poll(p._h, MT_BIT | 77) == -errno.EINVAL
        t = ctypes.c_uint64(99)
        assert L.md5hip_pool_submit_async(p._h, None, None, 0, None, ctypes.byref(t)) == 0 and t.value == 0
        with pytest.raises(NotImplementedError):
            p.submit_device_async(np.zeros(1, np.uint64), np.zeros(1, np.uint32))


def test_pool_failed_submission_then_good_ones(cuda):
    """A submission the batchers refuse (a chunk larger than a slice: -E2BIG)
    fails alone -- whole or split, nothing left in flight -- and later
    tickets report their own results (the batcher keeps per-ticket errors,
    md5_tickets.h)."""
    import errno
    lens = [200000] * 40
    bufs, want, blob, offs = _bufs(lens, 361)
    big = bufs[:10] + [np.zeros(3 << 20, np.uint8)] + bufs[10:20]          # 3 MiB > 2 MiB slice
    with m.Pool(_devs(2), slice_bytes=2 << 20, nslots=2) as p:
        for split in (0, 1 << 20):
            p.set_split(split)
            with pytest.raises(m.MD5HipError) as ei:
                p.submit(big)
            assert ei.value.rc == -errno.E2BIG
            with pytest.raises(m.MD5HipError):
                p.submit_async(big)
            with pytest.raises(m.MD5HipError):
                p.submit_async([big[10]])                                       # whole
            pend = [p.submit_async(bufs[k:k + 10]) for k in range(0, 40, 10)]
            for k, pn in zip(range(0, 40, 10), pend):
                assert np.array_equal(pn.wait(), want[k:k + 10])
            assert np.array_equal(p.submit(bufs), want)


def test_device_submit_ordered_after_producer_stream(cuda):
    """md5_batch_submit_device_on: chunks written by a kernel still running on
    the producer's stream are hashed after it, with no host sync in between."""
    n, Lc = 4096, 16384
    host = gen.xorshift_array(n * Lc, seed=341)
    src = torch.from_numpy(host).to(cuda)
    torch.cuda.synchronize()
    want = gen.oracle_digests_fixed(host, n, Lc)
    side = torch.cuda.Stream(device=cuda)
    dst = torch.zeros_like(src)
    ptrs = np.arange(n, dtype=np.uint64) * np.uint64(Lc) + np.uint64(dst.data_ptr())
    lens = np.full(n, Lc, np.uint32)
    with m.Queue(device=0) as q:
        for rep in range(3):
            dst.zero_()
            torch.cuda.synchronize()
            with torch.cuda.stream(side):
                for _ in range(8):                                 # a long producer
                    dst.copy_(src)
                got = q.submit_device(ptrs, lens, after=side)
            assert np.array_equal(got, want), rep
        torch.cuda.synchronize()
        dst.zero_()
        torch.cuda.synchronize()
        with torch.cuda.stream(side):
            dst.copy_(src)
            out = torch.empty((n, 16), dtype=torch.uint8, device=cuda)
            pend = q.submit_device_async(ptrs, lens, out=out)      # after = current (side)
        pend.wait()
        assert np.array_equal(out.cpu().numpy(), want)


def test_device_submit_ordered_after_default_stream(cuda):
    """after='current' while torch's DEFAULT stream is current (handle 0):
    the kernel still runs after the producer's work on the null stream
    (md5_batch_submit_device_after, order=1).  Round 3 passed the 0 handle
    to md5_batch_submit_device_on, which reads NULL as "no ordering", and the
    batcher's non-blocking streams do not wait for the null stream: the
    kernel read the chunks before the producer wrote them."""
    n, Lc = 2048, 16384
    host = gen.xorshift_array(n * Lc, seed=343)
    src = torch.from_numpy(host).to(cuda)
    torch.cuda.synchronize()
    want = gen.oracle_digests_fixed(host, n, Lc)
    dst = torch.zeros_like(src)
    ptrs = np.arange(n, dtype=np.uint64) * np.uint64(Lc) + np.uint64(dst.data_ptr())
    lens = np.full(n, Lc, np.uint32)
    assert torch.cuda.current_stream(cuda).cuda_stream == 0, "torch's default stream is the null stream"
    with m.Queue(device=0) as q:
        for rep in range(3):
            dst.zero_()
            torch.cuda.synchronize()
            torch.cuda._sleep(20_000_000)          # a producer still busy on the null stream ...
            dst.copy_(src)                         # ... whose last step writes the chunks
            if rep < 2:
                got = q.submit_device(ptrs, lens)              # after = current = default
            else:
                out = torch.empty((n, 16), dtype=torch.uint8, device=cuda)
                q.submit_device_async(ptrs, lens, out=out).wait()
                got = out.cpu().numpy()
            assert np.array_equal(got, want), rep
        # after=None is still "no ordering": the caller synchronizes first
        torch.cuda.synchronize()
        assert np.array_equal(q.submit_device(ptrs, lens, after=None), want)


def test_queue_crc32_device_submit(cuda):
    """A CRC-32 queue returns (n,) u32 digests from device submissions; a
    wrong-sized or foreign `out` is rejected before any device work."""
    lens = gen.mixed_lengths(200, seed=351, max_len=1 << 16)
    offs, total = gen.pack_offsets(lens, align=16)
    host = gen.xorshift_array(total + 64, seed=352)
    dev = torch.from_numpy(host).to(cuda)
    ptrs = np.asarray(offs, np.uint64) + np.uint64(dev.data_ptr())
    L = np.asarray(lens, np.uint32)
    want = gen.oracle_crc32_batch(host, offs, lens, 0)
    with m.Queue(device=0) as q:
        q.set_digest(m.Queue.CRC32, 0)
        assert np.array_equal(q.submit_device(ptrs, L), want)
        assert np.array_equal(q.submit_device_async(ptrs, L).wait(), want)
        out = torch.empty(len(lens), dtype=torch.int32, device=cuda)
        q.submit_device(ptrs, L, out=out)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), want)
        with pytest.raises(ValueError):
            q.submit_device(ptrs, L, out=np.empty((len(lens), 2), np.uint8))   # too small
        with pytest.raises(ValueError):
            q.submit_device(ptrs, L, out=np.empty(len(lens) * 4, np.int8))     # wrong dtype
        with pytest.raises(ValueError):
            q.submit_device(ptrs, L, out=torch.empty(len(lens) - 1, dtype=torch.int32, device=cuda))
