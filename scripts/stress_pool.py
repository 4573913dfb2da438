#!/usr/bin/env python3
"""Randomized stress of the call-site paths for --secs seconds: T threads on
one pool (over D batchers of device 0) and one device queue, each thread
choosing at random per step among
  pool submit / submit_async (+wait later, any order) / submit_iov(_async) /
  verify_iov with one flipped digest / host_fixed,
  queue submit_device(_async) with host or device digests, ordered after
  the thread's own torch stream, and the same through a CRC-32 queue
  (blk_make_crc digests; small and long-block vectors pick the split kernel),
  device-resident fixed-length runs on the queue (md5_batch_submit_device_fixed,
  host or device digests), fastcrc = 128 page lists through a CRC-32
  batcher that stages only each block's windows, and vectors past 4,096
  chunks (device-resident on the queue, and <= 1 KiB host chunks on the pool),
  whose slots take the stable device order (md5hip_order_device_stable),
over random vectors (1-300 chunks, 0 B - 1 MiB, tails, zero-length) cut from
a registered page heap or from pageable memory.  Every digest is checked
against digests the oracle computed up front.  Prints one JSON summary; exits
non-zero on the first mismatch or error.
usage: stress_pool.py [--secs 60] [--threads 12] [--devices 3]"""
import argparse
import json
import os
import random
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import gen  # noqa: E402


def _flat(got, exp):
    """A CRC ticket's result as uint32 values like its expectation."""
    got = np.asarray(got.cpu() if hasattr(got, "cpu") else got)
    return got.view(np.uint32).reshape(-1) if exp.dtype == np.uint32 else got


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--secs", type=float, default=60.0)
    ap.add_argument("--threads", type=int, default=12)
    ap.add_argument("--devices", type=int, default=3)
    a = ap.parse_args()
    import torch
    from sproxy_amd import md5 as m

    # a pool of chunks with known digests: (offset, length) into one heap
    rng = np.random.default_rng(2026)
    nchunks = 6000
    classes = [0, 1, 63, 64, 65, 4096, 16384, 16384, 16384, 65536, 262144, 1 << 20]
    lens = [int(rng.choice(classes)) if rng.random() < 0.7 else int(rng.integers(0, 70000))
            for _ in range(nchunks)]
    offs, total = gen.pack_offsets(lens, align=16)
    heap = gen.xorshift_array(total + 64, seed=77)
    want = gen.oracle_digests(heap, offs, lens)
    want_crc = gen.oracle_crc32_batch(heap, offs, lens)
    small = [i for i in range(nchunks) if lens[i] <= 1024]   # 9,000 of them stay under the 8 MiB split
    pageable = heap.copy()                      # the same bytes, never registered
    dev = torch.from_numpy(heap).cuda()
    torch.cuda.synchronize()
    m.register_host(heap)
    pool = m.Pool(tuple([0] * a.devices), slice_bytes=32 << 20, nslots=3)
    pool.set_split(8 << 20)
    q = m.Queue(device=0, max_chunks=1 << 16)
    qc = m.Queue(device=0, max_chunks=1 << 16)    # CRC-32 (blk_make_crc) through its own queue
    qc.set_digest(m.Batcher.CRC32)
    F = 128
    fb = m.Batcher(device=0, slice_bytes=8 << 20, nslots=3, kind=m.Batcher.CRC32, fastcrc=F)
    want_fast = gen.oracle_crc32_batch(heap, offs, lens, F)
    stop = time.perf_counter() + a.secs
    counts, errors = {}, []
    lock = threading.Lock()

    def note(k):
        with lock:
            counts[k] = counts.get(k, 0) + 1

    def worker(t):
        r = random.Random(1000 + t)
        stream = torch.cuda.Stream()
        held = []
        try:
            while time.perf_counter() < stop and not errors:
                k = r.randint(1, 300)
                idx = [r.randrange(nchunks) for _ in range(k)]
                src = heap if r.random() < 0.6 else pageable
                bufs = [src[offs[i]:offs[i] + lens[i]] for i in idx]
                exp = want[idx]
                op = r.choice(["sync", "async", "iov", "iov_async", "verify", "qdev", "qdev_async", "fixed",
                               "crc_qdev", "crc_qdev_async", "qfixed", "fastcrc_iov", "qdev_big", "many_small"])
                if op == "qdev_big":              # past 4,096 chunks: the stable device order (ABI 5)
                    k = r.randint(4097, 20000)
                    idx = [r.randrange(nchunks) for _ in range(k)]
                    exp = want[idx]
                elif op == "many_small":          # a host vector past 4,096 chunks of <= 1 KiB
                    k = r.randint(4097, 9000)
                    idx = [small[r.randrange(len(small))] for _ in range(k)]
                    bufs = [src[offs[i]:offs[i] + lens[i]] for i in idx]
                    exp = want[idx]
                if op == "sync":
                    assert np.array_equal(pool.submit(bufs), exp), op
                elif op == "async":
                    held.append((pool.submit_async(bufs), exp))
                elif op == "iov":
                    pages = [[b[:5000], b[5000:]] for b in bufs]
                    assert np.array_equal(pool.submit_iov(pages), exp), op
                elif op == "iov_async":
                    pages = [[b[:333], b[333:]] for b in bufs]
                    held.append((pool.submit_iov_async(pages), exp))
                elif op == "verify":
                    bad = exp.copy()
                    j = r.randrange(k)
                    bad[j, 0] ^= 1
                    ok, nbad = pool.verify_iov([[b] for b in bufs], bad)
                    assert nbad == 1 and not ok[j], op
                elif op == "many_small":
                    assert np.array_equal(pool.submit(bufs), exp), op
                elif op == "qdev_big":
                    ptrs = np.asarray([dev.data_ptr() + offs[i] for i in idx], np.uint64)
                    L = np.asarray([lens[i] for i in idx], np.uint32)
                    with torch.cuda.stream(stream):
                        if r.random() < 0.5:
                            assert np.array_equal(q.submit_device(ptrs, L), exp), op
                        else:
                            held.append((q.submit_device_async(ptrs, L), exp))
                elif op in ("qdev", "qdev_async"):
                    ptrs = np.asarray([dev.data_ptr() + offs[i] for i in idx], np.uint64)
                    L = np.asarray([lens[i] for i in idx], np.uint32)
                    with torch.cuda.stream(stream):
                        if op == "qdev":
                            out = torch.empty((k, 16), dtype=torch.uint8, device="cuda") if r.random() < 0.5 else None
                            got = q.submit_device(ptrs, L, out=out)
                            if out is not None:
                                torch.cuda.synchronize()
                                got = out.cpu().numpy()
                            assert np.array_equal(got, exp), op
                        else:
                            held.append((q.submit_device_async(ptrs, L), exp))
                elif op in ("crc_qdev", "crc_qdev_async"):
                    ptrs = np.asarray([dev.data_ptr() + offs[i] for i in idx], np.uint64)
                    L = np.asarray([lens[i] for i in idx], np.uint32)
                    ec = want_crc[idx]
                    with torch.cuda.stream(stream):
                        if op == "crc_qdev":
                            got = np.asarray(qc.submit_device(ptrs, L)).view(np.uint32).reshape(-1)
                            assert np.array_equal(got, ec), op
                        else:
                            held.append((qc.submit_device_async(ptrs, L), ec))
                elif op == "qfixed":
                    n = r.randint(1, 64)
                    Lf = r.choice([64, 4096, 16384])
                    S = Lf + r.choice([0, 0, 64, 128])
                    j = r.randrange(0, (total - n * S) // 64) * 64
                    exp2 = gen.oracle_digests(heap, [j + i * S for i in range(n)], [Lf] * n)
                    with torch.cuda.stream(stream):
                        out = torch.empty((n, 16), dtype=torch.uint8, device="cuda") if r.random() < 0.5 else None
                        pend = q.submit_device_fixed_async(dev[j:], n, Lf, S, out=out)
                    got = pend.wait()
                    if out is not None:
                        torch.cuda.synchronize()
                        got = out.cpu().numpy()
                    assert np.array_equal(np.asarray(got), exp2), op
                elif op == "fastcrc_iov":
                    pages = []
                    for b in bufs:
                        c1 = r.randint(0, len(b))
                        pages.append([b[:c1], b[c1:]])
                    got = np.asarray(fb.submit_iov(pages)).reshape(-1)
                    assert np.array_equal(got, want_fast[idx]), op
                else:
                    j = r.randrange(nchunks - 40)
                    n = r.randint(1, 40)
                    Lf = r.choice([64, 4096, 16384])
                    base = heap[:((total // Lf) * Lf)]
                    stride_chunks = base.size // Lf
                    j = min(j, stride_chunks - n)
                    got = pool.host_fixed(base[j * Lf:(j + n) * Lf], n, Lf)
                    exp2 = gen.oracle_digests(heap, [(j + i) * Lf for i in range(n)], [Lf] * n)
                    assert np.array_equal(got, exp2), op
                note(op)
                if len(held) > 6 or (held and r.random() < 0.3):
                    h, e = held.pop(r.randrange(len(held)))
                    assert np.array_equal(_flat(h.wait(), e), e), "held"
            for h, e in held:
                assert np.array_equal(_flat(h.wait(), e), e), "held"
        except Exception as ex:                      # pragma: no cover
            with lock:
                errors.append(f"thread {t}: {ex!r}")

    th = [threading.Thread(target=worker, args=(t,)) for t in range(a.threads)]
    t0 = time.perf_counter()
    for x in th:
        x.start()
    for x in th:
        x.join()
    wall = time.perf_counter() - t0
    st = pool.stats()
    dstats = [pool.device_stats(g) for g in range(a.devices)]
    qst = q.stats()
    qcst = qc.stats()
    pool.close()
    q.close()
    qc.close()
    fst = fb.stats()
    fb.close()
    m.unregister_host(heap)
    print(json.dumps({"secs": round(wall, 1), "threads": a.threads, "ops": counts,
                      "pool": st, "pool_device_launches": [d["launches"] for d in dstats],
                      "pool_coalesced": [d["coalesced_launches"] for d in dstats],
                      "queue": {k: qst[k] for k in ("submissions", "launches", "coalesced_launches")},
                      "crc_queue": {k: qcst[k] for k in ("submissions", "launches", "coalesced_launches")},
                      "fastcrc_batcher": {k: fst[k] for k in ("submissions", "launches", "bytes_staged")},
                      "errors": errors}))
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main())
