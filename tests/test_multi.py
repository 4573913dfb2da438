"""N>1 path on CPU: world_size-2 gloo groups run the control plane bench.py
itself runs (sproxy_amd/shard.py: init_group, barrier, MAX/SUM, object
gathers, close_group) and its sharding."""
import os
import socket
import time

import numpy as np
import torch.multiprocessing as mp

import gen
from sproxy_amd.shard import (aggregate_rate, barrier, close_group, gather_objects, group_on, init_group,
                              max_over_ranks, shard_range)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    assert init_group(world, "gloo") and group_on()
    try:
        # 1. each rank digests its shard of a fixed-length batch with the oracle
        n, L = 37, 1000
        buf = gen.xorshift_array(n * L, seed=4242)
        lo, hi = shard_range(n, rank, world)
        dig = gen.oracle_digests_fixed(buf[lo * L:hi * L], hi - lo, L)
        # 2. timing: ranks take different times; the job time is the max
        barrier()
        t0 = time.perf_counter()
        time.sleep(0.05 * (rank + 1))
        dt = time.perf_counter() - t0
        barrier()
        agg = aggregate_rate((hi - lo) * L, dt)
        seen = gather_objects({"rank": rank, "lo": lo})           # bench.py's per-rank line
        q.put((rank, lo, hi, dig.tobytes(), dt, max_over_ranks(dt), agg, seen))
    finally:
        close_group()


def test_shard_range_partitions():
    for n in (0, 1, 7, 64, 1 << 20, 16777216):
        for w in (1, 2, 3, 4, 8):
            spans = [shard_range(n, r, w) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(spans, spans[1:]))
            sizes = [h - lo for lo, h in spans]
            assert max(sizes) - min(sizes) <= 1


def test_gloo_world2_shards_and_max_time():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    n, L = 37, 1000
    buf = gen.xorshift_array(n * L, seed=4242)
    whole = gen.oracle_digests_fixed(buf, n, L).tobytes()
    assert b"".join(r[3] for r in res) == whole           # shards tile the batch exactly
    assert [(r[1], r[2]) for r in res] == [(0, 18), (18, 37)]
    tmax = max(r[4] for r in res)
    for r in res:
        assert abs(r[5] - tmax) < 1e-12                    # every rank sees the same max
        agg = r[6]
        assert agg["total_bytes"] == n * L
        assert abs(agg["bytes_per_s"] - n * L / tmax) < 1e-6 * n * L / tmax
        assert r[7] == [{"rank": 0, "lo": 0}, {"rank": 1, "lo": 18}]   # rank order, every rank
    assert tmax >= 0.1 - 1e-3
    np.testing.assert_array_less(0, [r[4] for r in res])


def test_no_group_is_one_rank():
    """Without a group (one rank, no --dist-always) every call is local."""
    assert not init_group(1, "gloo")
    assert not group_on()
    barrier()
    assert max_over_ranks(2.5) == 2.5 and gather_objects("x") == ["x"]
    assert aggregate_rate(10, 2.0)["bytes_per_s"] == 5.0
    close_group()
