"""N>1 path on CPU: world_size-2 gloo groups exercise the same sharding and
timing aggregation bench.py uses under RCCL (sproxy_amd/shard.py)."""
import os
import socket
import time

import numpy as np
import torch.multiprocessing as mp

import gen
from sproxy_amd.shard import aggregate_rate, barrier, max_over_ranks, shard_range


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        # 1. each rank digests its shard of a fixed-length batch with the oracle
        n, L = 37, 1000
        buf = gen.xorshift_array(n * L, seed=4242)
        lo, hi = shard_range(n, rank, world)
        dig = gen.oracle_digests_fixed(buf[lo * L:hi * L], hi - lo, L)
        # 2. timing: ranks take different times; the job time is the max
        barrier(world)
        t0 = time.perf_counter()
        time.sleep(0.05 * (rank + 1))
        dt = time.perf_counter() - t0
        barrier(world)
        agg = aggregate_rate((hi - lo) * L, dt, world)
        q.put((rank, lo, hi, dig.tobytes(), dt, max_over_ranks(dt, world), agg))
    finally:
        dist.destroy_process_group()


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
    assert tmax >= 0.1 - 1e-3
    np.testing.assert_array_less(0, [r[4] for r in res])
