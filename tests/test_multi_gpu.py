"""The multi-GPU code on distinct devices.  The first three
tests need more than one visible GPU and skip cleanly on a one-GPU box; on
a node with several they run

  * bench.py --gpus N (N = min(devices, 8)) as the driver does: N ranks on N
    distinct devices, every rank's rate and parity sample in the line;
  * one queue per device, each fed device-resident chunks that live on its
    own GPU, from a thread per device at once -- every digest against the
    oracle, and no call leaves the caller's current device changed;
  * a pool over every device, called from several threads whose current
    device differs: digests right, every device took work, the callers'
    current devices untouched (md5_submit.c dev_enter/dev_leave).

The reference calls its checksum from every ASIO pool thread at once
(netcache/common/asio_mgr.c:205, :1414).  The last test runs anywhere: a
device index past the last visible one is refused at creation."""
import json
import os
import subprocess
import sys
import threading

import numpy as np
import pytest
import torch

import gen
from sproxy_amd import md5 as m

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ndev():
    return torch.cuda.device_count() if torch.cuda.is_available() else 0


needs_two = pytest.mark.skipif(_ndev() < 2, reason="needs more than one GPU (one-GPU box)")


@needs_two
def test_bench_ranks_on_distinct_devices():
    n = min(_ndev(), 8)
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", str(n), "--steps", "2",
                        "--warmup", "1"], capture_output=True, text=True, timeout=600, env=env, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["ranks_seen"]["world"] == n
    assert d["ranks_seen"]["distinct_devices"] == n
    assert sorted(x["device"] for x in d["ranks_seen"]["ranks"]) == list(range(n))
    assert len(d["per_gpu"]) == n and all(v > 0 for v in d["per_gpu"])
    assert d["parity"]["ok"] and d["parity"]["checked"] >= 4096 * n


@needs_two
def test_queue_per_device_from_threads():
    ndev = _ndev()
    n, L = 3000, 16384
    host = gen.xorshift_array(n * L, seed=0x61)
    want = gen.oracle_digests_fixed(host, n, L)
    errors, got = [], {}

    def worker(g):
        try:
            torch.cuda.set_device((g + 1) % ndev)              # the caller sits on another device
            src = torch.from_numpy(host).to(f"cuda:{g}")
            torch.cuda.synchronize(g)
            ptrs = np.arange(n, dtype=np.uint64) * np.uint64(L) + np.uint64(src.data_ptr())
            lens = np.full(n, L, np.uint32)
            with m.Queue(device=g) as q:
                a = q.submit_device(ptrs, lens, after=None)
                out = torch.empty((n, 16), dtype=torch.uint8, device=f"cuda:{g}")
                q.submit_device_fixed_async(src, n, L, out=out, after=None).wait()
                got[g] = (a, out.cpu().numpy())
            assert torch.cuda.current_device() == (g + 1) % ndev
        except Exception as e:                                  # pragma: no cover
            errors.append(f"device {g}: {e!r}")

    th = [threading.Thread(target=worker, args=(g,)) for g in range(ndev)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    assert not errors, errors
    for g in range(ndev):
        assert np.array_equal(got[g][0], want), g
        assert np.array_equal(got[g][1], want), g


@needs_two
def test_pool_over_every_device_from_threads():
    ndev = _ndev()
    rng = np.random.default_rng(0x62)
    vecs = [[16384] * int(rng.integers(64, 513)) for _ in range(4 * ndev)]
    blobs = [gen.xorshift_array(sum(v), seed=0x6200 + j) for j, v in enumerate(vecs)]
    wants = [gen.oracle_digests_fixed(b, len(v), 16384) for b, v in zip(blobs, vecs)]
    errors, got = [], {}
    with m.Pool(tuple(range(ndev)), slice_bytes=16 << 20, nslots=3) as p:
        def worker(t):
            try:
                torch.cuda.set_device(t % ndev)
                mine = range(t, len(vecs), 2 * ndev)
                pend = [(j, p.submit_async([blobs[j][k * 16384:(k + 1) * 16384] for k in range(len(vecs[j]))]))
                        for j in mine]
                for j, pn in pend:
                    got[j] = pn.wait()
                host = blobs[t]
                got[("fixed", t)] = p.host_fixed(host, len(vecs[t]), 16384)
                assert torch.cuda.current_device() == t % ndev
            except Exception as e:                              # pragma: no cover
                errors.append(f"thread {t}: {e!r}")

        th = [threading.Thread(target=worker, args=(t,)) for t in range(2 * ndev)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errors, errors
        dev = [p.device_stats(g) for g in range(ndev)]
    for j in range(len(vecs)):
        assert np.array_equal(got[j], wants[j]), j
    for t in range(2 * ndev):
        assert np.array_equal(got[("fixed", t)], wants[t]), t
    assert all(d["launches"] > 0 for d in dev), dev


def test_a_device_past_the_last_is_refused(cuda):
    """Runs on any box: a pool or batcher naming a device index past the last
    visible one fails with -ENODEV at creation (md5_submit.c dev_enter), frees
    what it had built, leaves the caller's current device as it was, and
    leaves no sticky HIP error for torch's next launch check."""
    import errno
    ndev = _ndev()
    torch.cuda.set_device(0)
    for make in (lambda: m.Batcher(device=ndev), lambda: m.Queue(device=ndev),
                 lambda: m.Pool((0, ndev)), lambda: m.Pool((ndev,) * 2)):
        with pytest.raises(m.MD5HipError) as ei:
            make()
        assert ei.value.rc == -errno.ENODEV
        assert torch.cuda.current_device() == 0
        # no sticky HIP error left behind for torch's next launch check
        assert float((torch.ones(1024, device="cuda") * 2).sum().item()) == 2048.0
    with m.Pool((0,)) as p:                          # the library still works afterwards
        host = gen.xorshift_array(64 * 4096, seed=0x63)
        assert np.array_equal(p.host_fixed(host, 64, 4096), gen.oracle_digests_fixed(host, 64, 4096))
