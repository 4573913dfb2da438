"""bench.py's launch contract on CPU (no GPU): `--gpus N` without a launcher
starts N ranks itself (torch.distributed.run as a child process) and the line
reports them; a WORLD_SIZE that disagrees with --gpus is an error, never a
silent one-rank run (VERDICT r1 "What's missing" 1)."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, "bench.py")


def _run(args, env_extra=None, timeout=300):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(env_extra or {})
    return subprocess.run([sys.executable, BENCH, *args], capture_output=True, text=True,
                          timeout=timeout, env=env, cwd=REPO)


def _line(stdout):
    lines = [ln for ln in stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, stdout
    return json.loads(lines[0])


def test_gpus2_spawns_two_ranks():
    r = _run(["--gpus", "2", "--dist-backend", "gloo", "--dry-run", "--steps", "1", "--warmup", "0",
              "--chunks", "16"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 2
    assert d["ranks_seen"]["world"] == 2
    assert sorted(x["rank"] for x in d["ranks_seen"]["ranks"]) == [0, 1]
    assert len(d["per_gpu"]) == 2 and all(v > 0 for v in d["per_gpu"])
    assert d["parity"]["ok"] and d["parity"]["checked"] == 32
    assert d["config"]["parallelism"].startswith("dp2")


def test_gpus1_is_one_rank():
    r = _run(["--dry-run", "--steps", "1", "--warmup", "0", "--chunks", "8"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["ranks_seen"]["world"] == 1 and len(d["per_gpu"]) == 1


def test_world_size_mismatch_fails():
    r = _run(["--gpus", "2", "--dry-run", "--steps", "1", "--warmup", "0"],
             env_extra={"WORLD_SIZE": "3", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=3" in r.stderr
    assert not [ln for ln in r.stdout.splitlines() if ln.startswith("{")]


def test_dist_always_brings_up_a_one_rank_group():
    """--dist-always: the control plane (init, barrier, MAX, object gathers)
    runs even at one rank -- the rehearsal of the RCCL path on a one-GPU box."""
    r = _run(["--gpus", "1", "--dist-always", "--dist-backend", "gloo", "--dry-run", "--steps", "1",
              "--warmup", "0", "--chunks", "16"])
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 1 and d["ranks_seen"]["backend"] == "gloo" and d["ranks_seen"]["world"] == 1


def test_gpus8_dry_run():
    """The 8-rank path end to end on the CPU: spawn, 8
    distinct ranks, 8 per-rank rates and parity samples, rank-0 aggregation,
    and the workload named as the C4 shard the device run would hash."""
    r = _run(["--gpus", "8", "--dist-backend", "gloo", "--dry-run", "--steps", "1", "--warmup", "0",
              "--chunks", "8"], timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    d = _line(r.stdout)
    assert d["n_gpus"] == 8 and d["ranks_seen"]["world"] == 8
    assert sorted(x["rank"] for x in d["ranks_seen"]["ranks"]) == list(range(8))
    assert len(d["per_gpu"]) == 8 and all(v > 0 for v in d["per_gpu"])
    assert d["parity"]["ok"] and d["parity"]["checked"] == 64
    assert "C4 shard: 2,097,152 x 16 KiB chunks per GPU, 16,777,216 on 8 GPU(s)" in d["config"]["workload"]
    assert d["config"]["parallelism"].startswith("dp8")
