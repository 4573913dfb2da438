#!/usr/bin/env python3
"""bench.py -- device-resident batched MD5 throughput on MI355X.

Metric (BASELINE.json): device-resident MD5 GiB/s on batched 16 KiB chunks.
A "step" = one pass of the batched-MD5 kernel over the rank's whole batch
(default 1,048,576 x 16 KiB = 16 GiB, BASELINE config C2), inputs already in
HBM (filled on the device by md5hip_fill_synthetic, per-rank seed).

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c5|crc]

N > 1: one process per GPU (torch.distributed.run); each rank hashes its own
shard of independent chunks (weak scaling, no data-path collective); barrier +
device sync bracket the K timed steps and the MAX time over ranks is used.
Rank 0 prints ONE JSON line.  The cpu_baseline leg (rank 0, N=1 only) runs the
reference md5.c (oracle/_ref, else the oracle port) on the C1 sample; it is the
only use of oracle/ here.
"""
import argparse
import json
import os
import platform
import subprocess
import sys
import time

import torch

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)
from sproxy_amd import md5 as m  # noqa: E402
from sproxy_amd.shard import barrier, env_rank, max_over_ranks, shard_range  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PCIE_PEAK_GBS = 63.0           # PCIe Gen5 x16 (spec)
METRIC = "device-resident MD5 GiB/s on batched 16 KiB chunks at 1/2/4/8 MI355X"
GIB = float(1 << 30)


COLL_DEVICE = "cuda"             # where the control-plane scalars live (cpu under gloo)


def dist_setup(ngpus, backend="nccl"):
    """One process per GPU.  The only collectives are a barrier and one scalar
    MAX, so `--dist-backend gloo` (CPU) is equivalent; it lets N ranks share
    one GPU for a rehearsal of the N > 1 path on a one-GPU box."""
    global COLL_DEVICE
    rank, world, local = env_rank()
    if world != ngpus and world > 1:
        raise SystemExit(f"--gpus {ngpus} but WORLD_SIZE={world}")
    ndev = torch.cuda.device_count()
    if backend == "nccl" and world > 1 and local >= ndev:
        raise SystemExit(f"LOCAL_RANK {local} but only {ndev} GPUs visible")
    torch.cuda.set_device(local % ndev)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
            COLL_DEVICE = "cpu"
    return rank, world, local


def timed_steps(fn, steps, warmup, world):
    """W untimed steps, then exactly K steps between barrier+sync pairs.
    Returns (wall seconds for K steps, avg device ms per step from HIP events
    recorded on the stream the kernels run on)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    barrier(world)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    barrier(world)
    return t1 - t0, e0.elapsed_time(e1) / steps


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


CPU_SHARE = 16      # host cores a one-GPU box grants a job (the box's CPU share)


def cpu_baseline(reps=10, threads=1):
    """Host md5.c on the C1 sample: 65,536 x 16 KiB xorshift64,
    Init/Update/Final per chunk, `threads` threads over disjoint chunk ranges,
    median of `reps`."""
    ref = os.path.join(REPO, "oracle", "_ref", "md5_cpu_bench")
    port = os.path.join(REPO, "oracle", "_build", "md5_cpu_bench_port")
    exe, kind = (ref, "reference") if os.path.exists(ref) else (port, "port")
    if not os.path.exists(exe):
        return None
    out = subprocess.run([exe, "65536", "16384", str(reps), str(threads)], capture_output=True,
                         text=True, timeout=600, check=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    return {"value": round(r["gib_s"], 4), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": (f"C1: 65,536 x 16 KiB xorshift64 (1 GiB), MD5Init/Update/Final per chunk, "
                       f"median of {reps}, {threads} thread(s) of {cpu_model()} "
                       f"({os.cpu_count()} logical CPUs); fold {r['fold']} (expect 53a0a616)"),
            "fold_ok": r["fold"] == "53a0a616"}


def cpu_baseline_crc(reps=7):
    """Host netcache crc32_8bytes (crc32.c, compiled in place) per chunk on the
    C1 sample, 1 thread, median of `reps` (fold ad5b15d5 = reference == port)."""
    ref = os.path.join(REPO, "oracle", "_ref", "crc32_cpu_bench")
    port = os.path.join(REPO, "oracle", "_build", "crc32_cpu_bench_port")
    exe, kind = (ref, "reference") if os.path.exists(ref) else (port, "port")
    if not os.path.exists(exe):
        return None
    out = subprocess.run([exe, "65536", "16384", str(reps), "1"], capture_output=True, text=True,
                         timeout=600, check=True).stdout
    r = json.loads(out.strip().splitlines()[-1])
    return {"value": round(r["gib_s"], 4), "unit": "GiB/s", "cores": 1, "kind": kind,
            "sample": (f"C1 shape: 65,536 x 16 KiB xorshift64 (1 GiB), crc32_8bytes per chunk "
                       f"(blk_make_crc, fastcrc 0), median of {reps}, 1 thread of {cpu_model()}; "
                       f"fold {r['fold']} (expect ad5b15d5)"),
            "fold_ok": r["fold"] == "ad5b15d5"}


def load_traffic(path, variant):
    """HBM bytes per launch from a committed rocprofv3 PMC summary (profiles/)."""
    if not path or not os.path.exists(path):
        return None
    try:
        d = json.load(open(path))
        return d.get(variant, d.get("default"))
    except Exception:
        return None


def run_c2(a, rank, world):
    L = a.len
    if a.total_chunks:       # strong / C4 form: one global batch split into contiguous shards
        lo, hi = shard_range(a.total_chunks, rank, world)
        n = hi - lo
    else:                    # weak scaling: a fixed per-GPU batch (C2 shape on every GPU)
        n = a.chunks
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0x5EED0000 + rank)
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    variant = m.VARIANTS[a.variant]
    fn = lambda: m.digest_fixed(data, n, L, out=out, variant=variant)  # noqa: E731
    wall, dev_ms = timed_steps(fn, a.steps, a.warmup, world)
    wall_max = max_over_ranks(wall, world, COLL_DEVICE)
    dev_ms_max = max_over_ranks(dev_ms, world, COLL_DEVICE)
    n_all = a.total_chunks if a.total_chunks else n * world
    total_bytes = float(n_all) * L * a.steps
    value = total_bytes / wall_max / GIB
    alg_bytes = float(n) * (L + 16)            # read every chunk once + 16-B digest write
    achieved = alg_bytes / (dev_ms_max * 1e-3) / 1e9
    vname = m.variant_name(m.resolve_variant(variant))
    res = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(wall_max / a.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong" if a.total_chunks else "weak",
        "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (device-generated splitmix words, per-rank seed)",
        "config": {"workload": ("C2: 1,048,576 x 16 KiB chunks per GPU, device-resident"
                                if (n, L) == (1 << 20, 16384) and not a.total_chunks else
                                f"{n_all} x {L} B chunks total, {n} on rank 0, device-resident"),
                   "chunks_per_gpu": n, "chunk_bytes": L, "kernel_variant": vname,
                   "parallelism": f"dp{world} (independent chunk shards, no collective)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": load_traffic(a.traffic, vname),
                     "kernel": "md5hip " + vname, "avg_launch_ms": round(dev_ms_max, 4),
                     "alg_bytes_per_launch": int(alg_bytes)},
    }
    return res


def run_crc(a, rank, world):
    """§8f row 2: netcache's own block checksum (CRC-32, crc32.c) over the C2
    shape, device-resident; the same step/timing rules as C2."""
    L, n = a.len, a.chunks
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0x5EED0000 + rank)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    fn = lambda: m.crc32_fixed(data, n, L, out=out)  # noqa: E731
    wall, dev_ms = timed_steps(fn, a.steps, a.warmup, world)
    wall_max = max_over_ranks(wall, world, COLL_DEVICE)
    dev_ms_max = max_over_ranks(dev_ms, world, COLL_DEVICE)
    value = float(n) * L * world * a.steps / wall_max / GIB
    alg_bytes = float(n) * (L + 4)
    vname = "crc32 " + m.crc_variant_name(0)
    achieved = alg_bytes / (dev_ms_max * 1e-3) / 1e9
    return {"metric": "device-resident CRC-32 (netcache blk_make_crc) GiB/s on batched 16 KiB chunks",
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(wall_max / a.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (device-generated splitmix words, per-rank seed)",
            "config": {"workload": f"{n} x {L} B chunks per GPU, device-resident, fastcrc 0",
                       "chunks_per_gpu": n, "chunk_bytes": L, "kernel_variant": vname},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": load_traffic(a.traffic, vname), "kernel": vname,
                         "avg_launch_ms": round(dev_ms_max, 4), "alg_bytes_per_launch": int(alg_bytes)}}


def run_c3(a, rank, world):
    """Mixed lengths 4 KiB..1 MiB (netcache chunk_size range, httpd.c:7968) with
    1-in-8 ragged tails, packed 16-B aligned, lanes packed longest-first."""
    import numpy as np

    def c3_lens(seed):
        rng = np.random.default_rng(seed)
        classes = np.array([4096 << k for k in range(9)], dtype=np.int64)
        out, tot = [], 0
        while tot < a.c3_bytes:
            c = int(classes[rng.integers(0, 9)])
            if rng.integers(0, 8) == 0:
                c = int(rng.integers(1, c))
            out.append(c)
            tot += c
        return np.array(out, dtype=np.int64)

    lens = c3_lens(1000 + rank)
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
    total = int(offs[-1] + lens[-1] + 16)
    # the batch lives in an arena (md5hip_arena_alloc: 1 GiB-aligned virtual
    # range, large page-table fragments), where HYBRID's lane-direct chains
    # run ~7 % faster than in a 2 MiB-aligned hipMalloc buffer
    data = m.arena_empty((total + 15) // 16 * 16)
    m.fill_synthetic(data, seed=0xC3 + rank)
    t0 = time.perf_counter()
    order, dvar = m.plan_desc(lens.astype(np.uint32))     # longest-first lanes + kernel choice
    plan_ms = (time.perf_counter() - t0) * 1e3
    if a.c3_variant != "plan":
        dvar = a.c3_variant
    d_off = torch.from_numpy(offs).cuda()
    d_len = torch.from_numpy(lens.astype(np.int32)).cuda()
    d_ord = torch.from_numpy(order.astype(np.int32)).cuda()
    out = torch.empty((lens.size, 16), dtype=torch.uint8, device="cuda")
    fn = lambda: m.digest_desc(data, d_off, d_len, d_ord, out=out, variant=dvar)  # noqa: E731
    wall, dev_ms = timed_steps(fn, a.steps, a.warmup, world)
    wall_max = max_over_ranks(wall, world, COLL_DEVICE)
    payload = float(lens.sum())
    value = payload * world * a.steps / wall_max / GIB
    # the longest chunk bounds the step: a 1 MiB chunk is 16,385 dependent
    # compressions on one lane.  A batched engine keeps several batches in
    # flight (the batcher's slots), so batch k+1's short chunks run beside
    # batch k's long chains: the same K batches issued round-robin on
    # `c3_streams` streams (each batch complete, own digest array) give the
    # streamed rate, reported beside the single-batch one.
    ns = max(1, a.c3_streams)
    streams = [torch.cuda.Stream() for _ in range(ns)]
    outs = [torch.empty_like(out) for _ in range(ns)]
    cur = torch.cuda.current_stream()

    def streamed(k):
        for s_ in streams:
            s_.wait_stream(cur)
        for j in range(k):
            with torch.cuda.stream(streams[j % ns]):
                m.digest_desc(data, d_off, d_len, d_ord, out=outs[j % ns], variant=dvar)
        for s_ in streams:
            cur.wait_stream(s_)

    streamed(a.warmup)
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    streamed(a.steps)
    torch.cuda.synchronize()
    s_wall = max_over_ranks(time.perf_counter() - t0, world, COLL_DEVICE)
    barrier(world)
    ok = all(torch.equal(o, out) for o in outs[:min(ns, a.steps)])
    del outs
    # coalesced: K such batches (own lengths, own bytes) planned and launched
    # as one descriptor batch -- what a batcher holding K submissions does;
    # the long chains of all K then overlap inside one launch
    coal = None
    K = a.c3_coalesce
    if K > 1:
        lk = [lens] + [c3_lens(2000 + 17 * j + rank) for j in range(1, K)]
        ok_ = [np.concatenate([[0], np.cumsum((x + 15) // 16 * 16)[:-1]]) for x in lk]
        spans = [int((o[-1] + x[-1] + 16 + 15) // 16 * 16) for o, x in zip(ok_, lk)]
        starts = np.concatenate([[0], np.cumsum(spans)[:-1]])
        big = m.arena_empty(int(sum(spans)))
        m.fill_synthetic(big, seed=0xC3C + rank)
        L_all = np.concatenate(lk)
        O_all = np.concatenate([o + st for o, st in zip(ok_, starts)])
        ordK, varK = m.plan_desc(L_all.astype(np.uint32))
        dO, dL = torch.from_numpy(O_all).cuda(), torch.from_numpy(L_all.astype(np.int32)).cuda()
        dR = torch.from_numpy(ordK.astype(np.int32)).cuda()
        outK = torch.empty((L_all.size, 16), dtype=torch.uint8, device="cuda")
        _, k_ms = timed_steps(lambda: m.digest_desc(big, dO, dL, dR, out=outK, variant=varK),
                              max(5, a.steps // 2), max(2, a.warmup // 4), world)
        pay = float(L_all.sum())
        coal = {"batches": K, "chunks": int(L_all.size), "payload_bytes": int(pay), "kernel": varK,
                "ms_per_launch": round(k_ms, 4), "ms_per_batch": round(k_ms / K, 4),
                "value": round(pay * world / (k_ms * 1e-3) / GIB, 2), "unit": "GiB/s",
                "note": "K C3 batches coalesced into one planned descriptor launch (distinct bytes)"}
        del big, dO, dL, dR, outK
    # imbalance vs uniform -- the same payload bytes of the
    # same arena hashed as uniform 16 KiB chunks by the fixed-length kernel
    n_u = int(payload) // 16384
    dig_u = torch.empty((n_u, 16), dtype=torch.uint8, device="cuda")
    _, u_ms = timed_steps(lambda: m.digest_fixed(data, n_u, 16384, out=dig_u), max(5, a.steps // 2),
                          a.warmup, world)
    del dig_u
    # the bound of one mixed batch: each chunk is one serial chain on one lane
    # (md5.c:204-210, 64 dependent steps per block), so the batch ends no
    # earlier than its longest chunks -- timed alone (every chunk of the
    # maximum length, same kernel variant as the batch; one lone chunk would
    # understate the chip's clock, which drops when a single wave is active)
    il = np.flatnonzero(lens == lens.max())
    d_off1 = torch.from_numpy(offs[il]).cuda()
    d_len1 = torch.from_numpy(lens[il].astype(np.int32)).cuda()
    dig1 = torch.empty((il.size, 16), dtype=torch.uint8, device="cuda")
    _, chain_ms = timed_steps(lambda: m.digest_desc(data, d_off1, d_len1, out=dig1, variant=dvar),
                              5, 2, world)
    del dig1
    return {"metric": "device-resident MD5 GiB/s, mixed 4 KiB-1 MiB chunks (C3)",
            "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(wall_max / a.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic", "config": {"workload": "C3 mixed lengths", "chunks": int(lens.size),
                                            "payload_bytes": int(payload),
                                            "longest": int(lens.max()), "plan_ms": round(plan_ms, 3),
                                            "kernel": "md5hip desc " + dvar,
                                            "uniform_16k_ms": round(u_ms, 4),
                                            "imbalance_vs_uniform": round(dev_ms / u_ms, 3)},
            "roofline": {"bound": "hbm", "achieved": round(payload / (dev_ms * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(payload / (dev_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "traffic": None,
                         "longest_alone_ms": round(chain_ms, 4),
                         "n_longest": int(il.size),
                         "frac_of_longest_alone": round(chain_ms / dev_ms, 4),
                         "note": "one batch ends with its longest chunks' serial chains "
                                 "(longest_alone_ms: those chunks hashed alone); see streamed"},
            "streamed": {"streams": ns, "value": round(payload * world * a.steps / s_wall / GIB, 2),
                         "unit": "GiB/s", "ms_per_batch": round(s_wall / a.steps * 1e3, 4),
                         "digests_equal_single": ok,
                         "note": "the same K batches, round-robin over streams, "
                                 "batch k+1 overlapping batch k's long chains"},
            "coalesced": coal}


def run_c5(a, rank, world):
    """End to end from pinned host memory: H2D -> MD5 -> D2H over pipelined
    batcher slots (md5hip_batch_host_fixed)."""
    import numpy as np
    n, L = a.c5_chunks, a.len
    host = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    host.view(torch.int64).random_(generator=torch.Generator().manual_seed(5))
    arr = host.numpy()
    # PCIe H2D alone (the denominator for this config): the same slices, on one
    # stream and round-robin over as many streams as the batcher has slots
    # (concurrent DMA); the better of the two, warmed up
    nsl = 3
    devs = [torch.empty(a.c5_slice, dtype=torch.uint8, device="cuda") for _ in range(nsl)]
    streams = [torch.cuda.Stream() for _ in range(nsl)]
    per = a.c5_slice
    h2d_gbs = 0.0
    for nst in (1, nsl, 1, nsl):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for k, off in enumerate(range(0, n * L, per)):
            m_ = min(per, n * L - off)
            with torch.cuda.stream(streams[k % nst]):
                devs[k % nst][:m_].copy_(host[off:off + m_], non_blocking=True)
        torch.cuda.synchronize()
        h2d_gbs = max(h2d_gbs, n * L / (time.perf_counter() - t0) / 1e9)
    del devs
    with m.Batcher(device=torch.cuda.current_device(), slice_bytes=a.c5_slice, nslots=nsl) as b:
        for _ in range(a.warmup):
            b.host_fixed(arr, n, L)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            b.host_fixed(arr, n, L)
        wall = time.perf_counter() - t0
    gbs = n * L * a.steps / wall / 1e9
    return {"metric": "end-to-end MD5 GiB/s from pinned host memory (C5)",
            "value": round(n * L * a.steps / wall / GIB, 2), "unit": "GiB/s", "n_gpus": 1,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(wall / a.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
            "data": "synthetic (host random)", "config": {"workload": "C5", "chunks": n,
                                                          "chunk_bytes": L, "slice_bytes": a.c5_slice,
                                                          "slots": 3},
            "roofline": {"bound": "pcie", "achieved": round(gbs, 2), "peak": round(h2d_gbs, 2),
                         "unit": "GB/s", "frac": round(gbs / h2d_gbs, 4),
                         "peak_note": (f"measured pinned H2D copy alone, best of 1 and {nsl} "
                                       f"streams; spec {PCIE_PEAK_GBS} GB/s"),
                         "traffic": None}}


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=20,
                   help="untimed launches first: the board settles its clock over the first ~15 "
                        "launches of a 3 ms kernel (slow start, profiles/r01_bench_kernel_trace_startup.json)")
    p.add_argument("--config", default="c2", choices=["c2", "c3", "c5", "crc"])
    p.add_argument("--chunks", type=int, default=1 << 20, help="chunks per GPU (C2, weak scaling)")
    p.add_argument("--total-chunks", type=int, default=0,
                   help="one global batch split across ranks (C4: 16777216 on 8 GPUs)")
    p.add_argument("--len", type=int, default=16384)
    p.add_argument("--variant", default="auto", choices=sorted(m.VARIANTS))
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                   help="control-plane backend for N > 1 (barrier + scalar MAX only)")
    p.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"))
    p.add_argument("--c3-bytes", type=int, default=16 << 30)
    p.add_argument("--c3-variant", default="plan", choices=["plan"] + sorted(m.DESC_VARIANTS),
                   help="descriptor kernel for C3 (plan = md5hip_plan_desc's choice)")
    p.add_argument("--c3-coalesce", type=int, default=3,
                   help="C3 batches planned and launched together for the coalesced rate (0/1 = off)")
    p.add_argument("--c3-streams", type=int, default=3,
                   help="streams for C3's streamed rate (batches in flight)")
    p.add_argument("--c5-chunks", type=int, default=1 << 18)
    p.add_argument("--c5-slice", type=int, default=64 << 20)
    a = p.parse_args()
    rank, world, _ = dist_setup(a.gpus, a.dist_backend)
    res = {"c2": run_c2, "c3": run_c3, "c5": run_c5, "crc": run_crc}[a.config](a, rank, world)
    if rank == 0 and world == 1 and a.config == "c2" and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline()
        # labelled separately: the same reference md5.c on the box's CPU share
        res["cpu_baseline_all_cores"] = cpu_baseline(reps=10, threads=CPU_SHARE)
    if rank == 0 and world == 1 and a.config == "crc" and not a.no_cpu_baseline:
        res["cpu_baseline"] = cpu_baseline_crc()
    if rank == 0:
        print(json.dumps(res), flush=True)
    if world > 1:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
