#!/usr/bin/env python3
"""bench.py -- device-resident batched MD5 throughput on MI355X.

Metric (BASELINE.json): device-resident MD5 GiB/s on batched 16 KiB chunks at
1/2/4/8 MI355X.  A "step" = one pass of the batched-MD5 kernel over the rank's
whole batch, inputs already in HBM (filled on the device by
md5hip_fill_synthetic, per-rank seed).  Per GPU: 1,048,576 x 16 KiB (C2) at
N = 1, 2,097,152 x 16 KiB (the C4 shard: 16 M chunks over 8 GPUs) at N > 1.

    python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c3q|c5|crc|crcq|ctx]

N > 1: one process per GPU.  Under torch.distributed.run (WORLD_SIZE set) the
ranks are the launcher's and WORLD_SIZE must equal N.  A plain
`python bench.py --gpus N` starts torch.distributed.run itself, as a CHILD
process before this process touches the GPU (never an exec), and exits with
its status: rank 0's JSON line is the output.  Each rank hashes its own shard
of independent chunks (weak scaling, no data-path collective); barrier +
device sync bracket the K timed steps and the MAX time over ranks is used.
The line carries `per_gpu` (each rank's own GiB/s) and `ranks_seen` (world
size, backend, and the device every rank hashed on).

The cpu_baseline leg (the only use of oracle/ here) runs the host reference
md5.c (oracle/_ref, else the oracle port): timed on the C1 sample (rank 0,
N = 1), and -- as the checker, outside the timed region -- re-digesting a
sample of the very batch each rank hashed (`parity` in the line).
"""
import argparse
import ctypes
import json
import os
import platform
import socket
import subprocess
import sys
import time
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.abspath(__file__))
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s (spec)
PCIE_PEAK_GBS = 63.0           # PCIe Gen5 x16 (spec)
METRIC = "device-resident MD5 GiB/s on batched 16 KiB chunks at 1/2/4/8 MI355X"
GIB = float(1 << 30)
CPU_SHARE = 16                 # host cores a one-GPU box grants a job (the box's CPU share)

torch = m = shard = None       # imported after the launcher decision (see main)


# --------------------------------------------------------------------------- launch
def parse_args(argv):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=20,
                   help="untimed launches first: the board settles its clock over the first ~15 "
                        "launches of a 3 ms kernel (slow start, profiles/r01_bench_kernel_trace_startup.json)")
    p.add_argument("--config", default="c2", choices=["c2", "c3", "c3q", "c5", "crc", "crcq", "ctx"])
    p.add_argument("--chunks", type=int, default=0,
                   help="chunks per GPU (weak scaling); 0 = 1,048,576 (C2) at N=1, "
                        "2,097,152 (the C4 shard) at N>1")
    p.add_argument("--total-chunks", type=int, default=0,
                   help="one global batch split across ranks (strong scaling; C4 = 16777216)")
    p.add_argument("--len", type=int, default=16384)
    p.add_argument("--variant", default="auto")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--parity-sample", type=int, default=4096,
                   help="chunks per rank re-digested by the host reference after timing (0 = off)")
    p.add_argument("--dist-always", action="store_true",
                   help="bring the process group up even at WORLD_SIZE 1 (a one-GPU rehearsal "
                        "of the control plane: init, barrier, MAX, object gathers)")
    p.add_argument("--dist-backend", default="gloo", choices=["nccl", "gloo"],
                   help="control-plane backend for N > 1: a barrier, scalar MAX and object "
                        "gathers, no data-path collective.  gloo by default: with an RCCL "
                        "communicator up, the C2 kernel ran 3-5 %% slower on the same GPU "
                        "(profiles/r05w/); nccl brings RCCL up for the same control plane")
    p.add_argument("--share-gpu", action="store_true",
                   help="N > 1 ranks on fewer GPUs (a rehearsal on a one-GPU box); without it "
                        "every rank needs a GPU of its own")
    p.add_argument("--dry-run", action="store_true",
                   help="CPU only (no GPU): exercises launch, ranks and aggregation with the "
                        "product's host MD5 (md5_stream.c) on a small host batch")
    p.add_argument("--traffic", default=os.path.join(REPO, "profiles", "traffic.json"))
    p.add_argument("--fastcrc", type=int, default=0, help="--config crc: blk_make_crc fastcrc window")
    p.add_argument("--c3-bytes", type=int, default=16 << 30)
    p.add_argument("--c3-variant", default="plan",
                   help="descriptor kernel for C3 (plan = md5hip_plan_desc's choice)")
    p.add_argument("--c3-coalesce", type=int, default=0,
                   help="C3 batches planned and launched together for the coalesced rate; 0 = sized "
                        "by the list-scheduling rule (the fewest batches, up to 8, whose LPT makespan "
                        "is within 5 %% of the mean SIMD load, lpt_schedule); 1 = off")
    p.add_argument("--c3-streams", type=int, default=3,
                   help="streams for C3's streamed rate (batches in flight)")
    p.add_argument("--c3-legs", default="all", choices=["all", "main", "coalesced"],
                   help="main / coalesced: only the single-batch / the coalesced launches "
                        "(PMC passes count one kernel on one workload)")
    p.add_argument("--c3q-batches", type=int, default=6,
                   help="--config c3q: C3 submissions streamed through one md5hip_queue")
    p.add_argument("--c3q-inflight", type=int, default=1,
                   help="--config c3q: launches in flight before the queue coalesces")
    p.add_argument("--c3q-slots", type=int, default=4, help="--config c3q: queue slots")
    p.add_argument("--c3q-chain", type=int, default=2,
                   help="--config c3q: chained launches (md5hip_batcher_set_chain: 0 off, 1 on, 2 = on + BALANCED tails overlap, the default)")
    p.add_argument("--crcq-subs", type=int, default=8,
                   help="--config crcq: fixed-length device submissions per step through one queue")
    p.add_argument("--crcq-chunks", type=int, default=1 << 20, help="--config crcq: blocks per submission")
    p.add_argument("--crcq-fastcrc", type=int, default=128,
                   help="--config crcq: blk_make_crc's fastcrc window F (0 = the whole block)")
    p.add_argument("--extras", default="c3q,c5",
                   help="--config c2 at one GPU: BASELINE configs measured after the headline's "
                        "timed region and parity, as sub-records of the same line (c3q = the C3 "
                        "stream through md5hip_queue, c5 = end to end from pinned host memory); "
                        "'none' for the headline alone (profiling passes)")
    p.add_argument("--no-board-probe", action="store_true",
                   help="skip the C2 board probe (clock / power / PPT residency under the kernel, "
                        "after the timed region)")
    p.add_argument("--c5-chunks", type=int, default=1 << 18)
    p.add_argument("--c5-slice", type=int, default=64 << 20)
    return p.parse_args(argv)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(a, argv):
    """`--gpus N` (N > 1) without a launcher: run torch.distributed.run as a
    child process -- this process has not initialised the GPU, and it is not
    replaced (no exec) -- and return the child's exit status.  Rank 0 of the
    child prints the JSON line on the inherited stdout."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={a.gpus}", "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.abspath(__file__), *argv]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.call(cmd, env=env)


def dist_setup(a):
    """One process per GPU, the control plane from sproxy_amd/shard.py (a
    barrier, scalar MAX/SUM reductions and small object gathers -- the chunks
    are independent, so no byte crosses between ranks), over gloo by default.
    With --share-gpu, N ranks may share one GPU (a rehearsal on a one-GPU box)."""
    rank, world, local = shard.env_rank()
    if world != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={world}")
    backend = "gloo" if a.dry_run else a.dist_backend
    device = None
    if not a.dry_run:
        ndev = torch.cuda.device_count()
        if ndev < 1:
            raise SystemExit("bench.py: no HIP device visible (use --dry-run on a CPU host)")
        if world > 1 and local >= ndev and (backend == "nccl" or not a.share_gpu):
            raise SystemExit(f"bench.py: LOCAL_RANK {local} but only {ndev} GPUs visible"
                             + ("" if backend == "nccl" else " (--share-gpu for a rehearsal)"))
        device = local % ndev
        torch.cuda.set_device(device)
    shard.init_group(world, backend, device, always=a.dist_always)
    return rank, world, local, device, backend


def device_info(rank, local, device):
    d = {"rank": rank, "local_rank": local, "host": socket.gethostname(), "device": device}
    if device is not None:
        p = torch.cuda.get_device_properties(device)
        d.update(name=p.name, uuid=str(getattr(p, "uuid", "")),
                 pci=f"{getattr(p, 'pci_domain_id', 0):04x}:{getattr(p, 'pci_bus_id', 0):02x}:"
                     f"{getattr(p, 'pci_device_id', 0):02x}")
    return d


def timed_steps(fn, steps, warmup, world):
    """W untimed steps, then exactly K steps between barrier+sync pairs.
    Returns (wall seconds for K steps, avg device ms per step from HIP events
    recorded on the stream the kernels run on)."""
    for _ in range(warmup):
        fn()
    torch.cuda.synchronize()
    stream = torch.cuda.current_stream()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    shard.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(steps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    shard.barrier()
    return t1 - t0, e0.elapsed_time(e1) / steps


def cpu_model():
    try:
        for ln in open("/proc/cpuinfo"):
            if ln.startswith("model name"):
                return ln.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


# --------------------------------------------------------------------------- cpu_baseline leg
# The host reference md5.c (oracle/_ref, built in place from /root/reference;
# else the oracle restatement).  Timed on the C1 sample for the baseline, and
# used -- outside every timed region -- as the CHECKER of a sample of the
# batch the GPU hashed.  Nothing here is on the measured path.
class _HostRef:
    def __init__(self):
        ref = os.path.join(REPO, "oracle", "_ref", "libmd5_ref.so")
        port = os.path.join(REPO, "oracle", "_build", "libmd5_oracle.so")
        if os.path.exists(ref):
            self.lib, self.kind = ctypes.CDLL(ref), "reference md5.c (oracle/_ref)"
            vp = ctypes.c_void_p
            self.lib.MD5Init.argtypes = [vp]
            self.lib.MD5Update.argtypes = [vp, vp, ctypes.c_uint]
            self.lib.MD5Final.argtypes = [vp, vp]
        elif os.path.exists(port):
            self.lib, self.kind = ctypes.CDLL(port), "oracle restatement (oracle/_build)"
            self.lib.oracle_md5.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p]
        else:
            self.lib = None
            self.kind = "absent"

    def digest(self, buf, off, n):
        """MD5 of buf[off:off+n] (buf: contiguous numpy uint8)."""
        out = (ctypes.c_ubyte * 16)()
        p = buf.ctypes.data + off
        if self.kind.startswith("reference"):
            ctx = (ctypes.c_ubyte * 88)()
            self.lib.MD5Init(ctx)
            done = 0
            while True:                          # md5.h:47 takes an unsigned length
                part = min(n - done, 1 << 30)
                self.lib.MD5Update(ctx, p + done, part)
                done += part
                if done >= n:
                    break
            self.lib.MD5Final(out, ctx)
        else:
            self.lib.oracle_md5(p, n, out)
        return bytes(out)


def check_sample(buf, offs, lens, got, threads=8):
    """parity of a sample: host reference digests of (buf, offs, lens) vs the
    GPU's digests `got` (uint8 [k, 16])."""
    import numpy as np
    ref = _HostRef()
    if ref.lib is None:
        return {"checked": 0, "ok": None, "checker": "absent"}
    k = len(lens)
    with ThreadPoolExecutor(max_workers=threads) as ex:     # ctypes releases the GIL
        exp = list(ex.map(lambda j: ref.digest(buf, int(offs[j]), int(lens[j])), range(k)))
    exp = np.frombuffer(b"".join(exp), dtype=np.uint8).reshape(k, 16)
    bad = int((exp != got).any(axis=1).sum())
    return {"checked": k, "mismatches": bad, "ok": bad == 0, "checker": ref.kind,
            "sample_bytes": int(np.sum(np.asarray(lens, dtype=np.int64)))}


def sample_fixed(data, out, n, L, k, seed):
    """(parity dict) for k distinct random chunks plus the first and last of a
    fixed-length device batch; chunk rows gathered on the device, one D2H."""
    import numpy as np
    if k <= 0:
        return None
    rng = np.random.default_rng(seed)
    # k distinct random chunks (drawn without replacement) plus the first and
    # last: at least k checked (>= 4096)
    idx = np.unique(np.concatenate([[0, n - 1], rng.choice(n, size=min(k, n), replace=False)]))
    it = torch.from_numpy(idx.astype(np.int64)).to(data.device)
    rows = data[: n * L].view(n, L).index_select(0, it).cpu().numpy().reshape(-1)
    got = out.index_select(0, it).cpu().numpy()
    return check_sample(rows, np.arange(idx.size, dtype=np.int64) * L, np.full(idx.size, L), got)


def sample_desc(data, offs, lens, out, idx):
    """(parity dict) for the chunks `idx` of a descriptor batch in device `data`."""
    import numpy as np
    idx = np.unique(np.asarray(idx, dtype=np.int64))
    parts = [data[int(offs[j]): int(offs[j]) + int(lens[j])] for j in idx]
    flat = torch.cat(parts).cpu().numpy() if parts else np.empty(0, np.uint8)
    l_s = lens[idx].astype(np.int64)
    o_s = np.concatenate([[0], np.cumsum(l_s)[:-1]]) if idx.size else l_s
    got = out.index_select(0, torch.from_numpy(idx).to(out.device)).cpu().numpy()
    return check_sample(flat, o_s, l_s, got)


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


# --------------------------------------------------------------------------- traffic evidence
def load_traffic(path, kernel, workload):
    """HBM bytes per launch of `kernel` on `workload` from the committed
    rocprofv3 PMC summary (profiles/traffic.json, scripts/traffic_json.py).
    Each entry carries the SHA-256 of the kernel's machine code it measured;
    unless the library's current code for that kernel has the same hash, the
    entry is stale and traffic reads null."""
    if not path or not os.path.exists(path):
        return None, "no traffic summary"
    try:
        ent = json.load(open(path)).get("entries", {}).get(f"{kernel}@{workload}")
    except Exception as e:  # pragma: no cover
        return None, f"unreadable: {e}"
    if ent is None:
        return None, f"no PMC entry for {kernel}@{workload}"
    h = m.kernel_code_hash(kernel)
    if ent.get("code_hash") != h:
        return None, f"stale: {kernel} code {h[:16]} != measured {str(ent.get('code_hash'))[:16]}"
    note = f"rocprofv3 PMC FETCH_SIZE/WRITE_SIZE, kernel code {h[:16]}; {ent.get('source', '')}"
    return ent["bytes"], note


def load_valu_busy(path, kernel, workload):
    """VALUBusy of `kernel` on `workload` (the secondary ceiling
    beside HBM) from the same code-hash-checked PMC entry, or None."""
    try:
        ent = json.load(open(path)).get("entries", {}).get(f"{kernel}@{workload}")
    except Exception:  # pragma: no cover
        return None
    if not ent or ent.get("code_hash") != m.kernel_code_hash(kernel):
        return None
    return ent.get("valu_busy")


# --------------------------------------------------------------------------- configs
def per_rank_line(res, rank, world, local, device, backend, rank_bytes, rank_wall, parity):
    """Gather every rank's own rate, device and parity into the line."""
    mine = {"gib_s": round(rank_bytes / rank_wall / GIB, 2) if rank_wall else 0.0,
            "dev": device_info(rank, local, device), "parity": parity}
    allr = shard.gather_objects(mine)
    res["per_gpu"] = [r["gib_s"] for r in allr]
    devs = [r["dev"] for r in allr]
    res["ranks_seen"] = {"world": world, "backend": backend if shard.group_on() else None,
                         "distinct_devices": len({(d["host"], d.get("uuid") or d["device"]) for d in devs
                                                  if d["device"] is not None}),
                         "ranks": devs}
    ps = [r["parity"] for r in allr if r["parity"] is not None]
    if ps:
        res["parity"] = {"ok": all(p["ok"] for p in ps), "checked": sum(p["checked"] for p in ps),
                         "mismatches": sum(p.get("mismatches", 0) for p in ps),
                         "checker": ps[0]["checker"],
                         "sample": ps[0].get("sample") or
                                   "first + last + seeded distinct random chunks of every rank's batch, "
                                   "re-digested on the host after the timed region"}
    return res


def run_dry(a, rank, world, local, device, backend):
    """CPU dry run: the launch, rank and aggregation path with no GPU -- each
    rank hashes a small host batch with the product's host MD5 (md5_stream.c)."""
    import numpy as np
    n, L = (a.chunks or 64), a.len
    buf = np.random.default_rng(0x5EED0000 + rank).integers(0, 256, n * L, dtype=np.uint8)
    out = np.empty((n, 16), dtype=np.uint8)

    def step():
        for i in range(n):
            out[i] = np.frombuffer(m.md5(buf[i * L:(i + 1) * L]), dtype=np.uint8)

    for _ in range(a.warmup):
        step()
    shard.barrier()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    wall = time.perf_counter() - t0
    shard.barrier()
    wall_max = shard.max_over_ranks(wall)
    par = None
    if a.parity_sample:
        k = min(n, a.parity_sample)
        par = check_sample(buf, np.arange(k) * L, np.full(k, L), out[:k])
    res = {"metric": METRIC + " [CPU dry run]", "value": round(n * L * world * a.steps / wall_max / GIB, 4),
           "unit": "GiB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(wall_max / a.steps * 1e3, 4), "higher_is_better": True,
           "scaling": "weak", "vs_baseline": None, "dtype": "u32", "dry_run": True,
           "data": "synthetic host buffers (CPU dry run: product host MD5, no GPU)",
           "config": {"workload": f"dry run: {n} x {L} B host chunks per rank, standing in for "
                                  f"{c2_workload(*c2_shape_gpu(a, world), L, world, bool(a.total_chunks))}",
                      "chunks_per_gpu": n, "chunk_bytes": L,
                      "parallelism": f"dp{world} (independent chunk shards, no collective)"}}
    return per_rank_line(res, rank, world, local, device, backend, n * L * a.steps, wall, par)


def c2_shape(a, rank, world):
    if a.total_chunks:       # strong form: one global batch split into contiguous shards
        lo = a.total_chunks * rank // world
        hi = a.total_chunks * (rank + 1) // world
        return hi - lo, a.total_chunks
    n = a.chunks or ((1 << 20) if world == 1 else (1 << 21))
    return n, n * world


def c2_shape_gpu(a, world):
    """(chunks per GPU, chunks in all) of the device run these flags select
    (the dry run names it; --chunks sizes only the dry run's host batch)."""
    if a.total_chunks:
        return a.total_chunks // world, a.total_chunks
    n = (1 << 20) if world == 1 else (1 << 21)
    return n, n * world


def c2_workload(n, n_all, L, world, strong):
    if (n, L, world, strong) == (1 << 20, 16384, 1, False):
        return "C2: 1,048,576 x 16 KiB chunks per GPU, device-resident"
    if n == (1 << 21) and L == 16384 and not strong:
        return (f"C4 shard: 2,097,152 x 16 KiB chunks per GPU, {n_all:,} on {world} GPU(s) "
                f"(C4 = 16,777,216 on 8), device-resident")
    return f"{n_all} x {L} B chunks total, {n} per GPU, device-resident"


def run_c2(a, rank, world, local, device, backend):
    L = a.len
    n, n_all = c2_shape(a, rank, world)
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0x5EED0000 + rank)
    out = torch.empty((n, 16), dtype=torch.uint8, device="cuda")
    variant = m.VARIANTS[a.variant]
    fn = lambda: m.digest_fixed(data, n, L, out=out, variant=variant)  # noqa: E731
    wall, dev_ms = timed_steps(fn, a.steps, a.warmup, world)
    wall_max = shard.max_over_ranks(wall)
    dev_ms_max = shard.max_over_ranks(dev_ms)
    value = float(n_all) * L * a.steps / wall_max / GIB
    alg_bytes = float(n) * (L + 16)            # read every chunk once + 16-B digest write
    achieved = alg_bytes / (dev_ms_max * 1e-3) / 1e9
    vname = m.variant_name(m.resolve_variant(variant))
    kname = "md5_fixed_" + vname
    traffic, tnote = load_traffic(a.traffic, kname, f"c2@{n}x{L}")
    vbusy = load_valu_busy(a.traffic, kname, f"c2@{n}x{L}")
    res = {
        "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(wall_max / a.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "strong" if a.total_chunks else "weak",
        "vs_baseline": None, "dtype": "u32",
        "data": "synthetic (device-generated splitmix words, per-rank seed)",
        "config": {"workload": c2_workload(n, n_all, L, world, bool(a.total_chunks)),
                   "chunks_per_gpu": n, "chunk_bytes": L, "kernel_variant": vname,
                   "parallelism": f"dp{world} (independent chunk shards, no collective)"},
        "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                     "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                     "traffic": traffic, "traffic_source": tnote, "valu_busy_pmc": vbusy,
                     "kernel": "md5hip::" + kname, "avg_launch_ms": round(dev_ms_max, 4),
                     "alg_bytes_per_launch": int(alg_bytes)},
    }
    par = sample_fixed(data, out, n, L, a.parity_sample, seed=77 + rank)
    if world == 1 and not a.no_board_probe:
        res["board"] = board_probe(fn, device, dev_ms_max)
    return per_rank_line(res, rank, world, local, device, backend, float(n) * L * a.steps, wall, par)


def run_crc(a, rank, world, local, device, backend):
    """§8f row 2: netcache's own block checksum (CRC-32, crc32.c) over the C2
    shape, device-resident; the same step/timing rules as C2.  --fastcrc F:
    blk_make_crc's head^tail window (blk_io.c:408-424), F bytes at each end."""
    L = a.len
    n = a.chunks or (1 << 20)
    F = a.fastcrc
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0x5EED0000 + rank)
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    fn = lambda: m.crc32_fixed(data, n, L, fastcrc=F, out=out)  # noqa: E731
    wall, dev_ms = timed_steps(fn, a.steps, a.warmup, world)
    wall_max = shard.max_over_ranks(wall)
    dev_ms_max = shard.max_over_ranks(dev_ms)
    fast = 0 < F < L
    read = 2 * F if fast else L                 # bytes blk_make_crc reads per block
    alg_bytes = float(n) * (read + 4)
    kname = m.crc_kernel_name(L, F)
    achieved = alg_bytes / (dev_ms_max * 1e-3) / 1e9
    traffic, tnote = load_traffic(a.traffic, kname, f"crc@{n}x{L}f{F}")
    vbusy = load_valu_busy(a.traffic, kname, f"crc@{n}x{L}f{F}")
    res = {"metric": ("device-resident CRC-32 (netcache blk_make_crc) GiB/s on batched 16 KiB chunks"
                      if not fast else
                      f"device-resident fastcrc={F} CRC-32 (netcache blk_make_crc) blocks/s"),
           "value": (round(float(n) * L * world * a.steps / wall_max / GIB, 2) if not fast else
                     round(float(n) * world * a.steps / wall_max, 1)),
           "unit": "GiB/s" if not fast else "blocks/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(wall_max / a.steps * 1e3, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (device-generated splitmix words, per-rank seed)",
           "config": {"workload": f"{n} x {L} B chunks per GPU, device-resident, fastcrc {F}",
                      "chunks_per_gpu": n, "chunk_bytes": L, "kernel": kname,
                      "block_payload_gib_s": round(float(n) * L * world * a.steps / wall_max / GIB, 2)},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_source": tnote, "valu_busy_pmc": vbusy, "kernel": "md5hip::" + kname,
                        "avg_launch_ms": round(dev_ms_max, 4), "alg_bytes_per_launch": int(alg_bytes),
                        "alg_bytes_note": f"{read} B read per block (+4 B CRC written)"}}
    par = crc_sample(data, n, L, F, out, a.parity_sample, rank) if a.parity_sample else None
    return per_rank_line(res, rank, world, local, device, backend, float(n) * L * a.steps, wall, par)


def run_crcq(a, rank, world, local, device, backend):
    """The block checksum as a STREAM through the product's device-input
    queue: --crcq-subs fixed-length submissions of
    --crcq-chunks blocks per step (md5_batch_submit_device_fixed, ABI 4: no
    per-block descriptor crosses PCIe), each its own launch on the queue's
    slot streams, pipelined as --config c3q (step k submitted before step
    k-1's tickets are waited for).  CRC-32 with --crcq-fastcrc F (default 128, 0 = whole block):
    blk_make_crc reads F bytes at each end of a block (blk_io.c:408-424), so
    the algorithmic bytes are 2F + 4 per block."""
    L = a.len
    F = a.crcq_fastcrc
    K, n = max(1, a.crcq_subs), a.crcq_chunks
    need, (free, _) = K * n * L, torch.cuda.mem_get_info()
    if need > free:
        raise SystemExit(f"bench.py --config crcq: {K} x {n} x {L} B = {need / GIB:.1f} GiB of blocks, "
                         f"{free / GIB:.1f} GiB free on the device (lower --crcq-chunks or --crcq-subs)")
    data = torch.empty(K * n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0xC4C0 + rank)
    torch.cuda.synchronize()
    outs = [[torch.empty(n, dtype=torch.int32, device="cuda") for _ in range(K)] for _ in range(2)]
    # two steps' worth of slots: step k's launches are all queued on the
    # device while step k-1's run (one step's worth left the GPU waiting on
    # the host for each retire, r05f: 0.35)
    q = m.Queue(device=torch.cuda.current_device(), max_chunks=n, nslots=min(16, 2 * K + 1))
    q.set_digest(m.Batcher.CRC32, F)
    base = data.data_ptr()

    def submit(k):
        return [q.submit_device_fixed_async(base + j * n * L, n, L, L, out=outs[k & 1][j], after=None)
                for j in range(K)]

    def drain(pend):
        for pn in reversed(pend):
            pn.wait()

    def timed(fn):
        torch.cuda.synchronize()
        shard.barrier()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        shard.barrier()
        return wall, shard.max_over_ranks(wall)

    def pipelined():
        prev = submit(0)
        for k in range(1, a.steps):
            cur = submit(k)
            drain(prev)
            prev = cur
        drain(prev)

    for _ in range(a.warmup):
        drain(submit(0))
    wall_d, wall_d_max = timed(lambda: [drain(submit(0)) for _ in range(a.steps)])
    wall, wall_max = timed(pipelined)
    stats = q.stats()
    q.close()
    blocks = float(K * n)
    read = 2 * F if 0 < F < L else L
    alg = blocks * (read + 4)
    kname = m.crc_kernel_name(L, F)
    wl = f"crcq{K}@{n}x{L}f{F}"
    traffic, tnote = load_traffic(a.traffic, kname, wl)
    vbusy = load_valu_busy(a.traffic, kname, wl)
    step_s = wall_max / a.steps
    res = {"metric": f"device-resident fastcrc={F} CRC-32 (netcache blk_make_crc) blocks/s through md5hip_queue",
           "value": round(blocks * world * a.steps / wall_max, 1), "unit": "blocks/s", "n_gpus": world,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(step_s * 1e3, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (device-generated splitmix words, per-rank seed)",
           "config": {"workload": f"fastcrc stream: {K} fixed-length submissions of {n} x {L} B blocks per "
                                  f"step, device-resident, through md5hip_queue (md5_batch_submit_device_fixed)",
                      "submissions": K, "blocks_per_submission": n, "chunk_bytes": L, "fastcrc": F,
                      "kernel": kname, "queue": stats},
           "roofline": {"bound": "hbm", "achieved": round(alg / step_s / 1e9, 1), "peak": HBM_PEAK_GBS,
                        "unit": "GB/s", "frac": round(alg / step_s / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_source": tnote, "valu_busy_pmc": vbusy,
                        "kernel": "md5hip::" + kname + " (queue launches)",
                        "alg_bytes_per_step": int(alg),
                        "alg_bytes_note": f"{read} B read per block (+4 B CRC written); achieved: wall-clock "
                                          f"per pipelined step (submit + wait); traffic: HBM bytes per launch "
                                          f"({n} blocks)"},
           "drained": {"value": round(blocks * world * a.steps / wall_d_max, 1), "unit": "blocks/s",
                       "ms_per_step": round(wall_d_max / a.steps * 1e3, 4),
                       "frac": round(alg / (wall_d_max / a.steps) / 1e9 / HBM_PEAK_GBS, 4)}}
    par = None
    if a.parity_sample:
        ps = [crc_sample(data[j * n * L:(j + 1) * n * L], n, L, F, outs[(a.steps - 1) & 1][j],
                         a.parity_sample // K, rank + 10 * j) for j in range(K)]
        par = {"checked": sum(p.get("checked", 0) for p in ps), "mismatches": sum(p.get("mismatches", 0) for p in ps),
               "ok": all(p["ok"] for p in ps), "checker": ps[0].get("checker")}
    return per_rank_line(res, rank, world, local, device, backend, blocks * L * a.steps, wall, par)


def crc_sample(data, n, L, F, out, k, rank):
    """Parity of the CRC line: the first, the last and seeded-random blocks
    re-checksummed on the host after the timed region by the CRC-32
    restatement (oracle/crc32_oracle.c, pinned to the reference crc32.c by
    tests/test_oracle.py), blk_make_crc's fastcrc rule included."""
    import numpy as np
    lib = os.path.join(REPO, "oracle", "_build", "libmd5_oracle.so")
    if not os.path.exists(lib):
        return {"ok": None, "checker": "absent"}
    O = ctypes.CDLL(lib)
    O.oracle_crc32_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                     ctypes.c_uint64, ctypes.c_uint32, ctypes.c_void_p]
    idx = np.unique(np.concatenate([[0, n - 1], np.random.default_rng(77 + rank).choice(n, min(k, n), replace=False)]))
    rows = data.view(n, L)[torch.from_numpy(idx).to(data.device)].cpu().numpy()
    offs = np.arange(idx.size, dtype=np.uint64) * np.uint64(L)
    lens = np.full(idx.size, L, dtype=np.uint32)
    want = np.empty(idx.size, dtype=np.uint32)
    O.oracle_crc32_batch(rows.ctypes.data, offs.ctypes.data, lens.ctypes.data, idx.size, F,
                         want.ctypes.data)
    got = out.index_select(0, torch.from_numpy(idx).to(out.device)).cpu().numpy().view(np.uint32)
    bad = int((got != want).sum())
    return {"ok": bad == 0, "checked": int(idx.size), "mismatches": bad,
            "checker": "CRC-32 restatement (oracle/crc32_oracle.c, pinned to crc32.c)",
            "sample": "first + last + seeded-random blocks, re-checksummed on the host after the timed region"}


def c3_lens(total_bytes, seed):
    """C3 lengths: classes 4 KiB..1 MiB, 1 in 8 a ragged
    tail in [1, class) (blk_io.c:377), until `total_bytes` of payload."""
    import numpy as np
    rng = np.random.default_rng(seed)
    classes = np.array([4096 << k for k in range(9)], dtype=np.int64)
    out, tot = [], 0
    while tot < total_bytes:
        c = int(classes[rng.integers(0, 9)])
        if rng.integers(0, 8) == 0:
            c = int(rng.integers(1, c))
        out.append(c)
        tot += c
    return np.array(out, dtype=np.int64)


def c3_offsets(lens):
    import numpy as np
    offs = np.concatenate([[0], np.cumsum((lens + 15) // 16 * 16)[:-1]])
    return offs, int(offs[-1] + lens[-1] + 16)


def c3_sample(lens, order, k, seed):
    """C3 parity sample: seeded-random chunks, the first and last in lane
    order, every length class and 64 of each ragged residue len % 64 in
    {1, 55, 56, 63, 0}."""
    import numpy as np
    rng = np.random.default_rng(seed)
    pick = [rng.integers(0, lens.size, size=max(0, k - 2)), [order[0], order[-1]]]
    for c in [4096 << j for j in range(9)]:
        pick.append(np.flatnonzero(lens == c)[:8])
    rag = ~np.isin(lens, [4096 << j for j in range(9)])
    for r in (1, 55, 56, 63, 0):
        pick.append(np.flatnonzero(rag & (lens % 64 == r))[:64])
    return np.unique(np.concatenate([np.asarray(p, dtype=np.int64) for p in pick]))


LPT_SIMDS, LPT_GROUP = 1024, 64      # BALANCED: one wave per SIMD, 64-chunk groups


def lpt_schedule(lens, simds=LPT_SIMDS):
    """The list schedule of one BALANCED launch (md5_desc_balanced_t): 64-chunk
    groups in md5hip_plan_desc's longest-first order, taken by whichever of
    the `simds` waves is free first; a group costs its longest chunk's
    compressions (its lanes run in lockstep; floor((len+8)/64)+1, md5.c:221-265).
    Returns mean load, makespan (both in compressions) and util = mean /
    makespan, the share of SIMD-time the launch can keep busy: a 1 MiB chunk
    is a serial chain of 16,385 compressions, so a launch with too little
    work beside its longest chains idles SIMDs in its tail."""
    import heapq
    import numpy as np
    c = np.sort((np.asarray(lens, dtype=np.int64) + 8) // 64 + 1)[::-1]
    groups = c[::LPT_GROUP]
    free = [0] * simds
    for g in groups.tolist():
        heapq.heappush(free, heapq.heappop(free) + g)
    mean, makespan = float(groups.sum()) / simds, float(max(free))
    return {"mean_compressions": round(mean, 1), "makespan_compressions": makespan,
            "util": round(mean / makespan, 4), "groups": int(groups.size)}


def c3_coalesced(a, lens, rank, world):
    """K C3 batches (the main batch's lengths + K-1 more, own bytes) planned
    and launched as one descriptor batch -- what md5hip_queue does with K
    pending submissions (--config c3q) -- timed with HIP events.  K =
    --c3-coalesce, or (0) the fewest batches whose list schedule keeps 95 %
    of SIMD-time busy (lpt_schedule): at 3 batches the 1 MiB chains set the
    makespan and a quarter of the SIMD-time idles in the tail."""
    import numpy as np
    lk = [lens]
    if a.c3_coalesce:
        K = a.c3_coalesce
        lk += [c3_lens(a.c3_bytes, 2000 + 17 * j + rank) for j in range(1, K)]
    else:
        while len(lk) < 8 and lpt_schedule(np.concatenate(lk))["util"] < 0.95:
            lk.append(c3_lens(a.c3_bytes, 2000 + 17 * len(lk) + rank))
        K = len(lk)
    lpt = lpt_schedule(np.concatenate(lk))
    ok_ = [c3_offsets(x)[0] for x in lk]
    spans = [(c3_offsets(x)[1] + 15) // 16 * 16 for x in lk]
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
    kname = "md5_desc_" + ("balanced_t" if varK == "balanced" else varK)
    traffic, tnote = load_traffic(a.traffic, kname, f"c3k{K}@{a.c3_bytes}s{1000 + rank}")
    vbusy = load_valu_busy(a.traffic, kname, f"c3k{K}@{a.c3_bytes}s{1000 + rank}")
    par = sample_desc(big, O_all, L_all, outK, c3_sample(L_all, ordK, a.parity_sample // 2, 191 + rank)) \
        if a.parity_sample else None
    alg = pay + 16 * L_all.size
    return {"batches": K, "chunks": int(L_all.size), "payload_bytes": int(pay), "kernel": varK,
            "ms_per_launch": round(k_ms, 4), "ms_per_batch": round(k_ms / K, 4),
            "value": round(pay * world / (k_ms * 1e-3) / GIB, 2), "unit": "GiB/s",
            "sized_by": "--c3-coalesce" if a.c3_coalesce else "lpt util >= 0.95",
            "lpt": lpt,
            "roofline": {"bound": "hbm", "achieved": round(alg / (k_ms * 1e-3) / 1e9, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                         "frac_of_lpt_ceiling": round(alg / (k_ms * 1e-3) / 1e9 / HBM_PEAK_GBS / lpt["util"], 4),
                         "traffic": traffic, "traffic_source": tnote, "valu_busy_pmc": vbusy, "kernel": "md5hip::" + kname,
                         "alg_bytes_per_launch": int(alg)},
            "parity": par,
            "note": "K C3 batches coalesced into one planned descriptor launch (distinct bytes)"}


def run_c3(a, rank, world, local, device, backend):
    """Mixed lengths 4 KiB..1 MiB (netcache chunk_size range, httpd.c:7968) with
    1-in-8 ragged tails, packed 16-B aligned, lanes packed longest-first."""
    import numpy as np
    lens = c3_lens(a.c3_bytes, 1000 + rank)
    if a.c3_legs == "coalesced":
        coal = c3_coalesced(a, lens, rank, world)
        return per_rank_line({"metric": "C3 coalesced launches only (profiling run)", "value": coal["value"],
                              "unit": "GiB/s", "n_gpus": world, "config": {"workload": "C3 coalesced"},
                              "coalesced": coal}, rank, world, local, device, backend,
                             coal["payload_bytes"], coal["ms_per_launch"] * 1e-3, coal["parity"])
    offs, total = c3_offsets(lens)
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
    wall_max = shard.max_over_ranks(wall)
    payload = float(lens.sum())
    value = payload * world * a.steps / wall_max / GIB
    par = sample_desc(data, offs, lens, out, c3_sample(lens, order, a.parity_sample // 2, 91 + rank)) \
        if a.parity_sample else None
    # the longest chunk bounds the step: a 1 MiB chunk is 16,385 dependent
    # compressions on one lane.  A batched engine keeps several batches in
    # flight, so batch k+1's short chunks run beside batch k's long chains:
    # the same K batches issued round-robin on `c3_streams` streams (each
    # batch complete, own digest array) give the streamed rate.
    if a.c3_legs == "main":
        kname = "md5_desc_" + dvar
        return per_rank_line({"metric": "C3 main launches only (profiling run)", "value": round(value, 2),
                              "unit": "GiB/s", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                              "config": {"workload": "C3 mixed lengths", "kernel": kname},
                              "roofline": {"avg_launch_ms": round(dev_ms, 4)}},
                             rank, world, local, device, backend, payload * a.steps, wall, par)
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
    shard.barrier()
    t0 = time.perf_counter()
    streamed(a.steps)
    torch.cuda.synchronize()
    s_wall = shard.max_over_ranks(time.perf_counter() - t0)
    shard.barrier()
    ok = all(torch.equal(o, out) for o in outs[:min(ns, a.steps)])
    del outs
    # coalesced: K such batches (own lengths, own bytes) planned and launched
    # as one descriptor batch by hand (what md5hip_queue does, --config c3q)
    coal = c3_coalesced(a, lens, rank, world) if a.c3_coalesce != 1 else None
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
    # maximum length, same kernel variant as the batch)
    il = np.flatnonzero(lens == lens.max())
    d_off1 = torch.from_numpy(offs[il]).cuda()
    d_len1 = torch.from_numpy(lens[il].astype(np.int32)).cuda()
    dig1 = torch.empty((il.size, 16), dtype=torch.uint8, device="cuda")
    _, chain_ms = timed_steps(lambda: m.digest_desc(data, d_off1, d_len1, out=dig1, variant=dvar),
                              5, 2, world)
    del dig1
    kname = "md5_desc_" + dvar
    traffic, tnote = load_traffic(a.traffic, kname, f"c3@{a.c3_bytes}s{1000 + rank}")
    vbusy = load_valu_busy(a.traffic, kname, f"c3@{a.c3_bytes}s{1000 + rank}")
    achieved = payload / (dev_ms * 1e-3) / 1e9
    res = {"metric": "device-resident MD5 GiB/s, mixed 4 KiB-1 MiB chunks (C3)",
           "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(wall_max / a.steps * 1e3, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
           "data": "synthetic", "config": {"workload": "C3 mixed lengths", "chunks": int(lens.size),
                                           "payload_bytes": int(payload),
                                           "longest": int(lens.max()), "plan_ms": round(plan_ms, 3),
                                           "kernel": "md5hip desc " + dvar,
                                           "uniform_16k_ms": round(u_ms, 4),
                                           "imbalance_vs_uniform": round(dev_ms / u_ms, 3)},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_source": tnote, "valu_busy_pmc": vbusy, "kernel": "md5hip::" + kname,
                        "avg_launch_ms": round(dev_ms, 4),
                        "alg_bytes_per_launch": int(payload + 16 * lens.size),
                        "chain_bound": {"longest_alone_ms": round(chain_ms, 4), "n_longest": int(il.size),
                                        "frac": round(chain_ms / dev_ms, 4),
                                        "note": "second roofline: the batch's longest chunks hashed "
                                                "alone (serial chains, md5.c:204-210) / the batch"}},
           "streamed": {"streams": ns, "value": round(payload * world * a.steps / s_wall / GIB, 2),
                        "unit": "GiB/s", "ms_per_batch": round(s_wall / a.steps * 1e3, 4),
                        "digests_equal_single": ok,
                        "note": "the same K batches, round-robin over streams, "
                                "batch k+1 overlapping batch k's long chains"},
           "coalesced": coal}
    return per_rank_line(res, rank, world, local, device, backend, payload * a.steps, wall, par)


def run_c3q(a, rank, world, local, device, backend):
    """C3 through the product's device-input queue (md5hip_queue, include/
    md5hip.h): `c3q_batches` distinct C3 batches (own lengths, own bytes)
    submitted back to back, as netcache's ASIO threads would submit vectors;
    the queue coalesces whatever is pending into one planned launch per slot
    and completes each ticket on its own.  A step = submit all K; the value is
    the pipelined stream (step k's submissions go in before step k-1's tickets
    are waited for, so the queue never runs dry between steps), `drained` the
    same steps with every ticket waited for before the next submission."""
    import numpy as np
    K = max(1, a.c3q_batches)
    lk = [c3_lens(a.c3_bytes, 3000 + 31 * j + rank) for j in range(K)]
    ok_ = [c3_offsets(x)[0] for x in lk]
    spans = [(c3_offsets(x)[1] + 15) // 16 * 16 for x in lk]
    starts = np.concatenate([[0], np.cumsum(spans)[:-1]]).astype(np.int64)
    big = m.arena_empty(int(sum(spans)))
    m.fill_synthetic(big, seed=0xC3D + rank)
    torch.cuda.synchronize()           # the queue also orders itself after torch's stream
    base = big.data_ptr()
    subs = []
    for j in range(K):
        ptrs = (base + starts[j] + ok_[j]).astype(np.uint64)
        subs.append((ptrs, lk[j].astype(np.uint32), None))
    outs = [[torch.empty((x.size, 16), dtype=torch.uint8, device="cuda") for x in lk] for _ in range(2)]
    q = m.Queue(device=torch.cuda.current_device(), nslots=a.c3q_slots, inflight=a.c3q_inflight)
    if a.c3q_chain != 2:
        q.set_chain(a.c3q_chain)

    def submit(k):
        return [q.submit_device_async(p, L_, o) for (p, L_, _), o in zip(subs, outs[k & 1])]

    def drain(pend):
        for pn in reversed(pend):          # any order: tickets complete independently
            pn.wait()

    def drained_step():
        drain(submit(0))

    def timed(fn):
        torch.cuda.synchronize()
        shard.barrier()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        shard.barrier()
        return wall, shard.max_over_ranks(wall)

    def pipelined():
        # step k submits its K vectors, then waits for step k-1's: the queue
        # always holds the next step's work while a launch runs.  The stream
        # starts with a flush (step 0 goes out at once instead of lingering
        # into step 1's burst); after that the queue's own policy runs it.
        prev = submit(0)
        q.flush()
        for k in range(1, a.steps):
            cur = submit(k)
            drain(prev)
            prev = cur
        drain(prev)

    for _ in range(a.warmup):
        drained_step()
    wall_d, wall_d_max = timed(lambda: [drained_step() for _ in range(a.steps)])
    wall, wall_max = timed(pipelined)
    subs = [(p, L_, o) for (p, L_, _), o in zip(subs, outs[(a.steps - 1) & 1])]
    stats = q.stats()
    q.close()
    payload = float(sum(x.sum() for x in lk))
    value = payload * world * a.steps / wall_max / GIB
    par = None
    if a.parity_sample:
        ps = []
        for j in range(K):
            idx = c3_sample(lk[j], np.argsort(-lk[j], kind="stable"), a.parity_sample // (2 * K), 5 + j)
            ps.append(sample_desc(big, starts[j] + ok_[j], lk[j], subs[j][2], idx))
        par = {"checked": sum(p["checked"] for p in ps), "mismatches": sum(p.get("mismatches", 0) for p in ps),
               "ok": all(p["ok"] for p in ps), "checker": ps[0]["checker"]}
    # PMC of the queue's BALANCED launches (one per pipelined step: K vectors)
    traffic, tnote = load_traffic(a.traffic, "md5_desc_balanced_t", f"c3q{K}@{a.c3_bytes}")
    vbusy = load_valu_busy(a.traffic, "md5_desc_balanced_t", f"c3q{K}@{a.c3_bytes}")
    res = {"metric": "device-resident MD5 GiB/s, mixed 4 KiB-1 MiB chunks (C3) through md5hip_queue",
           "value": round(value, 2), "unit": "GiB/s", "n_gpus": world, "steps": a.steps,
           "warmup": a.warmup, "ms_per_step": round(wall_max / a.steps * 1e3, 4),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
           "data": "synthetic", "tb_s": round(value * GIB / 1e12, 3),
           "config": {"workload": f"C3 stream: {K} submissions of 16 GiB mixed 4 KiB-1 MiB chunks "
                                  f"per step, device-resident, through md5hip_queue",
                      "submissions": K, "chunks": int(sum(x.size for x in lk)),
                      "payload_bytes": int(payload), "queue": stats},
           "roofline": {"bound": "hbm", "achieved": round(payload / (wall_max / a.steps) / 1e9, 1),
                        "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(payload / (wall_max / a.steps) / 1e9 / HBM_PEAK_GBS, 4),
                        "traffic": traffic, "traffic_source": tnote, "valu_busy_pmc": vbusy,
                        "kernel": "md5hip::md5_desc_balanced_t (queue launches)",
                        "note": "achieved: wall-clock per step (submit + wait); traffic: HBM bytes "
                                "per BALANCED launch, mean over a profiled run's launches (about "
                                "one per step of K vectors)"},
           "drained": {"value": round(payload * world * a.steps / wall_d_max / GIB, 2), "unit": "GiB/s",
                       "ms_per_step": round(wall_d_max / a.steps * 1e3, 4),
                       "note": "every step's tickets waited for before the next step submits: each "
                               "step's burst lingers on an idle queue until its first wait, then is "
                               "planned and launched while the device waits"}}
    return per_rank_line(res, rank, world, local, device, backend, payload * a.steps, wall, par)


def run_ctx(a, rank, world, local, device, backend):
    """Batched MD5Update on caller contexts (md5hip_update_ctx): one context
    per object, each step appends the next 16 KiB block of every object (the
    netcache streaming shape: objects arriving block by block).  A step = one
    md5hip_update_ctx launch over all contexts; MD5Final after timing."""
    import numpy as np
    L = a.len
    n = a.chunks or (1 << 20)
    data = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    m.fill_synthetic(data, seed=0x5EED0000 + rank)
    ctx = torch.zeros((n, 88), dtype=torch.uint8, device="cuda")
    m.init_ctx(ctx)
    ptrs = torch.arange(n, dtype=torch.int64, device="cuda") * L + data.data_ptr()
    lens = torch.full((n,), L, dtype=torch.int32, device="cuda")
    fn = lambda: m.update_ctx(ctx, ptrs, lens)  # noqa: E731
    wall, dev_ms = timed_steps(fn, a.steps, a.warmup, world)
    wall_max = shard.max_over_ranks(wall)
    dev_ms_max = shard.max_over_ranks(dev_ms)
    dig = m.final_ctx(ctx)
    # parity: each object hashed (warmup + steps) times its block -> the same
    # digest as MD5 over the block repeated; checked on a sample by the host reference
    par = None
    if a.parity_sample:
        k = min(n, max(16, a.parity_sample // 64))
        idx = np.unique(np.concatenate([[0, n - 1], np.random.default_rng(5).integers(0, n, k)]))
        rows = data.view(n, L)[torch.from_numpy(idx).to(data.device)].cpu().numpy()
        reps = a.warmup + a.steps
        rep = np.tile(rows, (1, reps)).reshape(-1)
        par = check_sample(rep, np.arange(idx.size, dtype=np.int64) * L * reps,
                           np.full(idx.size, L * reps), dig.index_select(0, torch.from_numpy(idx).to(dig.device)).cpu().numpy())
    alg = float(n) * (L + 2 * 88)
    achieved = alg / (dev_ms_max * 1e-3) / 1e9
    traffic, tnote = load_traffic(a.traffic, "md5_update_ctx", f"ctx@{n}x{L}")
    vbusy = load_valu_busy(a.traffic, "md5_update_ctx", f"ctx@{n}x{L}")
    res = {"metric": "device-resident batched MD5Update GiB/s (md5hip_update_ctx, 16 KiB per context per call)",
           "value": round(float(n) * L * world * a.steps / wall_max / GIB, 2), "unit": "GiB/s",
           "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
           "ms_per_step": round(wall_max / a.steps * 1e3, 4), "higher_is_better": True, "scaling": "weak",
           "vs_baseline": None, "dtype": "u32", "data": "synthetic",
           "config": {"workload": f"{n} contexts x {L} B per update", "contexts": n, "update_bytes": L},
           "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                        "frac": round(achieved / HBM_PEAK_GBS, 4), "kernel": "md5hip::md5_update_ctx",
                        "avg_launch_ms": round(dev_ms_max, 4), "alg_bytes_per_launch": int(alg),
                        "alg_bytes_note": "block bytes + the 88-B context read and written",
                        "traffic": traffic, "traffic_source": tnote, "valu_busy_pmc": vbusy}}
    return per_rank_line(res, rank, world, local, device, backend, float(n) * L * a.steps, wall, par)


def c5_sample(arr, dig, n, L, per, k, seed):
    """C5 parity: the first and last chunk, both sides of every slot
    boundary (a slot holds `per` chunks: the batcher's slice / L), and k
    distinct random chunks, re-digested from the host buffer after timing."""
    import numpy as np
    b = np.arange(per, n, per, dtype=np.int64)
    rnd = np.random.default_rng(seed).choice(n, size=min(k, n), replace=False)
    idx = np.unique(np.concatenate([[0, n - 1], b - 1, b, rnd]))
    par = check_sample(arr, idx * L, np.full(idx.size, L), dig[idx])
    par["sample"] = (f"first + last + both sides of {b.size} slot boundaries + {min(k, n)} distinct "
                     f"random chunks, re-digested on the host after the timed region")
    return par


def run_c5(a, rank, world, local, device, backend):
    """End to end from pinned host memory: H2D -> MD5 -> D2H over pipelined
    batcher slots (md5hip_batch_host_fixed)."""
    n, L = a.c5_chunks, a.len
    host = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
    host.view(torch.int64).random_(generator=torch.Generator().manual_seed(5))
    arr = host.numpy()
    # PCIe H2D alone (the denominator for this config): the same slices, on one
    # stream and round-robin over as many streams as the batcher has slots
    # (concurrent DMA); the best of four passes of each, warmed up (a single
    # pass of each read the link up to 6 % low on some boxes, above the
    # pipeline's own rate)
    nsl = 3
    devs = [torch.empty(a.c5_slice, dtype=torch.uint8, device="cuda") for _ in range(nsl)]
    streams = [torch.cuda.Stream() for _ in range(nsl)]
    per = a.c5_slice
    h2d_gbs = 0.0
    for nst in (1, nsl) * 4:
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
            dig = b.host_fixed(arr, n, L)
        wall = time.perf_counter() - t0
    gbs = n * L * a.steps / wall / 1e9
    par = c5_sample(arr, dig, n, L, a.c5_slice // L, a.parity_sample, 55 + rank) if a.parity_sample else None
    res = {"metric": "end-to-end MD5 GiB/s from pinned host memory (C5)",
           "value": round(n * L * a.steps / wall / GIB, 2), "unit": "GiB/s", "n_gpus": world,
           "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(wall / a.steps * 1e3, 3),
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u32",
           "data": "synthetic (host random)", "config": {"workload": "C5", "chunks": n,
                                                         "chunk_bytes": L, "slice_bytes": a.c5_slice,
                                                         "slots": 3},
           "roofline": {"bound": "pcie", "achieved": round(gbs, 2), "peak": round(h2d_gbs, 2),
                        "unit": "GB/s", "frac": round(gbs / h2d_gbs, 4),
                        "peak_note": (f"measured pinned H2D copy alone, best of 4 passes on 1 and "
                                      f"on {nsl} streams; spec {PCIE_PEAK_GBS} GB/s"),
                        "traffic": None}}
    return per_rank_line(res, rank, world, local, device, backend, n * L * a.steps, wall, par)


def board_probe(fn, device, ms_per_launch, seconds=1.5):
    """What the board does under the C2 kernel (the line
    had no way to show the power cap): after the timed region, the same
    launches again for ~`seconds` while amdsmi's gpu_metrics are sampled
    every 10 ms -- the current gfx clock (mean over the XCDs), socket power,
    and the share of the window the package-power limit (PPT) held the
    clock down.  Never part of `value`; {"error": ...} where amdsmi cannot
    read the board (a box that hides the metrics)."""
    import statistics
    try:
        import amdsmi
        amdsmi.amdsmi_init()
    except Exception as e:  # pragma: no cover - depends on the box
        return {"error": f"amdsmi: {e!r}"[:200]}
    try:
        p = torch.cuda.get_device_properties(device)
        want = (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0), getattr(p, "pci_device_id", 0))
        handle = None
        for h in amdsmi.amdsmi_get_processor_handles():
            b = amdsmi.amdsmi_get_gpu_device_bdf(h)            # "dddd:bb:dd.f"
            dom, bus, rest = b.split(":")
            if (int(dom, 16), int(bus, 16), int(rest.split(".")[0], 16)) == want:
                handle = h
        if handle is None:
            return {"error": f"no amdsmi device at {want}"}
        met = lambda: amdsmi.amdsmi_get_gpu_metrics_info(handle)  # noqa: E731

        def num(x):
            return float(x) if isinstance(x, (int, float)) and x not in (0xFFFF, 0xFFFFFFFF) else None

        m0 = met()
        launches = max(10, int(seconds * 1e3 / max(ms_per_launch, 0.05)))
        stream = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        e0.record(stream)
        for _ in range(launches):
            fn()
        e1.record(stream)
        clk, pw = [], []
        t_end = time.perf_counter() + seconds * 3
        while not e1.query() and time.perf_counter() < t_end:
            mm = met()
            cs = [num(c) for c in (mm.get("current_gfxclks") or []) if num(c)]
            c = statistics.fmean(cs) if cs else num(mm.get("current_gfxclk"))
            w = num(mm.get("current_socket_power")) or num(mm.get("average_socket_power"))
            if c:
                clk.append(c)
            if w:
                pw.append(w)
            time.sleep(0.01)
        torch.cuda.synchronize()
        m1 = met()
        acc0, acc1 = num(m0.get("accumulation_counter")), num(m1.get("accumulation_counter"))
        ppt0, ppt1 = num(m0.get("ppt_residency_acc")), num(m1.get("ppt_residency_acc"))
        ppt = (round((ppt1 - ppt0) / (acc1 - acc0), 3)
               if None not in (acc0, acc1, ppt0, ppt1) and acc1 > acc0 else None)
        # trim the first and last fifth of the samples (clock ramp, drain)
        k = len(clk) // 5
        mid = clk[k:len(clk) - k] or clk
        kp = len(pw) // 5
        midp = pw[kp:len(pw) - kp] or pw
        return {"launches": launches, "ms_per_launch": round(e0.elapsed_time(e1) / launches, 4),
                "samples": len(clk),
                "gfxclk_mhz_median": round(statistics.median(mid), 1) if mid else None,
                "socket_power_w_median": round(statistics.median(midp), 1) if midp else None,
                "ppt_limited_frac": ppt,
                "note": "the C2 launches again after the timed region; amdsmi gpu_metrics every 10 ms "
                        "(current_gfxclks mean over XCDs, current_socket_power, ppt_residency_acc)"}
    except Exception as e:  # pragma: no cover - depends on the box
        return {"error": repr(e)[:200]}
    finally:
        try:
            amdsmi.amdsmi_shut_down()
        except Exception:
            pass


EXTRA_STEPS = {"c3q": (8, 3), "c5": (5, 2)}     # (steps, warmup) of a sub-record


def run_extra(name, a, rank, world, local, device, backend):
    """A BASELINE config beside the headline (C3 as the queue streams it, C5
    end to end), run after C2's timed region and parity in the same process,
    so the driver's own run carries it: the config's own timing, roofline and
    parity, nothing of it inside C2's measurement."""
    import copy
    b = copy.copy(a)
    b.steps, b.warmup = EXTRA_STEPS[name]
    torch.cuda.empty_cache()
    t0 = time.perf_counter()
    r = {"c3q": run_c3q, "c5": run_c5}[name](b, rank, world, local, device, backend)
    keep = ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "tb_s", "roofline", "drained",
            "parity", "config")
    out = {k: r[k] for k in keep if k in r}
    out["run_s"] = round(time.perf_counter() - t0, 2)
    return out


def main(argv=None):
    global torch, m, shard
    argv = sys.argv[1:] if argv is None else list(argv)
    a = parse_args(argv)
    if a.gpus < 1:
        raise SystemExit("bench.py: --gpus must be >= 1")
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a, argv))           # before anything touches the GPU
    import torch as _torch
    torch = _torch
    sys.path.insert(0, REPO)
    from sproxy_amd import md5 as _m, shard as _shard
    m, shard = _m, _shard
    rank, world, local, device, backend = dist_setup(a)
    if a.dry_run:
        res = run_dry(a, rank, world, local, device, backend)
    else:
        res = {"c2": run_c2, "c3": run_c3, "c3q": run_c3q, "c5": run_c5, "crc": run_crc,
               "crcq": run_crcq, "ctx": run_ctx}[a.config](a, rank, world, local, device, backend)
    if a.config == "c2" and world == 1 and not a.dry_run and a.extras != "none":
        for name in [x for x in a.extras.split(",") if x]:
            if name not in EXTRA_STEPS:
                raise SystemExit(f"bench.py: --extras {name}: one of {sorted(EXTRA_STEPS)} or none")
            res[name] = run_extra(name, a, rank, world, local, device, backend)
    if rank == 0 and world == 1 and not a.dry_run and not a.no_cpu_baseline:
        if a.config == "c2":
            res["cpu_baseline"] = cpu_baseline()
            # labelled separately: the same reference md5.c on the box's CPU share
            res["cpu_baseline_all_cores"] = cpu_baseline(reps=10, threads=CPU_SHARE)
        elif a.config == "crc":
            res["cpu_baseline"] = cpu_baseline_crc()
    if rank == 0:
        print(json.dumps(res), flush=True)
    shard.close_group()


if __name__ == "__main__":
    main()
