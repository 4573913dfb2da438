#!/bin/bash
# Round-5 call V: does a one-rank RCCL group slow the C2 kernel?  (round 2's
# and r05u's --dist-always lines: 3.19-3.26 ms per launch against 2.90.)
# The same bench command plain, with a gloo group, with an RCCL group, and
# under torch.distributed.run; then the RCCL one under rocprofv3 kernel-trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
one() {  # name args...
  local name=$1; shift
  timeout -k 10 300 "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; tail -3 $O/$name.err; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('$O/$name.json').read().splitlines() if l.startswith('{')][-1]);print('$name', d['value'], d['ms_per_step'], d['roofline'].get('avg_launch_ms'), d['ranks_seen']['backend'], d['ranks_seen']['world'])"
}
B="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline"
one plain python3 $B
one gloo1 python3 $B --dist-always --dist-backend gloo
one nccl1 python3 $B --dist-always
one plain2 python3 $B
one torchrun1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 $B --dist-always
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_nccl1 -o nccl1 -- python3 $B --dist-always > $O/prof_nccl1.log 2>&1 || { echo "prof failed"; exit 1; }
python3 - "$O/prof_nccl1/nccl1_kernel_trace.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
names = {}
for r in rows:
    names[r["Kernel_Name"][:60]] = names.get(r["Kernel_Name"][:60], 0) + 1
print(names)
d = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if "xdma1nt" in r["Kernel_Name"]]
print("xdma1nt launches", len(d), [round(x, 3) for x in d])
PY
echo done
