#!/bin/bash
# Round-5 call W: the C2 line with no process group, a one-rank gloo group and
# a one-rank RCCL group, interleaved three times each (r05v: RCCL 3.04-3.10 ms
# per launch against 2.92 plain and gloo).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
B="bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --parity-sample 0"
for r in 1 2 3; do
  for v in nccl plain gloo; do
    case $v in
      plain) extra="";;
      gloo) extra="--dist-always --dist-backend gloo";;
      nccl) extra="--dist-always";;
    esac
    timeout -k 10 300 python3 $B $extra > $O/${v}_$r.json 2> $O/${v}_$r.err || { echo "$v $r failed"; tail -3 $O/${v}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads([l for l in open('$O/${v}_$r.json').read().splitlines() if l.startswith('{')][-1]);print('$v', $r, d['value'], d['roofline'].get('avg_launch_ms'))"
  done
done
echo done
