#!/bin/bash
# Round-2 call AD: c3q with a flush at stream start, inflight 1 default;
# 10 pipelined steps; queue probe.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ad
mkdir -p $O
for s in 5 10; do
  timeout -k 10 300 python bench.py --config c3q --steps $s --warmup 2 > $O/c3q_s$s.json 2> $O/c3q_s$s.err; r=$?
  echo "c3q steps $s rc=$r"; [ $r -eq 0 ] || exit $r
  python3 -c "import json;d=json.loads(open('$O/c3q_s$s.json').read().strip().splitlines()[-1]);print(d['value'], d['tb_s'], d['ms_per_step'], d['drained'], d['config']['queue'], d.get('parity'))"
done
