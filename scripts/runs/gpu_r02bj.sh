#!/bin/bash
# Round-2 call BJ: rocprofv3 --kernel-trace --stats of every bench line on the final tree
# (the kernel averages beside each line's own hipEvent numbers).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bj
mkdir -p $O
prof() {  # name args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$name -o $name -- python3 bench.py --no-cpu-baseline "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; return 1; }
  python3 -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$name', d['value'], d.get('ms_per_step'), r.get('avg_launch_ms'))"
  head -3 $(ls $O/prof_$name/*kernel_stats.csv | head -1) | cut -c1-200
}
prof c2 && prof c3 --config c3 && prof c3q --config c3q --steps 10 && prof ctx --config ctx && \
prof crc0 --config crc && prof crc128 --config crc --fastcrc 128 && prof c5 --config c5
