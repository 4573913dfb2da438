#!/bin/bash
# Round-4 call M: chain lead cap (MD5HIP_CHAIN_LEAD_US) 2 ms vs 5 ms under
# chain mode 2, c3q interleaved x3, plus a mode-2 kernel trace at 5 ms.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
for r in 1 2 3; do
  for L in 2000 5000; do
    MD5HIP_CHAIN_LEAD_US=$L timeout -k 10 300 python3 bench.py --config c3q --no-cpu-baseline > $O/c3q_lead${L}_$r.json 2> $O/c3q_lead${L}_$r.err || { echo "c3q failed"; tail -3 $O/c3q_lead${L}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/c3q_lead${L}_$r.json').read().strip().splitlines()[-1]);print('lead $L', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['value'], d['parity']['ok'])"
  done
done
echo done
