#!/bin/bash
# Round-4 call L: chain mode 2 (BALANCED launches overlap their tails: no
# device-side wait) against mode 1, c3q bench interleaved 1,2,1,2,1,2; then
# the kernel timeline of a mode-2 run.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_queue.py > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -5 $O/pytest.log; exit 1; }
for r in 1 2 3; do
  for c in 1 2; do
    timeout -k 10 300 python3 bench.py --config c3q --no-cpu-baseline --c3q-chain $c > $O/c3q_chain${c}_$r.json 2> $O/c3q_chain${c}_$r.err || { echo "c3q failed"; tail -3 $O/c3q_chain${c}_$r.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/c3q_chain${c}_$r.json').read().strip().splitlines()[-1]);print('chain $c', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['value'], d['parity']['ok'])"
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace2 -o trace -- python3 bench.py --config c3q --steps 10 --no-cpu-baseline --c3q-chain 2 > $O/c3q_traced2.json 2> $O/c3q_traced2.err || { echo "traced failed"; exit 1; }
echo done
