#!/bin/bash
# Round-2 call AB: waits no longer force launches beside running ones;
# parallel planner -- queue tests, c3q lines, queue timeline.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ab
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_queue.py tests/test_nc_digest.py tests/test_c_site.py tests/test_abi.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
for f in 1 2; do
  timeout -k 10 300 python bench.py --config c3q --c3q-inflight $f --steps 5 --warmup 2 > $O/c3q_f$f.json 2> $O/c3q_f$f.err; r=$?
  echo "c3q f$f rc=$r"; [ $r -eq 0 ] || exit $r
  python3 -c "import json;d=json.loads(open('$O/c3q_f$f.json').read().strip().splitlines()[-1]);print(d['value'], d['tb_s'], d['drained']['value'], d['config']['queue'], d['ranks_seen']['ranks'][0]['parity'] if 'ranks_seen' in d else '')"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o c3q -- python3 bench.py --config c3q --c3q-inflight 1 --steps 5 --warmup 2 --parity-sample 0 > $O/c3q_trace.log 2>&1; r=$?
echo "trace rc=$r"; [ $r -eq 0 ] || exit $r
python3 scripts/queue_gaps.py $O/trace > $O/gaps.json; head -5 $O/gaps.json
