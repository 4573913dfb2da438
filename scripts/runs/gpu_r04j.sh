#!/bin/bash
# Round-4 call J: non-temporal descriptor stores in reserve_device.  Queue and
# pool GPU tests, the c3q bench twice, the submit-cost probe, the c3q step
# breakdown under a kernel + copy trace.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_queue.py tests/test_pool.py tests/test_c3_full.py tests/test_lines.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config c3q --no-cpu-baseline > $O/c3q_$r.json 2> $O/c3q_$r.err || { echo "c3q failed"; tail -3 $O/c3q_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c3q_$r.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['value'], d['parity']['ok'])"
done
timeout -k 10 300 python3 -u scripts/probes/submit_cost.py --bursts 8 --out $O/submit_cost.json > $O/submit_cost.log 2>&1 || { echo "submit probe failed"; tail -3 $O/submit_cost.log; exit 1; }
tail -1 $O/submit_cost.log | cut -c1-400
timeout -s KILL 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/c3q_trace -o trace -- python3 scripts/c3q_breakdown.py --steps 6 --out $O/c3q_stamps.json > $O/c3q_breakdown.log 2>&1 || { echo "c3q breakdown failed"; tail -3 $O/c3q_breakdown.log; exit 1; }
python3 scripts/c3q_breakdown.py --join $O/c3q_trace --stamps $O/c3q_stamps.json --out $O/c3q_breakdown.json >> $O/c3q_breakdown.log 2>&1
tail -1 $O/c3q_breakdown.log
echo done
