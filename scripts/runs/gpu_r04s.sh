#!/bin/bash
# Round-4 call S: descriptors of large device-resident submissions copied at
# submit time; the guard-free BALANCED quads.  Queue/pool/C3 GPU tests, c3q
# twice, the drained-step breakdown, then PMC traffic for every bench line's
# kernel on this tree.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_queue.py tests/test_pool.py tests/test_c3_full.py tests/test_lines.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config c3q --no-cpu-baseline > $O/c3q_$r.json 2> $O/c3q_$r.err || { echo "c3q failed"; tail -3 $O/c3q_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c3q_$r.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['value'], d['parity']['ok'])"
done
timeout -s KILL 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/c3q_trace -o trace -- python3 scripts/c3q_breakdown.py --steps 6 --out $O/c3q_stamps.json > $O/c3q_breakdown.log 2>&1 || { echo "c3q breakdown failed"; tail -3 $O/c3q_breakdown.log; exit 1; }
python3 scripts/c3q_breakdown.py --join $O/c3q_trace --stamps $O/c3q_stamps.json --out $O/c3q_breakdown.json >> $O/c3q_breakdown.log 2>&1
tail -1 $O/c3q_breakdown.log
bash scripts/gpu_pmc_traffic.sh $O/pmc || { echo "pmc failed"; exit 1; }
echo done
