#!/bin/bash
# Round-4 call AD: the final tree after the synchronous slot policy: the
# whole GPU suite and smoke(), then the randomized stress at 64 threads.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ad
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 170 python3 -u scripts/stress_pool.py --secs 60 --threads 64 > $O/stress_t64.json 2> $O/stress_t64.err || { echo "stress failed"; tail -5 $O/stress_t64.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/stress_t64.json').read().strip().splitlines()[-1]);print('stress', sum(d['ops'].values()), d['errors'])"
echo done
