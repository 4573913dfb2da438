#!/bin/bash
# Round-5 call A: baseline on a fresh box -- the whole GPU suite and the
# driver's bench command, before any round-5 change.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err || { echo "c2 driver failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c2_driver.json').read().strip().splitlines()[-1]);print('c2 driver', d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo done
