#!/bin/bash
# Round-4 call W: the final tree once more (after the last batcher change):
# the whole GPU suite and smoke(); the driver's exact bench command; c3q;
# bench.py --gpus 2 spawning its own two gloo ranks on the one GPU.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err || { echo "c2 driver failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c2_driver.json').read().strip().splitlines()[-1]);print('c2 driver', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -k 10 300 python3 bench.py --config c3q --no-cpu-baseline > $O/c3q.json 2> $O/c3q.err || { echo "c3q failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['value'])"
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 5 --no-cpu-baseline > $O/n2_gloo.json 2> $O/n2_gloo.err || { echo "n2 failed"; tail -5 $O/n2_gloo.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/n2_gloo.json').read().strip().splitlines()[-1]);print('n2', d['value'], d['n_gpus'], d['ms_per_step'], d['ranks_seen']['world'], d['parity']['ok'])"
echo done
