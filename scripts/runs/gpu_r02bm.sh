#!/bin/bash
# Round-2 call BM: final check after the batcher latency changes -- GPU suite, smoke, the default bench
# line, the 2-rank spawn (gloo) and a one-rank nccl group.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bm
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -2 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; r=$?
tail -1 $O/smoke.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py > $O/c2.json 2> $O/c2.err; r=$?
[ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 5 > $O/n2_gloo.json 2> $O/n2_gloo.err; r=$?
[ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --gpus 1 --dist-always --steps 10 --warmup 5 --no-cpu-baseline > $O/nccl1.json 2> $O/nccl1.err; r=$?
for f in c2 n2_gloo nccl1; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', d['value'], d['n_gpus'], r.get('frac'), r.get('traffic'), r.get('valu_busy_pmc'), (d.get('parity') or {}).get('ok'))"; done
exit $r
