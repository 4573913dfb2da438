#!/bin/bash
# Round-5 call G: the fastcrc stream with two steps' worth of queue slots,
# at 4 x 1 M, 2 x 2 M and 8 x 1 M blocks per step; queue tests after the
# binding change.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_queue.py tests/test_crc32.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
for cfg in "4 1048576" "2 2097152" "8 1048576"; do
  set -- $cfg
  timeout -k 10 300 python3 bench.py --config crcq --crcq-subs $1 --crcq-chunks $2 --steps 10 --warmup 2 > $O/crcq_$1x$2.json 2> $O/crcq_$1x$2.err || { echo "crcq $cfg failed"; tail -3 $O/crcq_$1x$2.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/crcq_$1x$2.json').read().strip().splitlines()[-1]);print('crcq', '$cfg', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['frac'], d.get('parity',{}).get('ok'))"
done
echo done
