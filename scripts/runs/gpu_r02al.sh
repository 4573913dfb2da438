#!/bin/bash
# Round-2 call AL: batcher plans from its key histogram, order built on the
# device -- queue / batcher tests, c3q lines, queue probe.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02al
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_queue.py tests/test_nc_digest.py tests/test_c_site.py tests/test_gpu_parity.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --config c3q --steps 10 --warmup 2 > $O/c3q.json 2> $O/c3q.err || exit 1
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print(d['value'], d['tb_s'], d['drained'], d['config']['queue'], d.get('parity'))"
timeout -k 10 300 python3 -u scripts/queue_probe.py > $O/probe.json 2> $O/probe.err || exit 1
python3 -c "
import json;d=json.load(open('$O/probe.json'))
for x in d['log']:
  if 'drained' in x[1]: print(x)"
