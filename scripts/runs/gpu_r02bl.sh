#!/bin/bash
# Round-2 call BK/BL: device-queue call latency: OLD, POLL (waiter-aware polling), NEW (+ digests written in place)
# then the queue / batcher GPU tests and the c3q line on NEW.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bl
mkdir -p $O
timeout -k 10 300 python3 -u scripts/latency_probe.py --iters 200 --lib old=build/ab/libmd5hip_prepoll.so poll=build/ab/libmd5hip_poll.so new=sproxy_amd/lib/libmd5hip.so > $O/latency.log 2>&1; r=$?
tail -c 1500 $O/latency.log; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_queue.py tests/test_c_site.py tests/test_gpu_parity.py -m gpu -k "queue or batcher or site or pool or host" > $O/pytest.log 2>&1; r=$?
tail -2 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py --config c3q --steps 10 > $O/c3q.json 2> $O/c3q.err; r=$?
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print('c3q', d['value'])"
exit $r
