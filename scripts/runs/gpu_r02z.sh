#!/bin/bash
# Round-2 call Z: where the queue's time goes -- kernel trace of the c3q line
# (gaps between launches), plus the new ctx test.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02z
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ctx.py tests/test_queue.py tests/test_nc_digest.py tests/test_c_site.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o c3q -- python3 bench.py --config c3q --c3q-inflight 1 --steps 5 --warmup 2 --parity-sample 0 > $O/c3q.log 2>&1; r=$?
echo "trace rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/c3q.log | cut -c1-200
python3 scripts/queue_gaps.py $O/trace > $O/gaps.json; cat $O/gaps.json | head -60
