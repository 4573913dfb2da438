#!/bin/bash
# Round-3 call I: the pool tests with the refused-submission case.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_pool.py tests/test_queue.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log
exit $r
