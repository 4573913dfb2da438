#!/bin/bash
# Round-2 call BN: the queue tests incl. in-place / scattered device digests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bn
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_queue.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -16 $O/pytest.log; exit $r
