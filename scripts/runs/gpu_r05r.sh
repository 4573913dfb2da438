#!/bin/bash
# Round-5 call R: the queue tests after adding device-resident fixed runs off
# the 16-B grid.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05r
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_queue.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; grep -E "FAIL|Error|assert" $O/pytest.log | head -8; exit 1; }
echo done
