#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02am
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k order_device -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; exit $r
