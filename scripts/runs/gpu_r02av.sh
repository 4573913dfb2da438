#!/bin/bash
# Round-2 call AV: the new HYBRID long-group edge-case test on the GPU.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02av
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_parity.py -m gpu -k "hybrid_long_group_edges or long_and_short" > $O/pytest.log 2>&1; r=$?
tail -8 $O/pytest.log; exit $r
