#!/bin/bash
# Round-2 call S: MD5Update on contexts through the LDS-DMA loader.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02s
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_ctx.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --config ctx > $O/ctx.json 2> $O/ctx.err; r=$?
echo "ctx rc=$r"; cut -c1-700 $O/ctx.json; exit $r
