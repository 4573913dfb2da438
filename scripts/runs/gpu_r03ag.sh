#!/bin/bash
# Round-3 call AG: windows split only from 2 KiB -- CRC / queue / pool GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ag
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_crc32.py tests/test_queue.py tests/test_pool.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log
exit $r
