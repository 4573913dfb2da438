#!/bin/bash
# Round-3 call AB: length-aware CRC split choice (fixed API and the batcher's
# mean chunk length) -- CRC, queue and pool GPU tests, CRC call latency.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_crc32.py tests/test_queue.py tests/test_pool.py tests/test_gpu_parity.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --crc --iters 200 > $O/crc_latency.json 2> $O/crc_latency.err; r=$?
tail -c 700 $O/crc_latency.json
exit $r
