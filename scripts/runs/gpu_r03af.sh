#!/bin/bash
# Round-3 call AF: fastcrc windows through the split kernel (two messages per
# chunk, F other than 64/128) -- CRC GPU tests, small-batch times at F = 4096
# and 1000 against the windowed LDS-DMA kernel, and the cached CU count.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03af
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_crc32.py tests/test_queue.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
for F in 4096 1000; do
  timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --crc --fastcrc $F --sizes 64,1024,4096 > $O/crc_small_f$F.json 2> $O/crc_small_f$F.err; r=$?
  tail -3 $O/crc_small_f$F.err | cut -c1-300; [ $r -eq 0 ] || exit $r
done
timeout -k 10 300 python3 -u scripts/latency_probe.py --crc --iters 300 > $O/crc_latency.json 2> $O/crc_latency.err; r=$?
tail -c 500 $O/crc_latency.json
exit $r
