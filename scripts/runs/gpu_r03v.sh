#!/bin/bash
# Round-3 call V: CRC split as AUTO's choice up to 16 chunks per CU -- full
# GPU suite, CRC call latency through the queue against the library before
# the split, and the MD5 call latency again on this box.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --crc --iters 300 --lib product=sproxy_amd/lib/libmd5hip.so before=build/abr03/libmd5hip_nosplit.so > $O/crc_latency_ab.json 2> $O/crc_latency_ab.err; r=$?
tail -c 1200 $O/crc_latency_ab.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --iters 300 --lib product=sproxy_amd/lib/libmd5hip.so before=build/abr03/libmd5hip_lane_small.so > $O/queue_latency_ab.json 2> $O/queue_latency_ab.err; r=$?
tail -c 1200 $O/queue_latency_ab.json
exit $r
