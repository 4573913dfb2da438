#!/bin/bash
# Round-3 call P: LANE for small batches -- GPU suite, then call latency
# against the previous library (XDMA for small batches), interleaved.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --iters 300 --lib product=sproxy_amd/lib/libmd5hip.so before=build/abr03/libmd5hip_xdma_small.so > $O/queue_latency_ab.json 2> $O/queue_latency_ab.err; r=$?
tail -c 1500 $O/queue_latency_ab.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/pool_latency_probe.py --iters 100 --threads 8 --secs 2 > $O/pool_latency.json 2> $O/pool_latency.err; r=$?
echo "pool rc=$r"
exit $r
