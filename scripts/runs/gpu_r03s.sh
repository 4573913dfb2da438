#!/bin/bash
# Round-3 call S: FED (fed pairs) as the planner's choice for small batches --
# full GPU suite, call latency against the library before it (LANE for small
# batches), the pool's call site, and the product descriptor kernels on small
# batches.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --iters 300 --lib product=sproxy_amd/lib/libmd5hip.so before=build/abr03/libmd5hip_lane_small.so > $O/queue_latency_ab.json 2> $O/queue_latency_ab.err; r=$?
tail -c 1500 $O/queue_latency_ab.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/pool_latency_probe.py --iters 100 --threads 8 --secs 2 > $O/pool_latency.json 2> $O/pool_latency.err; r=$?
echo "pool rc=$r"; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --sizes 16,64,256,1024,4096,16384,32768 > $O/small_batch_16k.json 2> $O/small_batch_16k.err; r=$?
cat $O/small_batch_16k.err
exit $r
