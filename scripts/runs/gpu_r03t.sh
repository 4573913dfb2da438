#!/bin/bash
# Round-3 call T: FED for small batches + blocked callers watching their own
# launch -- full GPU suite, a 60 s randomized 12-thread stress of the pool and
# queue, call latency against the library before both changes (LANE) and
# with FED only, and the pool's call site.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 200 python3 -u scripts/stress_pool.py --secs 60 --threads 12 > $O/stress_pool.json 2> $O/stress_pool.err; r=$?
tail -c 800 $O/stress_pool.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --iters 300 --lib product=sproxy_amd/lib/libmd5hip.so fed_only=build/abr03/libmd5hip_fed_nowatch.so before=build/abr03/libmd5hip_lane_small.so > $O/queue_latency_ab.json 2> $O/queue_latency_ab.err; r=$?
tail -c 1500 $O/queue_latency_ab.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/pool_latency_probe.py --iters 100 --threads 8 --secs 2 > $O/pool_latency.json 2> $O/pool_latency.err; r=$?
tail -c 1500 $O/pool_latency.json
exit $r
