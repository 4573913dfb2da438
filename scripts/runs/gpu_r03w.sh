#!/bin/bash
# Round-3 call W: small slots' kernels read the pinned (fine-grained)
# descriptors in place instead of two H2D copies -- full GPU suite, the
# randomized pool/queue stress, MD5 and CRC call latency against the library
# with the copies (and, for MD5, the LANE library of round 3's start).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 200 python3 -u scripts/stress_pool.py --secs 60 --threads 12 > $O/stress_pool.json 2> $O/stress_pool.err; r=$?
tail -c 600 $O/stress_pool.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --crc --iters 300 --lib product=sproxy_amd/lib/libmd5hip.so copies=build/abr03/libmd5hip_desc_copy.so before=build/abr03/libmd5hip_nosplit.so > $O/crc_latency_ab.json 2> $O/crc_latency_ab.err; r=$?
tail -c 1500 $O/crc_latency_ab.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --iters 300 --lib product=sproxy_amd/lib/libmd5hip.so copies=build/abr03/libmd5hip_desc_copy.so before=build/abr03/libmd5hip_lane_small.so > $O/queue_latency_ab.json 2> $O/queue_latency_ab.err; r=$?
tail -c 1500 $O/queue_latency_ab.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/pool_latency_probe.py --iters 100 --threads 8 --secs 2 > $O/pool_latency.json 2> $O/pool_latency.err; r=$?
echo "pool rc=$r"
exit $r
