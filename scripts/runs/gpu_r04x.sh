#!/bin/bash
# Round-4 call X: randomized stress of the final batcher / pool / queues on
# the GPU: 12 threads for 90 s, then 64 threads for 60 s (every digest and
# CRC checked against the oracle's).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04x
mkdir -p $O
timeout -k 10 200 python3 -u scripts/stress_pool.py --secs 90 --threads 12 > $O/stress_t12.json 2> $O/stress_t12.err || { echo "stress 12 failed"; tail -5 $O/stress_t12.err; tail -2 $O/stress_t12.json; exit 1; }
tail -c 400 $O/stress_t12.json; echo
timeout -k 10 170 python3 -u scripts/stress_pool.py --secs 60 --threads 64 > $O/stress_t64.json 2> $O/stress_t64.err || { echo "stress 64 failed"; tail -5 $O/stress_t64.err; tail -2 $O/stress_t64.json; exit 1; }
tail -c 400 $O/stress_t64.json; echo
echo done
