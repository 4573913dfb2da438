#!/bin/bash
# Round-6 call H: the randomized call-site stress on the final tree, now with
# vectors past 4,096 chunks (the stable device order and its fallback), 12
# threads for 90 s, then 64 threads for 60 s.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06h
mkdir -p $O
timeout -k 10 240 python3 -u scripts/stress_pool.py --secs 90 --threads 12 > $O/stress_pool.json 2> $O/stress.err
rc=$?; tail -c 1500 $O/stress_pool.json; [ $rc = 0 ] || { echo "stress failed $rc"; tail -5 $O/stress.err; exit 1; }
timeout -k 10 240 python3 -u scripts/stress_pool.py --secs 60 --threads 64 > $O/stress_t64.json 2> $O/stress_t64.err
rc=$?; tail -c 1500 $O/stress_t64.json; [ $rc = 0 ] || { echo "stress t64 failed $rc"; tail -5 $O/stress_t64.err; exit 1; }
echo done
