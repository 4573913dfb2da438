#!/bin/bash
# Round-5 call M: the randomized call-site stress on the round-5 tree, now
# with device-resident fixed-length runs and fastcrc page lists (windowed
# staging) beside the pool, queue and CRC-queue paths; every digest checked.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05m
mkdir -p $O
timeout -k 10 240 python3 -u scripts/stress_pool.py --secs 90 --threads 12 > $O/stress_pool.json 2> $O/stress.err
rc=$?; tail -c 1500 $O/stress_pool.json; [ $rc = 0 ] || { echo "stress failed $rc"; tail -5 $O/stress.err; exit 1; }
echo done
