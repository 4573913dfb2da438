#!/bin/bash
# Round-3 call AJ: the randomized 12-thread stress with CRC-32 queue traffic
# added (split kernel by the slot's mean length, caller polling, in-place
# descriptors), 90 s, every digest and CRC checked.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
timeout -k 10 300 python3 -u scripts/stress_pool.py --secs 90 --threads 12 > $O/stress_pool.json 2> $O/stress_pool.err; r=$?
tail -c 900 $O/stress_pool.json; tail -3 $O/stress_pool.err
exit $r
