#!/bin/bash
# Round-3 call K: 90 s randomized stress of the pool router and the device
# queue from 12 threads (scripts/stress_pool.py), every digest checked.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 240 python3 -u scripts/stress_pool.py --secs 90 --threads 12 --devices 3 > $O/stress.json 2> $O/stress.err; r=$?
echo "rc=$r"; tail -3 $O/stress.err; cat $O/stress.json
exit $r
