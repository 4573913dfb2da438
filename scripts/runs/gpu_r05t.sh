#!/bin/bash
# Round-5 call T: the randomized call-site stress at 64 threads for 60 s on
# the final tree (device-resident fixed runs and fastcrc page lists included).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 240 python3 -u scripts/stress_pool.py --secs 60 --threads 64 > $O/stress_t64.json 2> $O/stress.err
rc=$?; tail -c 1500 $O/stress_t64.json; [ $rc = 0 ] || { echo "stress failed $rc"; tail -5 $O/stress.err; exit 1; }
echo done
