#!/bin/bash
# Round-2 call X: planner threshold -- product BALANCED / HYBRID / XDMA on
# 2, 3, 4 coalesced C3 batches, 5 interleaved rounds.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02x
mkdir -p $O
timeout -k 10 500 python3 -u scripts/c3_wide_ab.py --batches 2 3 4 --rounds 5 --kinds > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/ab.json | cut -c1-3000
