#!/bin/bash
# Round-2 call M: BALANCED shapes under the default cache policy.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02m
mkdir -p $O
timeout -k 10 300 python3 -u scripts/c3_wide_ab.py --batches 2 3 5 --rounds 3 --kinds 19 20 21 23 22 16 > $O/wide.json 2> $O/wide.err; r=$?
echo "wide rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/wide.json | cut -c1-3500
