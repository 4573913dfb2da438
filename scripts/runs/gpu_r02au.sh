#!/bin/bash
# Round-2 call AU: HYBRID on the C3 batch at 3 / 2 / 1 waves per SIMD (scripts/hog_ab.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02au
mkdir -p $O
timeout -k 10 300 python3 -u scripts/hog_ab.py --rounds 7 > $O/hog_ab.log 2>&1; r=$?
tail -c 1500 $O/hog_ab.log; exit $r
