#!/bin/bash
# Round-2 call W: BALANCED with long groups lane-direct (diag 24/25) vs product.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02w
mkdir -p $O
timeout -k 10 400 python3 -u scripts/c3_wide_ab.py --batches 1 2 3 5 --rounds 3 --kinds 24 25 > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/ab.json | cut -c1-3500
