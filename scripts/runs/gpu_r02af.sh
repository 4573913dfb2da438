#!/bin/bash
# Round-2 call AF: BALANCED double-buffered (NB2) under the default policy vs
# the product, 5 interleaved rounds on 3 and 5 coalesced C3 batches.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02af
mkdir -p $O
timeout -k 10 500 python3 -u scripts/c3_wide_ab.py --batches 3 5 --rounds 5 --kinds 19 20 > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/ab.json | cut -c1-2500
