#!/bin/bash
# Round-2 call I: BALANCED memory side -- loads-only ceilings and wide stages
# (scripts/c3_wide_ab.py) on 3 and 5 coalesced C3 batches.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02i
mkdir -p $O
timeout -k 10 300 python3 -u scripts/c3_wide_ab.py --batches 3 5 --rounds 3 > $O/wide.json 2> $O/wide.err; r=$?
echo "wide rc=$r"
cat $O/wide.json | cut -c1-1500
exit $r
