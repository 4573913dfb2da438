#!/bin/bash
# Round-2 call AI: C2 energy item -- stages per LDS round trip (A/B).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ai
mkdir -p $O
timeout -k 10 400 python3 -u scripts/c2_wide_ab.py --rounds 5 --burst 10 > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; cat $O/ab.json | cut -c1-2500; exit $r
