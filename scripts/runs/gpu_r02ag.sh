#!/bin/bash
# Round-2 call AG: fastcrc window groups in flight per wave (A/B).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ag
mkdir -p $O
timeout -k 10 300 python3 -u scripts/fastcrc_ab.py --rounds 5 > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; tail -1 $O/ab.json | cut -c1-2500; exit $r
