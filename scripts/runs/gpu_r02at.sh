#!/bin/bash
# Round-2 call AT: fed chains A/B -- 4-wave workgroups (a pair + two XDMA waves) vs 2-wave.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02at
mkdir -p $O
timeout -k 10 400 python3 -u scripts/fed_ab.py --rounds 5 --batches > $O/fed_ab.log 2>&1; r=$?
tail -c 2500 $O/fed_ab.log; exit $r
