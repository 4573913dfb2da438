#!/bin/bash
# Round-2 call BA: fed chains as a split launch (pairs on a high-priority stream, XDMA on the caller stream).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ba
mkdir -p $O
timeout -k 10 400 python3 -u scripts/fed_ab.py --rounds 5 --batches > $O/fed_ab.log 2>&1; r=$?
tail -c 2500 $O/fed_ab.log; exit $r
