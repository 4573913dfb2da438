#!/bin/bash
# Round-2 call AW: BALANCED with three images and register-pipelined stages (diag kind 26)
# vs the product shape (kind 19) and the product launch, coalesced C3 (3 and 5 batches).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02aw
mkdir -p $O
timeout -k 10 400 python3 -u scripts/c3_wide_ab.py --batches 3 5 --rounds 5 --kinds 19 26 > $O/ab.log 2>&1; r=$?
tail -c 2000 $O/ab.log; exit $r
