#!/bin/bash
# Round-3 call AH: the single C3 batch with its 1 MiB groups as fed pairs on
# CUs of their own and the rest as HYBRID (its own longest groups
# lane-direct) instead of XDMA (fed_ab.py leg fed_excl_rest_hybrid).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
timeout -k 10 400 python3 -u scripts/diag/fed_ab.py --rounds 7 --batches > $O/fed_ab.json 2> $O/fed_ab.err; r=$?
tail -c 2500 $O/fed_ab.json; tail -3 $O/fed_ab.err
exit $r
