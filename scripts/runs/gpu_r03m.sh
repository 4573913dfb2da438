#!/bin/bash
# Round-3 call M: does the memory type (hipMalloc / fine-grained / uncached /
# contiguous) of the C2 batch change the product kernel's launch time?
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python3 -u scripts/diag/alloc_ab.py --rounds 2 > $O/alloc_ab.json 2> $O/alloc_ab.err; r=$?
cat $O/alloc_ab.err | tail -12
exit $r
