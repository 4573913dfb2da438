#!/bin/bash
# Round-3 call N: descriptor kernels on small batches (the call site's
# vector sizes): XDMA / LANE / HYBRID / BALANCED launch times.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py > $O/small_batch_ab.json 2> $O/small_batch_ab.err; r=$?
tail -8 $O/small_batch_ab.err
[ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --len 65536 --sizes 16,64,256,1024 > $O/small_batch_ab_64k.json 2> $O/small_batch_ab_64k.err; r=$?
tail -5 $O/small_batch_ab_64k.err
exit $r
