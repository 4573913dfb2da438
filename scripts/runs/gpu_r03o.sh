#!/bin/bash
# Round-3 call O: where LANE stops beating XDMA as batches grow (16 KiB and
# 4 KiB chunks).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --sizes 4096,8192,16384,32768,65536,131072,262144 --iters 30 > $O/sweep_16k.json 2> $O/sweep_16k.err; r=$?
tail -8 $O/sweep_16k.err
[ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --len 4096 --sizes 64,1024,16384,65536,262144,1048576 --iters 30 > $O/sweep_4k.json 2> $O/sweep_4k.err; r=$?
tail -7 $O/sweep_4k.err
exit $r
