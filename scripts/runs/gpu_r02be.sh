#!/bin/bash
# Round-2 call BE: descriptor XDMA with two LDS-DMA images per wave on ragged batches (scripts/x2_ab.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02be
mkdir -p $O
timeout -k 10 400 python3 -u scripts/x2_ab.py --rounds 7 > $O/x2_ab.log 2>&1; r=$?
tail -c 2500 $O/x2_ab.log; exit $r
