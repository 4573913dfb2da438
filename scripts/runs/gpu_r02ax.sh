#!/bin/bash
# Round-2 call AX: a lone wave with one vs two interleaved MD5 chains per lane.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ax
mkdir -p $O
timeout -k 10 200 python3 -u scripts/chain2_probe.py > $O/chain2.log 2>&1; r=$?
tail -c 1500 $O/chain2.log; exit $r
