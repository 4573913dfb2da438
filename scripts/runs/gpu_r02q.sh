#!/bin/bash
# Round-2 call Q: descriptor XDMA occupancy (20 / 16 / 12 / 8 waves per CU)
# against HYBRID and BALANCED on uniform and ragged netcache batches.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02q
mkdir -p $O
timeout -k 10 400 python3 -u scripts/desc_policy_ab.py --rounds 3 --sets u16k rag16 rag128 c3 --kinds 0 5 6 7 1 --products xdma hybrid balanced > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/ab.json | cut -c1-4000
