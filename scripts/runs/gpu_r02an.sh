#!/bin/bash
# Round-2 call AN: one C3 batch (chain-bound): BALANCED with one / two images
# against HYBRID.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02an
mkdir -p $O
timeout -k 10 300 python3 -u scripts/c3_wide_ab.py --batches 1 --rounds 5 --kinds 19 20 > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; tail -1 $O/ab.json | cut -c1-1500; exit $r
