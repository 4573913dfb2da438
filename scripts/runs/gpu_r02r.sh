#!/bin/bash
# Round-2 call R: descriptor XDMA capped by VGPRs (even per SIMD) vs HYBRID.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02r
mkdir -p $O
timeout -k 10 400 python3 -u scripts/desc_policy_ab.py --rounds 3 --sets u16k rag16 rag128 c3 --kinds 0 8 9 10 1 --products xdma hybrid > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/ab.json | cut -c1-4000
