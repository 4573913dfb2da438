#!/bin/bash
# Round-3 call J: DRAM-locality probes of the C2 body (scripts/diag/locality_probe.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python3 -u scripts/diag/locality_probe.py --rounds 3 > $O/locality.json 2> $O/locality.err; r=$?
echo "rc=$r"; tail -2 $O/locality.err; cat $O/locality.json
exit $r
