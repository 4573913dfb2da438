#!/bin/bash
# Round-2 call AC: queue probe -- launch count after every submit / wait.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ac
mkdir -p $O
timeout -k 10 300 python3 -u scripts/queue_probe.py > $O/probe.json 2> $O/probe.err; r=$?
echo "probe rc=$r"; python3 -c "
import json;d=json.load(open('$O/probe.json'))
print(d['stats'])
for x in d['log']: print(x)"
exit $r
