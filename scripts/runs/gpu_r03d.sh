#!/bin/bash
# Round-3 call D: pool tests (1 MiB-block vectors for the coalescing check),
# the whole GPU suite, the pool's call-site probe, the PMC counter list.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/pool_latency_probe.py --iters 100 --threads 8 --secs 2 > $O/pool_latency.json 2> $O/pool_latency.err; r=$?
echo "pool probe rc=$r"; tail -2 $O/pool_latency.err; [ $r -eq 0 ] || exit $r
timeout -k 5 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"
grep -E "TCC_EA0_RD|TCC_EA_RD|TCC_BUBBLE|TCC_REQ|TCC_READ" $O/counters.txt | head -40
exit 0
