#!/bin/bash
# Board power (rocm-smi, ~0.2 s samples) while C2-shape kernels run back to
# back for ~4 s each (scripts/power_ab.py); scripts/power_summary.py joins them.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
CASES=${CASES:-xpose1nt,diag:49,diag:6,diag:4,diag:5,diag:1}
( for i in $(seq 1 400); do echo "T $(date +%s.%N)"; timeout -k 2 5 rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Power|sclk"; sleep 0.1; done ) > gpurun_out/power_trace.txt 2>&1 &
BG=$!
timeout -k 10 300 python -u scripts/power_ab.py --cases "$CASES" > gpurun_out/power_ab.json 2> gpurun_out/power_ab.err; r=$?
kill $BG 2>/dev/null; wait $BG 2>/dev/null
echo "power_ab rc=$r"; cat gpurun_out/power_ab.json; tail -2 gpurun_out/power_ab.err
python scripts/power_summary.py gpurun_out/power_ab.json gpurun_out/power_trace.txt; exit $r
