#!/bin/bash
# in-kernel clocks: product (48), compute only (49), load only (50)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/clock_probe.py --kinds 48,49,50 > gpurun_out/clock.json 2> gpurun_out/clock.err; r=$?
echo "clock rc=$r"; cat gpurun_out/clock.json; tail -2 gpurun_out/clock.err; exit $r
