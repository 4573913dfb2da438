#!/bin/bash
# Planner-chosen HYBRID descriptor kernel: full GPU suite, sweep A/B, C3 bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_all.log 2>&1; r=$?
tail -1 gpurun_out/pytest_all.log; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u scripts/desc_xdma_ab.py --hybrid > gpurun_out/hyb_ab.json 2> gpurun_out/hyb_ab.err; r=$?
cat gpurun_out/hyb_ab.json; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u bench.py --config c3 > gpurun_out/c3.json 2> gpurun_out/c3.err; r=$?
cat gpurun_out/c3.json; exit $r
