#!/bin/bash
# 64-B-stage / occupancy experiment: parity suite, diag kernels bit-exact, interleaved timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -5; ok $r || exit $r
timeout -k 10 300 python -u scripts/diag_check.py ${KINDS:-38 39 44 45} > gpurun_out/diag_check.log 2>&1; r=$?
echo "diag_check rc=$r"; cat gpurun_out/diag_check.log | tail -25; ok $r || exit $r
timeout -k 10 300 python -u scripts/profile_kernels.py --rounds 7 --only ${ONLY:-xpose1nt,x64nt,x64,d64nt,d64,compute_only,comp32,comp24,comp20,comp16} > gpurun_out/x64_ab.json 2> gpurun_out/x64_ab.err; r=$?
echo "ab rc=$r"; cat gpurun_out/x64_ab.json; tail -3 gpurun_out/x64_ab.err
