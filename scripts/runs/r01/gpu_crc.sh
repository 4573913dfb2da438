#!/bin/bash
# parity suite + CRC/MD5 interleaved timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -5; ok $r || exit $r
timeout -k 10 300 python -u scripts/profile_kernels.py --rounds 8 --reps 10 --only ${ONLY:-xpose1nt,crc_shared8,crc_lane32,compute_only} > gpurun_out/crc_ab.json 2> gpurun_out/crc_ab.err; r=$?
echo "ab rc=$r"; cat gpurun_out/crc_ab.json; tail -3 gpurun_out/crc_ab.err
