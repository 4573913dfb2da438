#!/bin/bash
# CRC variant parity + interleaved timings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 600 python -u -m pytest tests/test_crc32.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_crc.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_crc.log | tail -5; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u scripts/profile_kernels.py --rounds 8 --reps 10 --only ${ONLY:-xpose1nt,crc_shared8,crc_xlane16,crc_lane16} > gpurun_out/crc_ab.json 2> gpurun_out/crc_ab.err; r=$?
echo "ab rc=$r"; cat gpurun_out/crc_ab.json; tail -3 gpurun_out/crc_ab.err
