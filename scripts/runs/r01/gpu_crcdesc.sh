#!/bin/bash
# CRC descriptor parity + A/B of the descriptor kernels on a ragged netcache batch
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_crc32.py tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_crcdesc.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_crcdesc.log | tail -8; [ $r -eq 0 ] || exit $r
for v in 1 5; do
CRC32HIP_VARIANT=$v timeout -k 10 300 python -u scripts/crc_desc_bench.py > gpurun_out/crcdesc_v$v.json 2>gpurun_out/crcdesc_v$v.err; r=$?
echo "crc desc v$v rc=$r"; cat gpurun_out/crcdesc_v$v.json; [ $r -eq 0 ] || exit $r
done
