#!/bin/bash
# descriptor-kernel parity + chunk-size sweep + C3 bench line per descriptor variant
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "desc or mixed or kat or unaligned or huge" > gpurun_out/pytest_desc.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed|FAILED|Error" gpurun_out/pytest_desc.log | tail -8; [ $r -eq 0 ] || exit $r
for v in ${DESCV:-2 3}; do
MD5HIP_DESC_VARIANT=$v timeout -k 10 500 python -u scripts/c3_sweep.py --big "" > gpurun_out/c3_sweep_v$v.json 2> gpurun_out/c3_sweep_v$v.err; r=$?
echo "sweep v$v rc=$r"; grep -v amdgpu.ids gpurun_out/c3_sweep_v$v.err | tail -9 | cut -c1-200; [ $r -eq 0 ] || exit $r
MD5HIP_DESC_VARIANT=$v timeout -k 10 300 python bench.py --config c3 > gpurun_out/bench_c3_v$v.json 2> gpurun_out/bench_c3_v$v.err; r=$?
echo "c3 v$v rc=$r"; cut -c1-300 gpurun_out/bench_c3_v$v.json; [ $r -eq 0 ] || exit $r
done
