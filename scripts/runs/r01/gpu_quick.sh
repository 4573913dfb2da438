#!/bin/bash
# parity + interleaved timings of all variants and ceilings
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed|Error" gpurun_out/pytest_gpu.log | tail -8; ok $r || exit $r
timeout -k 10 300 python scripts/profile_kernels.py ${PROFILE_ARGS:-} > gpurun_out/ceilings.json 2> gpurun_out/ceilings.err; r=$?
echo "ceilings rc=$r"; python3 -c "
import json; d=json.load(open('gpurun_out/ceilings.json'))
for k,v in sorted(d['results'].items(), key=lambda kv: kv[1]['ms_median']): print('%-14s %8.4f ms  %8.1f GB/s' % (k, v['ms_median'], v['payload_GBps']))
" ; ok $r || exit $r
