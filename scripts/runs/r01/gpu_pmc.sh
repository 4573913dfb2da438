#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python scripts/valu_rate.py > gpurun_out/valu_rate.json 2> gpurun_out/valu_rate.err; r=$?
echo "valu rc=$r"; cat gpurun_out/valu_rate.json; tail -3 gpurun_out/valu_rate.err
[ $r -eq 0 ] || exit $r
bash scripts/pmc_passes.sh gpurun_out/pmc ${PROFILE_ARGS:-}
