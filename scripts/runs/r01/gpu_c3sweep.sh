#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u scripts/c3_sweep.py > gpurun_out/c3_sweep.json 2> gpurun_out/c3_sweep.err; r=$?
echo "sweep rc=$r"; cat gpurun_out/c3_sweep.err | grep -v amdgpu.ids | tail -30; exit $r
