#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_check.py 52 53 > gpurun_out/diag_check.log 2>&1; r=$?
echo "diag_check rc=$r"; grep -c ": ok" gpurun_out/diag_check.log; grep MISMATCH gpurun_out/diag_check.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u scripts/profile_kernels.py --rounds 10 --reps 10 --only xpose1nt,xpose2nt,dyn5,dyn4 > gpurun_out/dyn_ab.json 2> gpurun_out/dyn_ab.err; r=$?
echo "ab rc=$r"; cat gpurun_out/dyn_ab.json
