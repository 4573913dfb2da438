#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_check.py 57 58 > gpurun_out/diag_check.log 2>&1; r=$?
echo "diag_check rc=$r"; grep -c ": ok" gpurun_out/diag_check.log; grep MISMATCH gpurun_out/diag_check.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u scripts/profile_kernels.py --rounds 8 --reps 60 --only xpose1nt,xdmant,xdma > gpurun_out/xdma_ab.json 2> gpurun_out/xdma_ab.err; r=$?
cat gpurun_out/xdma_ab.json; [ $r -eq 0 ] || exit $r
CASES=xpose1nt,diag:57,xpose1nt,diag:57 bash scripts/power_probe.sh | tail -1
