#!/bin/bash
# round-3 xad pair form (kX3): parity, interleaved A/B, board power
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_check.py 55 > gpurun_out/diag_check.log 2>&1; r=$?
echo "diag_check rc=$r"; grep -c ": ok" gpurun_out/diag_check.log; grep MISMATCH gpurun_out/diag_check.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u scripts/profile_kernels.py --rounds 12 --reps 10 --only xpose1nt,x3,compute_only,comp_x3 > gpurun_out/x3_ab.json 2> gpurun_out/x3_ab.err; r=$?
cat gpurun_out/x3_ab.json; [ $r -eq 0 ] || exit $r
CASES=xpose1nt,diag:55,diag:0,diag:56,xpose1nt,diag:55 bash scripts/power_probe.sh | tail -1
