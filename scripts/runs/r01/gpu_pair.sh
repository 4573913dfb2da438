#!/bin/bash
# paired-refill xpose2 A/B + in-kernel clock of product vs compute-only
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 300 python -u scripts/diag_check.py ${KINDS:-46 47 48} > gpurun_out/diag_check.log 2>&1; r=$?
echo "diag_check rc=$r"; grep -c ok gpurun_out/diag_check.log; grep MISMATCH gpurun_out/diag_check.log; ok $r || exit $r
timeout -k 10 300 python -u scripts/clock_probe.py > gpurun_out/clock.json 2> gpurun_out/clock.err; r=$?
echo "clock rc=$r"; cat gpurun_out/clock.json; ok $r || exit $r
timeout -k 10 400 python -u scripts/profile_kernels.py --rounds 8 --reps 10 --only ${ONLY:-xpose1nt,xpose2nt,x2pairnt,x2pair,compute_only,load_xpose1} > gpurun_out/pair_ab.json 2> gpurun_out/pair_ab.err; r=$?
echo "ab rc=$r"; cat gpurun_out/pair_ab.json; tail -3 gpurun_out/pair_ab.err
