#!/bin/bash
# GPU pass 2: parity, interleaved kernel/ceiling timings, rocprofv3 trace + PMC.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }   # 1 = test/assert failure, not a fault
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; r=$?
echo "pytest rc=$r"; tail -3 gpurun_out/pytest_gpu.log; ok $r || exit $r
timeout -k 10 300 python scripts/profile_kernels.py > gpurun_out/ceilings.json 2> gpurun_out/ceilings.err; r=$?
echo "ceilings rc=$r"; cat gpurun_out/ceilings.json; ok $r || exit $r
rocprofv3 -L > gpurun_out/counters.txt 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o kt -- python3 scripts/profile_kernels.py --rounds 2 --reps 2 > gpurun_out/prof_kt.log 2>&1; r=$?
echo "kt rc=$r"; ok $r || exit $r
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof_fetch -o pmc -- python3 scripts/profile_kernels.py --rounds 1 --reps 1 > gpurun_out/prof_fetch.log 2>&1; r=$?
echo "pmc fetch rc=$r"; ok $r || exit $r
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/prof_sq -o pmc -- python3 scripts/profile_kernels.py --rounds 1 --reps 1 > gpurun_out/prof_sq.log 2>&1; r=$?
echo "pmc sq rc=$r"
exit 0
