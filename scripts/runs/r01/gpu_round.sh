#!/bin/bash
# Round evidence: parity suite, default bench line (+cpu baseline), rocprofv3
# kernel trace of the same bench command, PMC passes for HBM traffic.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3; ok $r || exit $r
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; r=$?
echo "smoke rc=$r"; tail -1 gpurun_out/smoke.log; ok $r || exit $r
timeout -k 10 600 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err; r=$?
echo "bench rc=$r"; cat gpurun_out/bench.json; ok $r || exit $r
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o bench -- python3 bench.py --no-cpu-baseline > gpurun_out/prof_bench.log 2>&1; r=$?
echo "rocprof bench rc=$r"; tail -2 gpurun_out/prof_bench.log; ok $r || exit $r
bash scripts/pmc_passes.sh gpurun_out/pmc --only ${PMC_ONLY:-xpose1nt,xpose2nt,lds128nt,xpose1,lds128,compute_only,load_xpose1} > gpurun_out/pmc.log 2>&1; r=$?
echo "pmc rc=$r"
