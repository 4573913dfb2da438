#!/bin/bash
# Round evidence in one call: full GPU parity suite, smoke, every bench config,
# rocprofv3 kernel trace of the default bench command, PMC passes (HBM bytes,
# VALU busy; scripts/gpu_pmc_traffic.sh).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/ev
export TMPDIR=/tmp
O=gpurun_out/ev
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed|FAILED" $O/pytest_gpu.log | tail -5; ok $r || exit $r
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; r=$?
echo "smoke rc=$r"; tail -1 $O/smoke.log; ok $r || exit $r
for cfg in c2 c3 c5 crc; do
  timeout -k 10 600 python bench.py --config $cfg > $O/bench_$cfg.json 2> $O/bench_$cfg.err; r=$?
  echo "bench $cfg rc=$r"; cut -c1-400 $O/bench_$cfg.json; ok $r || { tail -5 $O/bench_$cfg.err; exit $r; }
done
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_bench -o bench -- python3 bench.py --no-cpu-baseline > $O/prof_bench.log 2>&1; r=$?
echo "rocprof bench rc=$r"; tail -1 $O/prof_bench.log; ok $r || exit $r
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_crc -o crc -- python3 bench.py --config crc --no-cpu-baseline > $O/prof_crc.log 2>&1; r=$?
echo "rocprof crc rc=$r"; ok $r || exit $r
bash scripts/gpu_pmc_traffic.sh $O/pmc > $O/pmc.log 2>&1; r=$?
echo "pmc rc=$r"; tail -3 $O/pmc.log
find $O -name "*stats*.csv" | head
