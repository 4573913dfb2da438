#!/bin/bash
# first GPU pass: parity tests, then a bench line per kernel variant
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -5 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
for v in direct2 direct4 lds64 lds128; do
  timeout -k 10 240 python bench.py --steps 10 --warmup 2 --variant $v --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err
  r=$?; echo "bench $v rc=$r"; cat gpurun_out/bench_$v.json
  if [ $r -ne 0 ]; then tail -5 gpurun_out/bench_$v.err; exit $r; fi
done
