#!/bin/bash
# parity suite + smoke + every bench config (C2 default line, C3, C5, CRC timing)
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 900 python -m pytest tests -m gpu -q > gpurun_out/pytest_gpu.log 2>&1; r=$?
echo "pytest rc=$r"; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -5; ok $r || exit $r
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; r=$?
echo "smoke rc=$r"; tail -1 gpurun_out/smoke.log; ok $r || exit $r
for cfg in c2 c3 c5 crc; do
  timeout -k 10 600 python bench.py --config $cfg ${BENCH_ARGS:-} > gpurun_out/bench_$cfg.json 2> gpurun_out/bench_$cfg.err; r=$?
  echo "bench $cfg rc=$r"; cat gpurun_out/bench_$cfg.json; ok $r || { tail -5 gpurun_out/bench_$cfg.err; exit $r; }
done
