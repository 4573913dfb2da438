#!/bin/bash
# Round-2 call E: the LPT-scheduled descriptor kernel (BALANCED): parity
# (every descriptor test parametrized over it, the queue planner test, full C3),
# per-wave traces K=1/3/5 with product timings, the C3 stream at inflight 1/2.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_queue.py tests/test_c3_full.py -k "desc or queue or c3 or balanced" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u scripts/c3_trace_x.py --batches 1 3 5 > $O/trace.json 2> $O/trace.err; r=$?
echo "trace rc=$r"; [ $r -eq 0 ] || { tail -5 $O/trace.err; exit $r; }
for f in 1 2; do
  timeout -k 10 300 python bench.py --config c3q --c3q-inflight $f --steps 5 --warmup 2 > $O/c3q_f$f.json 2> $O/c3q_f$f.err; r=$?
  echo "c3q inflight $f rc=$r"; cut -c1-330 $O/c3q_f$f.json; [ $r -eq 0 ] || exit $r
done
timeout -k 10 400 python bench.py --config c3 --steps 10 --warmup 3 > $O/c3.json 2> $O/c3.err; r=$?
cut -c1-300 $O/c3.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --config ctx --steps 20 --warmup 5 > $O/ctx.json 2> $O/ctx.err; r=$?
cut -c1-400 $O/ctx.json
exit $r
