#!/bin/bash
# Round-2 call B: the batcher rewrite (coalescing queue, out-of-order tickets,
# device-resident submissions) against the whole GPU suite, then the
# batcher-driven C3 stream at inflight targets 1/2/3.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02b
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_queue.py -x -v --timeout 120 --timeout-method thread > $O/pytest_queue.log 2>&1; r=$?
tail -12 $O/pytest_queue.log; [ $r -eq 0 ] || exit $r
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
for f in 1 2 3; do
  timeout -k 10 300 python bench.py --config c3q --c3q-inflight $f --steps 5 --warmup 2 > $O/c3q_f$f.json 2> $O/c3q_f$f.err; r=$?
  echo "c3q inflight $f rc=$r"; cut -c1-400 $O/c3q_f$f.json; [ $r -eq 0 ] || exit $r
done
exit 0
