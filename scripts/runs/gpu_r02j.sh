#!/bin/bash
# Round-2 call J: BALANCED with 512-B wide stages as the product -- its tests,
# the A/B on 1/3/5 coalesced C3 batches, the queue-driven C3 line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02j
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_queue.py tests/test_abi.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/c3_wide_ab.py --batches 1 3 5 --rounds 3 --kinds 0 6 10 14 15 > $O/wide.json 2> $O/wide.err; r=$?
echo "wide rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/wide.json | cut -c1-3000
for f in 1 2; do
  timeout -k 10 300 python bench.py --config c3q --c3q-inflight $f --steps 5 --warmup 2 > $O/c3q_f$f.json 2> $O/c3q_f$f.err; r=$?
  echo "c3q f$f rc=$r"; [ $r -eq 0 ] || exit $r
  cut -c1-330 $O/c3q_f$f.json
done
