#!/bin/bash
# Round-2 call G: BALANCED with split long/short queues (parity + A/B of
# 4 vs 8 waves per CU, 1 vs 2 images), the queue tests, the C3 stream.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_queue.py -k "desc or queue or balanced or zero_copy" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 600 python -u scripts/c3_trace_x.py --batches 1 3 5 > $O/trace.json 2> $O/trace.err; r=$?
echo "trace rc=$r"; [ $r -eq 0 ] || { tail -5 $O/trace.err; exit $r; }
timeout -k 10 300 python bench.py --config c3q --c3q-inflight 1 --steps 5 --warmup 2 > $O/c3q_f1.json 2> $O/c3q_f1.err; r=$?
cut -c1-330 $O/c3q_f1.json
exit $r
