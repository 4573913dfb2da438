#!/bin/bash
# Round-3 call H: the batcher without an order for already-sorted slots and
# with a 1 us timer slack on its progress thread -- GPU suite, then the same
# per-call breakdowns as call G.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03h
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
for mode in host device; do
  for nb in 64 1024; do
    timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_${mode}_${nb} -o t -- python3 scripts/call_breakdown.py --mode $mode --nb $nb --calls 200 --out $O/stamps_${mode}_${nb}.json > $O/run_${mode}_${nb}.log 2>&1; r=$?
    echo "$mode $nb rc=$r"; tail -1 $O/run_${mode}_${nb}.log; [ $r -eq 0 ] || exit $r
    python3 scripts/call_breakdown.py --join $O/tr_${mode}_${nb} --stamps $O/stamps_${mode}_${nb}.json > $O/breakdown_${mode}_${nb}.json 2>&1
  done
done
for mode in host device; do for nb in 64 1024; do timeout -k 10 120 python3 scripts/call_breakdown.py --mode $mode --nb $nb --calls 300 --out $O/plain_${mode}_${nb}.json; done; done
timeout -k 10 300 python3 -u scripts/latency_probe.py --iters 200 > $O/queue_latency.json 2> $O/queue_latency.err; echo "latency rc=$?"; tail -1 $O/queue_latency.json | cut -c1-600
exit 0
