#!/bin/bash
# Round-3 call G: the C call-site program with four threads on one pool, and
# where a synchronous call's time goes (kernel + memory-copy trace joined with
# per-call host stamps) for host-page and device-resident vectors.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 200 python3 -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_c_site.py -m gpu > $O/pytest_c_site.log 2>&1; r=$?
tail -3 $O/pytest_c_site.log; [ $r -eq 0 ] || exit $r
for mode in host device; do
  for nb in 64 1024; do
    timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_${mode}_${nb} -o t -- python3 scripts/call_breakdown.py --mode $mode --nb $nb --calls 200 --out $O/stamps_${mode}_${nb}.json > $O/run_${mode}_${nb}.log 2>&1; r=$?
    echo "$mode $nb rc=$r"; tail -1 $O/run_${mode}_${nb}.log; [ $r -eq 0 ] || exit $r
    python3 scripts/call_breakdown.py --join $O/tr_${mode}_${nb} --stamps $O/stamps_${mode}_${nb}.json > $O/breakdown_${mode}_${nb}.json 2>&1
    head -c 1500 $O/breakdown_${mode}_${nb}.json; echo
  done
done
exit 0
