#!/bin/bash
# Round-2 call AQ: fed chains A/B (scripts/fed_ab.py), then the rebuilt tree's
# GPU suite, smoke and the C2 line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02aq
mkdir -p $O
timeout -k 10 400 python3 -u scripts/fed_ab.py --rounds 5 --batches 2 > $O/fed_ab.log 2>&1; r=$?
tail -c 1500 $O/fed_ab.log; [ $r -eq 0 ] || exit $r
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; r=$?
tail -1 $O/smoke.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py > $O/c2.json 2> $O/c2.err; r=$?
cut -c1-400 $O/c2.json; exit $r
