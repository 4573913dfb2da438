#!/bin/bash
# Round-2 call AP: the re-created container's rebuilt tree -- GPU suite, smoke, C2 line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ap
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; r=$?
tail -1 $O/smoke.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py > $O/c2.json 2> $O/c2.err; r=$?
cut -c1-400 $O/c2.json; exit $r
