#!/bin/bash
# Round-5 call Q: the whole GPU suite on the final tree, and smoke.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05q
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; grep -E "FAIL|Error" $O/pytest.log | head -5; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -3 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
echo done
