#!/bin/bash
# Round-2 call BB: descriptor LDS-DMA loader with the uniform-offset fast path and a
# once-cast LDS image pointer (NEW) vs the previous library (OLD), in one process;
# then the GPU suite on NEW.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bb
mkdir -p $O
timeout -k 10 400 python3 -u scripts/lib_ab.py --rounds 9 > $O/lib_ab.log 2>&1; r=$?
tail -c 1800 $O/lib_ab.log; [ $r -eq 0 ] || exit $r
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; exit $r
