#!/bin/bash
# Round-2 call BC: descriptor loader with two M0 writes per stage and pinned row-read
# addresses (NEW) vs the uniform-offset build (MID) vs the library before both (OLD),
# in one process; then the GPU suite on NEW.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bc
mkdir -p $O
timeout -k 10 500 python3 -u scripts/lib_ab.py --rounds 9 --extra mid=build/ab/libmd5hip_mid.so > $O/lib_ab.log 2>&1; r=$?
tail -c 2500 $O/lib_ab.log; [ $r -eq 0 ] || exit $r
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; exit $r
