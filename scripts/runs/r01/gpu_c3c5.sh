#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --config c3 --steps 5 --warmup 1 > gpurun_out/c3.json 2> gpurun_out/c3.err; r=$?
echo "c3 rc=$r"; cat gpurun_out/c3.json; [ $r -eq 0 ] || { tail -5 gpurun_out/c3.err; exit $r; }
timeout -k 10 400 python bench.py --config c5 --steps 3 --warmup 1 > gpurun_out/c5.json 2> gpurun_out/c5.err; r=$?
echo "c5 rc=$r"; cat gpurun_out/c5.json; [ $r -eq 0 ] || { tail -5 gpurun_out/c5.err; exit $r; }
