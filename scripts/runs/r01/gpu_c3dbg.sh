#!/bin/bash
# C3 hybrid: bench vs A/B script, with per-dispatch kernel traces
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/dbg
export TMPDIR=/tmp
timeout -k 10 600 python -u scripts/desc_xdma_ab.py --hybrid --c3-only --bench-batch --solo > gpurun_out/dbg/ab.json 2> gpurun_out/dbg/ab.err || exit 1
cat gpurun_out/dbg/ab.json
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/dbg/prof -o c3 -- python3 bench.py --config c3 --c3-variant hybrid --steps 20 --warmup 5 > gpurun_out/dbg/bench.json 2> gpurun_out/dbg/bench.err || exit 1
cut -c1-300 gpurun_out/dbg/bench.json
find gpurun_out/dbg/prof -name "*kernel_trace.csv" | head -3
