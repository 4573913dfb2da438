#!/bin/bash
# Round-2 call BD: PMC passes (HBM bytes + VALU busy) for every line on the final tree,
# installed as profiles/traffic.json in this box's copy, then the evidence steps of
# gpu_r02ay.sh (GPU suite, smoke, every bench line, 2-rank spawn, rocprof C2).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
bash scripts/gpu_pmc_traffic.sh gpurun_out/r02bd || exit 1
cp gpurun_out/r02bd/traffic.json profiles/traffic.json || exit 1
sed 's#gpurun_out/r02ay#gpurun_out/r02bd#' scripts/runs/gpu_r02ay.sh > /tmp/ev.sh && bash /tmp/ev.sh
