#!/bin/bash
# Round-2 call Y: PMC HBM bytes of every line's kernel on the current tree.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_pmc_traffic.sh gpurun_out/r02y
