#!/bin/bash
# Round-2 call AZ: PMC passes (HBM bytes + VALU busy) for every bench line's kernel -> traffic.json.
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_pmc_traffic.sh gpurun_out/r02az
