#!/bin/bash
# Round-2 call AK: board power and clock while the product C2 and CRC kernels
# (and the compute-only probe) run back to back.
cd "$GRAFT_REPO_ROOT" || exit 1
CASES=xdma1nt,crc:xdma16,diag:49 timeout -k 10 200 bash scripts/power_probe.sh
