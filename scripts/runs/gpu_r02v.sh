#!/bin/bash
# Round-2 call V: PMC of the product BALANCED (default policy) on 5 coalesced
# C3 batches: clock, VALU busy, waits.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02v
mkdir -p $O
G="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
timeout -s KILL 240 rocprofv3 --pmc $G --output-format csv -d $O/pmc_balanced -o pmc -- python3 scripts/c3_balanced_pmc.py 5 balanced 3 > $O/pmc_balanced.log 2>&1; r=$?
echo "pmc rc=$r"; [ $r -eq 0 ] || exit $r
python3 scripts/pmc_summary.py $O/pmc_balanced > $O/pmc_balanced_summary.json && grep -A14 '"md5_desc_balanced' $O/pmc_balanced_summary.json
