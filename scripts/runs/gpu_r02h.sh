#!/bin/bash
# Round-2 call H: PMC of the descriptor kernels on 5 coalesced C3 batches --
# clock (GRBM_GUI_ACTIVE), VALU busy, waits -- BALANCED vs XDMA, and the C2
# product for reference.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02h
mkdir -p $O
G="GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY"
for v in balanced xdma; do
  timeout -s KILL 240 rocprofv3 --pmc $G --output-format csv -d $O/pmc_$v -o pmc -- python3 scripts/c3_balanced_pmc.py 5 $v 3 > $O/pmc_$v.log 2>&1; r=$?
  echo "pmc $v rc=$r"; [ $r -eq 0 ] || exit $r
  python3 scripts/pmc_summary.py $O/pmc_$v > $O/pmc_${v}_summary.json
done
timeout -s KILL 240 rocprofv3 --pmc $G --output-format csv -d $O/pmc_c2 -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_c2.log 2>&1 || exit 1
python3 scripts/pmc_summary.py $O/pmc_c2 > $O/pmc_c2_summary.json
timeout -k 10 300 python bench.py --config c3q --c3q-inflight 1 --steps 5 --warmup 2 > $O/c3q_f1.json 2> $O/c3q_f1.err; r=$?
cut -c1-330 $O/c3q_f1.json
exit $r
