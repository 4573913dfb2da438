#!/bin/bash
# rocprofv3 PMC passes over scripts/profile_kernels.py (one counter group per
# pass, --kernel-trace/--stats never combined with --pmc: gpurun refuses that).
# usage: scripts/pmc_passes.sh OUTDIR [profile_kernels.py args...]
cd "$GRAFT_REPO_ROOT" || exit 1
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
i=0
for grp in \
  "FETCH_SIZE" \
  "WRITE_SIZE" \
  "GRBM_GUI_ACTIVE SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY" \
  "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_BUSY_CU_CYCLES" \
  "TA_TA_BUSY_sum TA_BUSY_avr TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out/p$i" -o pmc -- python3 scripts/profile_kernels.py --rounds 1 --reps 1 "$@" > "$out/p$i.log" 2>&1
  r=$?; echo "pass $i ($grp) rc=$r"
  if [ $r -ne 0 ] && [ $r -ne 1 ]; then tail -5 "$out/p$i.log"; [ $r -ge 124 ] && exit $r; fi
done
python3 scripts/pmc_summary.py "$out" > "$out/summary.json" && cat "$out/summary.json"
