#!/bin/bash
# PMC HBM bytes (FETCH_SIZE / WRITE_SIZE passes, one counter block per run)
# and VALU busy (SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE pass) for
# every bench line's dominant kernel on the current tree, merged into
# $O/traffic.json keyed by kernel@workload and the kernel's code hash.
# usage: gpu_pmc_traffic.sh OUTDIR [NAME...]   (NAMEs: only those lines)
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=${1:-gpurun_out/pmc_traffic}
ONLY="${*:2}"
mkdir -p $O
run() {  # name workload bench-args...
  local name=$1 wl=$2; shift 2
  [ -z "$ONLY" ] || [[ " $ONLY " == *" $name "* ]] || return 0
  for c in FETCH_SIZE WRITE_SIZE VALU; do
    local cs=$c
    [ $c = VALU ] && cs="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
    timeout -s KILL 240 rocprofv3 --pmc $cs --output-format csv -d $O/pmc_${name}_$c -o pmc -- python3 bench.py "$@" --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 --extras none --no-board-probe > $O/pmc_${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; return 1; }
  done
  python3 scripts/traffic_json.py $O/pmc_${name}_FETCH_SIZE $O/pmc_${name}_WRITE_SIZE $wl --valu $O/pmc_${name}_VALU --out $O/traffic.json --source "$(basename $O): bench.py $*" > /dev/null || return 1
  echo "pmc $name ok"
}
run c2 c2@1048576x16384 && \
run crc0 crc@1048576x16384f0 --config crc && \
run crc128 crc@1048576x16384f128 --config crc --fastcrc 128 && \
run c3 c3@17179869184s1000 --config c3 --c3-legs main && \
run c3k3 c3k3@17179869184s1000 --config c3 --c3-legs coalesced --c3-coalesce 3 && \
run c3k4 c3k4@17179869184s1000 --config c3 --c3-legs coalesced && \
run ctx ctx@1048576x16384 --config ctx && \
run c3q c3q6@17179869184 --config c3q && \
python3 - "$O/traffic.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))["entries"]
for k, v in sorted(d.items()):
    print(k, v["bytes"], v["dispatches"], v.get("valu_busy"))
PY
