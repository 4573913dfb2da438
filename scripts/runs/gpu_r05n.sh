#!/bin/bash
# Round-5 call N: PMC HBM bytes and VALU busy for the crcq line at its default
# (8 submissions of 1 M blocks per step), three separate --pmc passes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE VALU; do
  cs=$c
  [ $c = VALU ] && cs="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
  timeout -s KILL 240 rocprofv3 --pmc $cs --output-format csv -d $O/crcq8_$c -o pmc -- python3 bench.py --config crcq --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/crcq8_$c.log 2>&1
  r=$?; echo "crcq8 pmc $c rc $r"; [ $r = 0 ] || exit 1
done
echo done
