#!/bin/bash
# Round-2 call BI: PMC (HBM bytes + VALU busy) of the C4 per-rank shard (2,097,152 x 16 KiB,
# the N > 1 default) merged into this box's profiles/traffic.json copy.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bi
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE VALU; do
  cs=$c; [ $c = VALU ] && cs="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
  timeout -s KILL 240 rocprofv3 --pmc $cs --output-format csv -d $O/pmc_c4_$c -o pmc -- python3 bench.py --chunks 2097152 --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_c4_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
cp profiles/traffic.json $O/traffic.json
python3 scripts/traffic_json.py $O/pmc_c4_FETCH_SIZE $O/pmc_c4_WRITE_SIZE c2@2097152x16384 --valu $O/pmc_c4_VALU --out $O/traffic.json --source "r02bi: bench.py --chunks 2097152 (the C4 per-rank shard)"
