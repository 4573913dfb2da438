#!/bin/bash
# Round-2 call BF: PMC (HBM bytes + VALU busy) of the c3q queue's BALANCED launches, merged
# into this box's profiles/traffic.json copy, then the c3q bench line reading it.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bf
mkdir -p $O
for c in FETCH_SIZE WRITE_SIZE VALU; do
  cs=$c; [ $c = VALU ] && cs="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
  timeout -s KILL 240 rocprofv3 --pmc $cs --output-format csv -d $O/pmc_c3q_$c -o pmc -- python3 bench.py --config c3q --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_c3q_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
cp profiles/traffic.json $O/traffic.json
python3 scripts/traffic_json.py $O/pmc_c3q_FETCH_SIZE $O/pmc_c3q_WRITE_SIZE c3q6@17179869184 --valu $O/pmc_c3q_VALU --out $O/traffic.json --source "r02bf: bench.py --config c3q" || exit 1
cp $O/traffic.json profiles/traffic.json
timeout -k 10 400 python bench.py --config c3q --steps 10 > $O/c3q.json 2> $O/c3q.err; r=$?
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print(d['value'], json.dumps(d['roofline']))"
exit $r
