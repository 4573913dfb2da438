#!/bin/bash
# Round-2 call K: C3 lines on the wide-stage BALANCED product (single batch,
# coalesced, queue stream pipelined + drained) and PMC HBM bytes for the
# coalesced BALANCED launch and the single-batch HYBRID launch.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02k
mkdir -p $O
timeout -k 10 300 python bench.py --config c3 > $O/c3.json 2> $O/c3.err; r=$?
echo "c3 rc=$r"; [ $r -eq 0 ] || exit $r
cut -c1-400 $O/c3.json
for f in 1 2; do
  timeout -k 10 300 python bench.py --config c3q --c3q-inflight $f --steps 5 --warmup 2 > $O/c3q_f$f.json 2> $O/c3q_f$f.err; r=$?
  echo "c3q f$f rc=$r"; [ $r -eq 0 ] || exit $r
  cut -c1-330 $O/c3q_f$f.json
done
for leg in coalesced main; do
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_${leg}_$c -o pmc -- python3 bench.py --config c3 --c3-legs $leg --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_${leg}_$c.log 2>&1; r=$?
    echo "pmc $leg $c rc=$r"; [ $r -eq 0 ] || exit $r
  done
done
python3 scripts/traffic_json.py $O/pmc_coalesced_FETCH_SIZE $O/pmc_coalesced_WRITE_SIZE c3k3@17179869184s1000 --out $O/traffic.json --source "r02k: bench.py --config c3 --c3-legs coalesced" && \
python3 scripts/traffic_json.py $O/pmc_main_FETCH_SIZE $O/pmc_main_WRITE_SIZE c3@17179869184s1000 --out $O/traffic.json --source "r02k: bench.py --config c3 --c3-legs main" && cat $O/traffic.json
