#!/bin/bash
# Round-2 call T: evidence on the current tree -- full GPU suite, smoke,
# default bench line + rocprof stats, PMC bytes for ctx / fastcrc.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02t
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; r=$?
tail -2 $O/smoke.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py > $O/c2.json 2> $O/c2.err; r=$?
echo "c2 rc=$r"; [ $r -eq 0 ] || exit $r
cut -c1-300 $O/c2.json
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --no-cpu-baseline > $O/prof_c2.log 2>&1; r=$?
echo "prof c2 rc=$r"; [ $r -eq 0 ] || exit $r
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_ctx_$c -o pmc -- python3 bench.py --config ctx --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_ctx_$c.log 2>&1; r=$?
  echo "pmc ctx $c rc=$r"; [ $r -eq 0 ] || exit $r
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_crc128_$c -o pmc -- python3 bench.py --config crc --fastcrc 128 --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_crc128_$c.log 2>&1; r=$?
  echo "pmc crc128 $c rc=$r"; [ $r -eq 0 ] || exit $r
done
python3 scripts/traffic_json.py $O/pmc_ctx_FETCH_SIZE $O/pmc_ctx_WRITE_SIZE ctx@1048576x16384 --out $O/traffic.json --source "r02t: bench.py --config ctx" && \
python3 scripts/traffic_json.py $O/pmc_crc128_FETCH_SIZE $O/pmc_crc128_WRITE_SIZE crc@1048576x16384f128 --out $O/traffic.json --source "r02t: bench.py --config crc --fastcrc 128" && cat $O/traffic.json
