#!/bin/bash
# Round-2 call AH: CRC tests on the refactored fastcrc kernel, its PMC bytes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02ah
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_crc32.py tests/test_nc_digest.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --config crc --fastcrc 128 > $O/crc128.json 2> $O/crc128.err || exit 1
cut -c1-250 $O/crc128.json
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_crc128_$c -o pmc -- python3 bench.py --config crc --fastcrc 128 --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_crc128_$c.log 2>&1 || exit 1
done
python3 scripts/traffic_json.py $O/pmc_crc128_FETCH_SIZE $O/pmc_crc128_WRITE_SIZE crc@1048576x16384f128 --out $O/traffic.json --source "r02ah: bench.py --config crc --fastcrc 128" && cat $O/traffic.json
