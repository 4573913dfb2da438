#!/bin/bash
# Round-2 call N: BALANCED product on the default cache policy -- tests,
# A/B against the earlier shapes, C3 / C3-queue lines, PMC bytes.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02n
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_queue.py tests/test_abi.py tests/test_c3_full.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/c3_wide_ab.py --batches 3 5 --rounds 3 --kinds 0 6 19 > $O/wide.json 2> $O/wide.err; r=$?
echo "wide rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/wide.json | cut -c1-2000
timeout -k 10 300 python bench.py --config c3 > $O/c3.json 2> $O/c3.err; r=$?
echo "c3 rc=$r"; [ $r -eq 0 ] || exit $r
python3 -c "import json;d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]);print(d['value'], d['coalesced'])"
for f in 1 2; do
  timeout -k 10 300 python bench.py --config c3q --c3q-inflight $f --steps 5 --warmup 2 > $O/c3q_f$f.json 2> $O/c3q_f$f.err; r=$?
  echo "c3q f$f rc=$r"; [ $r -eq 0 ] || exit $r
  python3 -c "import json;d=json.loads(open('$O/c3q_f$f.json').read().strip().splitlines()[-1]);print(d['value'], d['tb_s'], d['drained'], d['parity'] if 'parity' in d else d.get('ranks_seen',{}).get('ranks',[{}])[0].get('parity'))"
done
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/pmc_coalesced_$c -o pmc -- python3 bench.py --config c3 --c3-legs coalesced --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_coalesced_$c.log 2>&1; r=$?
  echo "pmc $c rc=$r"; [ $r -eq 0 ] || exit $r
done
python3 scripts/traffic_json.py $O/pmc_coalesced_FETCH_SIZE $O/pmc_coalesced_WRITE_SIZE c3k3@17179869184s1000 --out $O/traffic.json --source "r02n: bench.py --config c3 --c3-legs coalesced" && cat $O/traffic.json
