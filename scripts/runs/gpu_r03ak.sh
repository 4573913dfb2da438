#!/bin/bash
# Round-3 call AK: MD5Update on few contexts as fed pairs (md5_update_ctx_fed)
# -- ctx / parity GPU tests, few-context update times against the previous
# library, the ctx bench line and its PMC bytes (the loader kernel's code
# changed with the refactor).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ak
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_ctx.py tests/test_abi.py tests/test_gpu_parity.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/ctx_small_ab.py --lib product=sproxy_amd/lib/libmd5hip.so before=build/abx/libmd5hip_ctx_old.so > $O/ctx_small_ab.json 2> $O/ctx_small_ab.err; r=$?
cat $O/ctx_small_ab.err | tail -4; [ $r -eq 0 ] || exit $r
cp profiles/traffic.json $O/traffic.json
for c in FETCH_SIZE WRITE_SIZE VALU; do
  cs=$c; [ $c = VALU ] && cs="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
  timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d $O/pmc_ctx_$c -o pmc -- python3 bench.py --config ctx --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_ctx_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 scripts/traffic_json.py $O/pmc_ctx_FETCH_SIZE $O/pmc_ctx_WRITE_SIZE ctx@1048576x16384 --valu $O/pmc_ctx_VALU --out $O/traffic.json --source "r03ak: bench.py --config ctx" > /dev/null || exit 1
cp $O/traffic.json profiles/traffic.json
timeout -k 10 300 python3 bench.py --config ctx > $O/ctx.json 2> $O/ctx.err; r=$?
python3 -c "import json;d=json.loads(open('$O/ctx.json').read().strip().splitlines()[-1]);r=d['roofline'];print('ctx', d['value'], r['frac'], r['traffic'], d['parity']['ok'])"
exit $r
