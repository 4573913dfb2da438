#!/bin/bash
# Round-3 call AI: final evidence after the fastcrc-window split and the cached CU count -- full
# GPU suite, smoke, PMC bytes of the CRC lines (their code changed), small
# CRC batches and the CRC call, then every bench line and rocprof stats of
# the driver's command.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ai
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; r=$?
tail -1 $O/smoke.log; [ $r -eq 0 ] || exit $r
cp profiles/traffic.json $O/traffic.json
pmc() {  # name workload bench-args...
  local name=$1 wl=$2; shift 2
  for c in FETCH_SIZE WRITE_SIZE VALU; do
    local cs=$c
    [ $c = VALU ] && cs="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
    timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d $O/pmc_${name}_$c -o pmc -- python3 bench.py "$@" --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_${name}_$c.log 2>&1 || { echo "pmc $name $c failed"; return 1; }
  done
  python3 scripts/traffic_json.py $O/pmc_${name}_FETCH_SIZE $O/pmc_${name}_WRITE_SIZE $wl --valu $O/pmc_${name}_VALU --out $O/traffic.json --source "r03ai: bench.py $*" > /dev/null || return 1
  echo "pmc $name ok"
}
pmc crc0 crc@1048576x16384f0 --config crc && pmc crc128 crc@1048576x16384f128 --config crc --fastcrc 128 || exit 1
cp $O/traffic.json profiles/traffic.json
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --crc --sizes 16,64,256,1024,4096,16384 > $O/crc_small_16k.json 2> $O/crc_small_16k.err; r=$?
tail -3 $O/crc_small_16k.err | cut -c1-300; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --crc --iters 300 > $O/crc_latency.json 2> $O/crc_latency.err; r=$?
tail -c 600 $O/crc_latency.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/latency_probe.py --iters 300 > $O/queue_latency.json 2> $O/queue_latency.err; r=$?
tail -c 600 $O/queue_latency.json; [ $r -eq 0 ] || exit $r
line() {  # name args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "$name failed"; return 1; }
  python3 -c "import json;d=json.loads(open('$O/$name.json').read().strip().splitlines()[-1]);r=d.get('roofline',{});print('$name', d['value'], d['unit'], d.get('ms_per_step'), 'frac', r.get('frac'), 'traffic', r.get('traffic'), 'parity', (d.get('parity') or {}).get('ok'))"
}
line c2_driver --gpus 1 --steps 20 --warmup 5 && line c2 && line c3 --config c3 && line c3q --config c3q --steps 10 && \
line ctx --config ctx && line crc0 --config crc && line crc128 --config crc --fastcrc 128 && line c5 --config c5 || exit 1
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 5 > $O/n2_gloo.json 2> $O/n2_gloo.err; r=$?
echo "n2 rc=$r"; [ $r -eq 0 ] || exit $r
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2 -o c2 -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/prof_c2.log 2>&1; r=$?
echo "prof rc=$r"
exit $r
