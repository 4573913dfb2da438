#!/bin/bash
# Round-3 call AL: final evidence after the fed MD5Update on few contexts --
# full GPU suite, smoke, the synchronous MD5 / CRC calls, every bench line,
# the gloo N=2 line and rocprof stats of the driver's command (PMC bytes of
# every bench kernel are current: code hashes match profiles/traffic.json).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03al
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; r=$?
tail -1 $O/smoke.log; [ $r -eq 0 ] || exit $r
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
