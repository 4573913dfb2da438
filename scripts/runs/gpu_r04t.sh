#!/bin/bash
# Round-4 call T: the final tree's evidence after the BALANCED and queue
# work.  The whole GPU suite and smoke(); the driver's exact bench command,
# plus every bench line; the driver's command under rocprofv3 (kernel
# stats).  The call-site matrices did not change since call D (r04d).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err || { echo "c2 driver failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c2_driver.json').read().strip().splitlines()[-1]);print('c2 driver', d['value'], d['ms_per_step'], d['roofline']['frac'])"
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/c2_driver_prof -o c2 -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver_prof.json 2> $O/c2_driver_prof.err || { echo "c2 rocprof failed"; exit 1; }
for cfg in c3q c3 ctx crc c5; do
  timeout -k 10 300 python3 bench.py --config $cfg --no-cpu-baseline > $O/$cfg.json 2> $O/$cfg.err || { echo "bench $cfg failed"; tail -3 $O/$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/$cfg.json').read().strip().splitlines()[-1]);print('$cfg', d['value'], d.get('ms_per_step'), d.get('roofline',{}).get('frac'), (d.get('drained') or {}).get('value'))"
done
echo done
