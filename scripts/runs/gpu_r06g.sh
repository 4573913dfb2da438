#!/bin/bash
# Round-6 call G: evidence for the tree with the stable device order -- the
# whole GPU suite and smoke(), the driver's bench command under rocprofv3
# --kernel-trace --stats and plain, the PMC bytes of c3q's launches in the
# new order, and the c3 / ctx / crc lines once for the record.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06g
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc = 0 ] || { echo "smoke failed $rc"; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err
rc=$?; [ $rc = 0 ] || { echo "bench failed $rc"; tail -5 $O/c2_driver.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c2_driver.json').read().strip().splitlines()[-1]);print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['checked'], d['board'].get('gfxclk_mhz_median'), d['board'].get('ppt_limited_frac'), 'c3q', d['c3q']['value'], d['c3q']['roofline']['frac'], d['c3q']['parity']['ok'], 'c5', d['c5']['value'], d['c5']['roofline']['frac'], d['c5']['parity']['ok'])"
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1
rc=$?; echo "rocprof rc $rc"; [ $rc = 0 ] || exit 1
bash scripts/gpu_pmc_traffic.sh $O/pmc c3q > $O/pmc.log 2>&1; echo "pmc rc $?"; tail -2 $O/pmc.log
for cfg in c3 ctx crc; do
  timeout -k 10 400 python3 bench.py --config $cfg --no-cpu-baseline > $O/$cfg.json 2> $O/$cfg.err || { echo "$cfg failed"; tail -3 $O/$cfg.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/$cfg.json').read().strip().splitlines()[-1]);print('$cfg', d['value'], d['roofline']['frac'], (d.get('parity') or {}).get('ok'), (d.get('coalesced') or {}).get('roofline', {}).get('frac'))"
done
echo done
