#!/bin/bash
# Round-6 call K: the library after the sticky-error fix -- the whole GPU suite,
# smoke(), and the driver's bench command.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06k
mkdir -p $O
md5sum sproxy_amd/lib/libmd5hip.so > $O/lib.md5
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc = 0 ] || { echo "smoke failed $rc"; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err
rc=$?; [ $rc = 0 ] || { echo "bench failed $rc"; tail -5 $O/c2_driver.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c2_driver.json').read().strip().splitlines()[-1]);print('c2', d['value'], d['ms_per_step'], d['roofline']['frac'], d['parity']['checked'], d['board'].get('gfxclk_mhz_median'), 'c3q', d['c3q']['value'], d['c3q']['roofline']['frac'], d['c3q']['parity']['ok'], 'c5', d['c5']['value'], d['c5']['roofline']['frac'], d['c5']['parity']['ok'])"
echo done
