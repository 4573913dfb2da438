#!/bin/bash
# Round-6 call B: the evidence for the round-6 tree -- the whole GPU suite
# and smoke(), the driver's bench command (C2 headline with its board probe
# and the c3q / c5 sub-records), the rocprofv3 kernel-trace summary of that
# same command, and the PMC bytes of the LPT-sized coalesced C3 launch.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06b
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
rc=$?; tail -1 $O/smoke.log; [ $rc = 0 ] || { echo "smoke failed $rc"; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err
rc=$?; [ $rc = 0 ] || { echo "bench failed $rc"; tail -5 $O/c2_driver.err; exit 1; }
python3 - $O/c2_driver.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c2", d["value"], d["ms_per_step"], d["roofline"]["frac"], d["parity"]["checked"], d["parity"]["ok"], d.get("board"))
for k in ("c3q", "c5"):
    x = d.get(k, {})
    print(k, x.get("value"), x.get("roofline", {}).get("frac"), (x.get("parity") or {}).get("ok"), x.get("run_s"))
PY
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof.log 2>&1
rc=$?; echo "rocprof rc $rc"; [ $rc = 0 ] || exit 1
find $O/prof -name "*kernel_stats.csv" | head -3
bash scripts/gpu_pmc_traffic.sh $O/pmc c3k4 > $O/pmc.log 2>&1; echo "pmc rc $?"; tail -3 $O/pmc.log
echo done
