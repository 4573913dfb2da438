#!/bin/bash
# Round-6 call A: the new GPU tests (C5 pinned branch, the header rule for
# header_size 0..19, the 1 MiB edge through xdma1nt, pools on distinct
# devices where the box has them), then the default bench line with its
# c3q / c5 sub-records.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06a
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_c5_pinned.py tests/test_nc_digest.py tests/test_multi_gpu.py tests/test_pool.py \
  "tests/test_gpu_parity.py::test_fixed_edge_lengths" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 300 python3 -u bench.py > $O/bench.json 2> $O/bench.err
rc=$?; [ $rc = 0 ] || { echo "bench failed $rc"; tail -5 $O/bench.err; exit 1; }
python3 - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c2", d["value"], d["roofline"]["frac"], d["parity"]["checked"], d["parity"]["ok"])
for k in ("c3q", "c5"):
    x = d.get(k, {})
    print(k, x.get("value"), x.get("roofline", {}).get("frac"), (x.get("parity") or {}).get("ok"),
          (x.get("parity") or {}).get("checked"), x.get("run_s"))
PY
# the coalesced BALANCED launch: 3 batches (makespan = one 1 MiB chain, LPT
# util 0.75) against the LPT-sized count, and the 3-batch launch's wave
# occupancy from SQ counters
for k in 3 0; do
  timeout -k 10 300 python3 -u bench.py --config c3 --c3-legs coalesced --c3-coalesce $k --steps 10 --warmup 4 \
    --no-cpu-baseline > $O/coal_k$k.json 2> $O/coal_k$k.err || { echo "coalesced k=$k failed"; tail -3 $O/coal_k$k.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/coal_k$k.json').read().strip().splitlines()[-1])['coalesced'];print('coal', d['batches'], d['value'], d['roofline']['frac'], d['lpt']['util'], d['roofline']['frac_of_lpt_ceiling'], (d['parity'] or {}).get('ok'))"
done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/coal3_pmc -o pmc -- python3 bench.py --config c3 --c3-legs coalesced --c3-coalesce 3 --steps 6 --warmup 2 --no-cpu-baseline --parity-sample 0 > $O/coal3_pmc.log 2>&1
r=$?; echo "pmc coal3 rc $r"; [ $r = 0 ] || exit 1
python3 scripts/pmc_stall.py --kernel balanced $O/coal3_pmc --out $O/coal3_occupancy.json | grep -E "wave_occupancy|SQ_ACTIVE_INST_VALU\"" || true
echo done
