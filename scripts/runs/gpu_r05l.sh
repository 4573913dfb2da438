#!/bin/bash
# Round-5 call L: the evidence for the shipped tree -- every bench line at its
# defaults (C2 as the driver runs it), and the rocprofv3 kernel-trace summary
# of the driver's own command.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
line() {  # name args...
  local name=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > $O/$name.json 2> $O/$name.err || { echo "bench $name failed"; tail -3 $O/$name.err; exit 1; }
  python3 - "$O/$name.json" "$name" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d.get("roofline") or {}
print(sys.argv[2], d["value"], d["unit"], "frac", r.get("frac"), "ms", d.get("ms_per_step"), "cpu", (d.get("cpu_baseline") or {}).get("value"), flush=True)
PY
}
line c2_driver --gpus 1 --steps 20 --warmup 5
line c3 --config c3
line c3q --config c3q
line ctx --config ctx
line crc --config crc
line crc_fast128 --config crc --fastcrc 128
line crcq --config crcq
line c5 --config c5
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver -o driver -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/prof_driver.log 2>&1 || { echo "rocprof failed"; tail -3 $O/prof_driver.log; exit 1; }
tail -1 $O/prof_driver.log | cut -c1-300
find $O/prof_driver -name "*stats*.csv"
echo done
