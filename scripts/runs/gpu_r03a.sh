#!/bin/bash
# Round-3 call A: why the first ~15 C2 launches are slow.
# Per-launch in-kernel shader clock of the product body in bench.py's exact
# sequence and variants (scripts/startup_probe.py), a kernel trace of the
# driver's own command, board telemetry sampled alongside.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
( for i in $(seq 1 300); do echo "T $(date +%s.%N)"; timeout -k 2 5 rocm-smi --showpower --showclocks 2>/dev/null | grep -E "Power|sclk|mclk|fclk"; sleep 0.05; done ) > $O/smi_trace.txt 2>&1 &
SMI=$!
for mode in bench arena gap prefill compute loads repeat; do
  timeout -k 10 120 python3 -u scripts/startup_probe.py --mode $mode > $O/probe_$mode.json 2> $O/probe_$mode.err; r=$?
  echo "$mode rc=$r"; [ $r -eq 0 ] || { kill $SMI; exit $r; }
done
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o n1 -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_trace.log 2>&1; r=$?
echo "trace rc=$r"
kill $SMI 2>/dev/null
exit $r
