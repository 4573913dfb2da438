#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/valu_rate.py 8192 > gpurun_out/valu_rate32.json 2> gpurun_out/valu_rate.err; r=$?
echo "rc=$r"; [ $r -eq 0 ] || { tail -5 gpurun_out/valu_rate.err; exit $r; }
timeout -k 10 300 python scripts/valu_rate.py 4096 > gpurun_out/valu_rate16.json 2>> gpurun_out/valu_rate.err; r=$?
echo "rc=$r"
python3 -c "
import json
a=json.load(open('gpurun_out/valu_rate32.json')); b=json.load(open('gpurun_out/valu_rate16.json'))
for k in a: print('%-24s 32w: %5.2f cyc (%.2f GHz)   16w: %5.2f cyc' % (k, a[k]['cycles_per_wave_inst'], a[k]['clock_ghz'], b[k]['cycles_per_wave_inst']))
"
