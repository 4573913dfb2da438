#!/bin/bash
# C3 bench line per descriptor variant / hybrid nlong, same box, two passes
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
for pass in 1 2; do
for cfg in "1 0" "2 0" "3 256" "3 512" "3 4294967295"; do
set -- $cfg
MD5HIP_DESC_VARIANT=$1 MD5HIP_DESC_NLONG=$2 timeout -k 10 300 python bench.py --config c3 --steps 10 > gpurun_out/c3ab.json 2> gpurun_out/c3ab.err; r=$?
echo "pass $pass v$1 nlong $2 rc=$r $(python -c "import json;d=json.load(open('gpurun_out/c3ab.json'));print(d['ms_per_step'], d['value'])")"; [ $r -eq 0 ] || exit $r
done; done
