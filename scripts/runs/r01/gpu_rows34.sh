#!/bin/bash
# §8f rows 3/4 measured on the box: header-scan verify (GPU vs CPU), nc_MD5 host speed.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/r34
export TMPDIR=/tmp
timeout -k 10 400 python -u scripts/header_scan.py --n 100000 > gpurun_out/r34/header_scan.json 2> gpurun_out/r34/header_scan.err; r=$?
echo "header_scan rc=$r"; cat gpurun_out/r34/header_scan.json; [ $r -eq 0 ] || { tail -5 gpurun_out/r34/header_scan.err; exit $r; }
timeout -k 10 300 bash scripts/nc_md5_speed.sh > gpurun_out/r34/nc_md5_speed.txt 2>&1; r=$?
echo "nc_md5_speed rc=$r"; cat gpurun_out/r34/nc_md5_speed.txt; exit $r
