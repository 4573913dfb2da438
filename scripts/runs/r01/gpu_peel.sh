#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/diag_check.py 54 > gpurun_out/diag_check.log 2>&1 || { tail -5 gpurun_out/diag_check.log; exit 1; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; r=$?; tail -2 gpurun_out/pt.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python -u scripts/profile_kernels.py --rounds 12 --reps 10 --only xpose1nt,nopeel > gpurun_out/peel_ab.json 2> gpurun_out/peel_ab.err; r=$?
cat gpurun_out/peel_ab.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/peel_pmc -o pmc -- python3 scripts/profile_kernels.py --rounds 1 --reps 1 --only xpose1nt,nopeel > gpurun_out/peel_pmc.log 2>&1; echo "pmc rc=$?"
python3 - <<'PY'
import csv, glob, collections
v = collections.defaultdict(list)
for f in glob.glob("gpurun_out/peel_pmc/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        v[r["Kernel_Name"].split("(")[0]].append(float(r["Counter_Value"]))
for k, x in v.items():
    print(k, "FETCH_SIZE KB per dispatch (mean):", sum(x) / len(x) * 1.0)
PY
