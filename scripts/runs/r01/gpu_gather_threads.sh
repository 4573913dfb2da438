#!/bin/bash
# Host gather threads A/B (MD5HIP_GATHER_THREADS, read once per process):
# batcher parity tests, then page-list end-to-end rates and the header scan.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gt
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "batcher or pool or zero_copy or c_site or headers or submit" > gpurun_out/gt/pytest.log 2>&1; r=$?
echo "pytest rc=$r"; tail -2 gpurun_out/gt/pytest.log; [ $r -eq 0 ] || exit $r
for T in 1 4 8; do
  for P in 16 1; do
    MD5HIP_GATHER_THREADS=$T timeout -k 10 300 python -u scripts/c5_iov.py --pages $P > gpurun_out/gt/iov_t${T}_p${P}.json 2> gpurun_out/gt/iov_t${T}_p${P}.err; r=$?
    echo "iov T=$T pages=$P rc=$r: $(cut -c1-600 gpurun_out/gt/iov_t${T}_p${P}.json)"; [ $r -eq 0 ] || exit $r
  done
  MD5HIP_GATHER_THREADS=$T timeout -k 10 300 python -u scripts/header_scan.py --n 100000 > gpurun_out/gt/hdr_t${T}.json 2> gpurun_out/gt/hdr_t${T}.err; r=$?
  echo "hdr T=$T rc=$r: $(python3 -c "import json;d=json.load(open('gpurun_out/gt/hdr_t${T}.json'));print(d['gpu'], d['cpu_baseline_all_cores']['gib_s'])")"; [ $r -eq 0 ] || exit $r
done
