#!/bin/bash
# Round-2 first GPU call: GPU parity suite on the pruned library, the C2 line,
# bench.py's own 2-rank spawn (gloo, both ranks on the one GPU), PMC traffic
# keyed by code object, and a kernel-trace summary of the C2 bench.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02a
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py > $O/c2.json 2> $O/c2.err; r=$?
cut -c1-300 $O/c2.json; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 5 > $O/n2.json 2> $O/n2.err; r=$?
tail -c 600 $O/n2.json; [ $r -eq 0 ] || exit $r
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_fetch.log 2>&1; r=$?
echo "fetch rc=$r"; [ $r -eq 0 ] || exit $r
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_write.log 2>&1; r=$?
echo "write rc=$r"; [ $r -eq 0 ] || exit $r
python3 scripts/traffic_json.py $O/pmc_fetch $O/pmc_write c2@1048576x16384 --source "r02a: bench.py C2, 4 dispatches" > $O/traffic_entry.json && cp profiles/traffic.json $O/traffic.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/ktrace -o kt -- python3 bench.py --no-cpu-baseline --parity-sample 0 > $O/ktrace.log 2>&1; r=$?
echo "ktrace rc=$r"; tail -c 400 $O/ktrace.log
exit $r
