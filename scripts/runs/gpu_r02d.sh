#!/bin/bash
# Round-2 call D: per-wave traces of single and coalesced C3 launches (xdma /
# hybrid), hybrid whole-line refill A/B, C3 PMC traffic with the new refill.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02d
mkdir -p $O
timeout -k 10 400 python -u scripts/c3_trace_x.py --batches 1 5 > $O/trace.json 2> $O/trace.err; r=$?
echo "trace rc=$r"; tail -c 3000 $O/trace.json; [ $r -eq 0 ] || { tail -5 $O/trace.err; exit $r; }
timeout -k 10 300 python -u -m pytest tests/test_c3_full.py tests/test_gpu_parity.py -k "desc or c3" -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1; r=$?
tail -2 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_c3_fetch -o pmc -- python3 bench.py --config c3 --c3-legs main --steps 3 --warmup 1 --parity-sample 0 > $O/pmc_fetch.log 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_c3_write -o pmc -- python3 bench.py --config c3 --c3-legs main --steps 3 --warmup 1 --parity-sample 0 > $O/pmc_write.log 2>&1 || exit 1
python3 scripts/traffic_json.py $O/pmc_c3_fetch $O/pmc_c3_write c3@17179869184s1000 --source "r02d: bench.py --config c3 --c3-legs main, 4 dispatches" || exit 1
cp profiles/traffic.json $O/traffic.json
timeout -k 10 400 python bench.py --config c3 --steps 10 --warmup 3 > $O/c3.json 2> $O/c3.err; r=$?
cut -c1-400 $O/c3.json
exit $r
