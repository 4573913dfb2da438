#!/bin/bash
# Round-2 call C: batched MD5Update/Final contexts and the full-scale C3
# parity test; the batcher-driven C3 stream at inflight 1/2/3; the C3 line;
# PMC traffic of the C3 descriptor kernel (HYBRID).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_ctx.py tests/test_c3_full.py -x -v --timeout 400 --timeout-method thread > $O/pytest_ctx_c3.log 2>&1; r=$?
tail -8 $O/pytest_ctx_c3.log; [ $r -eq 0 ] || exit $r
for f in 1 2 3; do
  timeout -k 10 300 python bench.py --config c3q --c3q-inflight $f --steps 5 --warmup 2 > $O/c3q_f$f.json 2> $O/c3q_f$f.err; r=$?
  echo "c3q inflight $f rc=$r"; cut -c1-330 $O/c3q_f$f.json; [ $r -eq 0 ] || exit $r
done
timeout -k 10 400 python bench.py --config c3 --steps 10 --warmup 3 > $O/c3.json 2> $O/c3.err; r=$?
echo "c3 rc=$r"; cut -c1-300 $O/c3.json; [ $r -eq 0 ] || exit $r
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 bench.py --config c3 --c3-legs main --steps 3 --warmup 1 --parity-sample 0 > $O/pmc_fetch.log 2>&1; r=$?
echo "fetch rc=$r"; [ $r -eq 0 ] || exit $r
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o pmc -- python3 bench.py --config c3 --c3-legs main --steps 3 --warmup 1 --parity-sample 0 > $O/pmc_write.log 2>&1; r=$?
echo "write rc=$r"; [ $r -eq 0 ] || exit $r
python3 scripts/traffic_json.py $O/pmc_fetch $O/pmc_write c3@17179869184s1000 --source "r02c: bench.py --config c3 --c3-legs main, 4 dispatches" > $O/traffic_entry.json && cp profiles/traffic.json $O/traffic.json
cat $O/traffic_entry.json | head -30
exit 0
