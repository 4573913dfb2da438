#!/bin/bash
# Round-4 call B: GPU tests of the blocked-caller rework, the null-stream
# ordering fix and the LINES loader; the call site at ASIO scale (8/64/256
# threads, pageable and registered pages) with the round-3 batcher beside
# it; XDMA vs LINES timing and HBM bytes; where a drained c3q step's time
# goes, the c3q line and its launch gaps; the chunk_size matrix.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_lines.py tests/test_pool.py tests/test_c_site.py tests/test_queue.py > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 240 python3 -u scripts/asio_scale.py --matrix threads --secs 3 --out $O/asio_threads.json > $O/asio_threads.log 2>&1 || { echo "threads matrix failed"; tail -3 $O/asio_threads.log; exit 1; }
LD_LIBRARY_PATH=$PWD/build/abr04/old timeout -k 10 240 python3 -u scripts/asio_scale.py --matrix threads --secs 3 --out $O/asio_threads_r03lib.json > $O/asio_threads_r03lib.log 2>&1 || { echo "r03 threads matrix failed"; tail -3 $O/asio_threads_r03lib.log; exit 1; }
timeout -k 10 200 python3 -u scripts/lines_ab.py > $O/lines_ab.log 2>&1 || { echo "lines_ab failed"; tail -3 $O/lines_ab.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --stats --output-format csv -d $O/pmc_lines -o pmc -- python3 scripts/lines_ab.py --rounds 2 --shapes packed16,packed128 > $O/pmc_lines.log 2>&1 || { echo "pmc lines failed"; exit 1; }
timeout -s KILL 150 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/c3q_trace -o trace -- python3 scripts/c3q_breakdown.py --steps 6 --out $O/c3q_stamps.json > $O/c3q_breakdown.log 2>&1 || { echo "c3q breakdown failed"; tail -3 $O/c3q_breakdown.log; exit 1; }
python3 scripts/c3q_breakdown.py --join $O/c3q_trace --stamps $O/c3q_stamps.json --out $O/c3q_breakdown.json >> $O/c3q_breakdown.log 2>&1
timeout -k 10 200 python3 bench.py --config c3q --steps 10 --no-cpu-baseline > $O/c3q.json 2> $O/c3q.err || { echo "c3q bench failed"; tail -3 $O/c3q.err; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/c3q_bench_trace -o trace -- python3 bench.py --config c3q --steps 10 --no-cpu-baseline > $O/c3q_traced.json 2> $O/c3q_traced.err || { echo "c3q traced failed"; exit 1; }
python3 scripts/queue_gaps.py $O/c3q_bench_trace > $O/c3q_gaps.json 2>&1
timeout -k 10 400 python3 -u scripts/asio_scale.py --matrix chunk --secs 2 --out $O/asio_chunk.json > $O/asio_chunk.log 2>&1 || { echo "chunk matrix failed"; tail -3 $O/asio_chunk.log; exit 1; }
echo done
