#!/bin/bash
# Round-4 call A: the blocked-caller rework (one watcher per launch, per-slot
# sleeps), the null-stream ordering fix and the device-entry fixes on the GPU;
# the call site at ASIO scale (8/64/256 threads) with the round-3 batcher
# (build/abr04/old) beside it; the chunk_size matrix (16 KiB / 128 KiB / 1 MiB).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_pool.py tests/test_asio_scale.py tests/test_c_site.py tests/test_queue.py > $O/pytest.log 2>&1
rc=$?; tail -5 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 300 python3 -u scripts/asio_scale.py --matrix threads --secs 3 --out $O/asio_threads.json > $O/asio_threads.log 2>&1 || { echo "threads matrix failed"; tail -3 $O/asio_threads.log; exit 1; }
LD_LIBRARY_PATH=$PWD/build/abr04/old timeout -k 10 300 python3 -u scripts/asio_scale.py --matrix threads --secs 3 --out $O/asio_threads_r03lib.json > $O/asio_threads_r03lib.log 2>&1 || { echo "r03 threads matrix failed"; tail -3 $O/asio_threads_r03lib.log; exit 1; }
timeout -k 10 500 python3 -u scripts/asio_scale.py --matrix chunk --secs 2 --out $O/asio_chunk.json > $O/asio_chunk.log 2>&1 || { echo "chunk matrix failed"; tail -3 $O/asio_chunk.log; exit 1; }
echo done
