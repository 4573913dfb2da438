#!/bin/bash
# Round-4 call AC: synchronous calls may use all but one slot (the last one
# coalesces) instead of holding to the inflight target.  The call-site
# threads matrix with this library and with the one before
# (build/abr04ac/old, through LD_LIBRARY_PATH), interleaved; the single-call
# latency; the queue / pool / ASIO-scale GPU tests.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04ac
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_queue.py tests/test_pool.py tests/test_asio_scale.py tests/test_c_site.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 240 python3 -u scripts/asio_scale.py --matrix threads --secs 3 --out $O/asio_threads_new.json > $O/asio_new.log 2>&1 || { echo "new matrix failed"; tail -3 $O/asio_new.log; exit 1; }
LD_LIBRARY_PATH=$PWD/build/abr04ac/old timeout -k 10 240 python3 -u scripts/asio_scale.py --matrix threads --secs 3 --out $O/asio_threads_old.json > $O/asio_old.log 2>&1 || { echo "old matrix failed"; tail -3 $O/asio_old.log; exit 1; }
timeout -k 10 240 python3 -u scripts/asio_scale.py --matrix threads --secs 3 --out $O/asio_threads_new2.json > $O/asio_new2.log 2>&1 || { echo "new2 matrix failed"; tail -3 $O/asio_new2.log; exit 1; }
timeout -k 10 200 python3 -u scripts/latency_probe.py --lib product=sproxy_amd/lib/libmd5hip.so old=build/abr04ac/old/libmd5hip.so > $O/queue_latency.json 2> $O/latency.log || { echo "latency failed"; tail -3 $O/latency.log; exit 1; }
tail -1 $O/queue_latency.json | cut -c1-600
echo done
