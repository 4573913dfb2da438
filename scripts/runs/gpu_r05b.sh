#!/bin/bash
# Round-5 call B: the failure policy / host_fixed / watcher tree -- the whole
# GPU suite, then the watcher A/B (spin / tail / block) at 8/64/256 callers,
# then the call site at 2-10 MiB blocks.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 400 python3 -u scripts/asio_scale.py --matrix watch --secs 2 --rounds 2 --out $O/asio_watch.json > $O/asio_watch.log 2>&1 || { echo "watch matrix failed"; tail -3 $O/asio_watch.log; exit 1; }
echo watch done
timeout -k 10 600 python3 -u scripts/asio_scale.py --matrix bigchunk --secs 2 --out $O/asio_bigchunk.json > $O/asio_bigchunk.log 2>&1 || { echo "bigchunk matrix failed"; tail -3 $O/asio_bigchunk.log; exit 1; }
echo done
