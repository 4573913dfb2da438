#!/bin/bash
# Round-5 call E: a lone wave's spare issue slots (chain ILP probe); the
# call site -- the watcher policy A/B (spin / tail / block) at 8/64/256
# callers, and netcache's chunk_size range 2-10 MiB.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05e
mkdir -p $O
timeout -k 10 120 python3 -u scripts/probes/chain_ilp.py --out $O/chain_ilp.json > $O/chain_ilp.log 2>&1 || { echo "chain probe failed"; tail -3 $O/chain_ilp.log; exit 1; }
cat $O/chain_ilp.log | head -4
timeout -k 10 400 python3 -u scripts/asio_scale.py --matrix watch --secs 2 --rounds 2 --out $O/asio_watch.json > $O/asio_watch.log 2>&1 || { echo "watch matrix failed"; tail -3 $O/asio_watch.log; exit 1; }
echo watch done
timeout -k 10 660 python3 -u scripts/asio_scale.py --matrix bigchunk --secs 2 --out $O/asio_bigchunk.json > $O/asio_bigchunk.log 2>&1 || { echo "bigchunk matrix failed"; tail -3 $O/asio_bigchunk.log; exit 1; }
echo done
