#!/bin/bash
# Round-5 call P: INTEGRATION.md §2's routing table re-measured on the round-5
# library (TAIL watcher, windowed staging, host_fixed outside the lock):
# 16 / 128 / 256 / 1,024 KiB blocks, 8 / 64-block vectors, 1 / 8 / 64
# callers, queue vs the calling thread, pageable, every digest checked.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
timeout -k 10 900 python3 -u scripts/asio_scale.py --matrix chunk --sizes-kib 16,128,256,1024 --secs 3 --out $O/asio_chunk.json > $O/asio.log 2>&1
rc=$?; [ $rc = 0 ] || { echo "asio failed $rc"; tail -3 $O/asio.log; exit 1; }
echo done
