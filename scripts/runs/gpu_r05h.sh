#!/bin/bash
# Round-5 call H: the fastcrc call site -- host blocks staging only their
# windows (this library) against the library before (build/abr05/old) and
# the calling thread, 64 x 16 KiB vectors, 1 / 8 / 64 callers.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 400 python3 -u scripts/asio_scale.py --matrix fastcrc --secs 2 --out $O/asio_fastcrc.json > $O/asio_fastcrc.log 2>&1 || { echo "fastcrc matrix failed"; tail -3 $O/asio_fastcrc.log; exit 1; }
echo done
