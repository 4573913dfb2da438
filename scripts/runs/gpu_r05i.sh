#!/bin/bash
# Round-5 call I: can a low-priority filler wave take a lone MD5 chain
# wave's idle issue slots (prio_fill probe); whole-block CRC-32 at the call
# site on the calling thread (the queue's side is in r05h).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 120 python3 -u scripts/probes/prio_fill.py --out $O/prio_fill.json > $O/prio_fill.log 2>&1 || { echo "prio probe failed"; tail -3 $O/prio_fill.log; exit 1; }
head -4 $O/prio_fill.log
for T in 1 8 64; do
  ASIO_WS_MIB=2048 ASIO_CRC=0 timeout -k 10 120 build/c/asio_scale host $T 64 16384 2 > $O/crc0_host_t$T.json 2>&1 || { echo "host crc $T failed"; exit 1; }
done
python3 -c "
import json
for T in (1,8,64):
    d=json.loads(open('$O/crc0_host_t%d.json'%T).read().strip().splitlines()[-1]); print('host crc0', T, d['lat_us']['p50'], d['gib_s'], d['mismatches'])
"
echo done
