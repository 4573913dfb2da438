#!/bin/bash
# Round-3 call AA: where the CRC split stops winning for long chunks -- the
# streaming kernels against crc32_split at 64 KiB and 1 MiB blocks (netcache
# chunk_size up to 10 MiB), and at 16 KiB / 4 KiB past 16 chunks per CU.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --crc --len 1048576 --iters 20 --sizes 64,1024,4096 > $O/crc_1m.json 2> $O/crc_1m.err; r=$?
cat $O/crc_1m.err; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --crc --len 65536 --iters 30 --sizes 1024,4096,16384,32768 > $O/crc_64k.json 2> $O/crc_64k.err; r=$?
cat $O/crc_64k.err; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --crc --len 16384 --iters 30 --sizes 8192,16384,32768,49152 > $O/crc_16k.json 2> $O/crc_16k.err; r=$?
cat $O/crc_16k.err; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --crc --len 1024 --iters 30 --sizes 1024,4096,16384 > $O/crc_1k.json 2> $O/crc_1k.err; r=$?
cat $O/crc_1k.err
exit $r
