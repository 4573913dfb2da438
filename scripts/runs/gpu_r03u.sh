#!/bin/bash
# Round-3 call U: CRC-32 split across a wave (crc32_split, CRC32HIP_SPLIT) --
# the CRC GPU tests, then small-batch launch times of the streaming kernels
# against the split one (16 KiB and 4 KiB blocks, up to 65,536 chunks).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_crc32.py -m gpu > $O/pytest_crc.log 2>&1; r=$?
tail -3 $O/pytest_crc.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --crc --sizes 16,64,256,1024,4096,16384,65536 > $O/crc_small_16k.json 2> $O/crc_small_16k.err; r=$?
cat $O/crc_small_16k.err; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --crc --len 4096 --sizes 64,1024,16384,65536 > $O/crc_small_4k.json 2> $O/crc_small_4k.err; r=$?
cat $O/crc_small_4k.err
exit $r
