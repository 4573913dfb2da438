#!/bin/bash
# Round-3 call AC: pure kernel time of crc32_split and md5_desc_fed on small
# batches (rocprofv3 kernel trace of small_batch_ab), to split a call's time
# between kernel, launch and host.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_crc -o crc -- python3 scripts/diag/small_batch_ab.py --crc --sizes 64,1024 --iters 50 --rounds 1 > $O/prof_crc.log 2>&1; r=$?
echo "crc prof rc=$r"; [ $r -eq 0 ] || exit $r
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_md5 -o md5 -- python3 scripts/diag/small_batch_ab.py --sizes 64,1024 --iters 50 --rounds 1 > $O/prof_md5.log 2>&1; r=$?
echo "md5 prof rc=$r"
cat $O/prof_crc/crc_kernel_stats.csv | cut -c1-220; cat $O/prof_md5/md5_kernel_stats.csv | cut -c1-220
exit $r
