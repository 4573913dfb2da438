#!/bin/bash
# Round-3 call AD: where a synchronous device-resident call's time goes now
# (FED / CRC split, caller polling, in-place descriptors): host stamps joined
# with the kernel trace, MD5 and CRC-32, 64 x 16 KiB; and un-profiled.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
for k in md5 crc; do
  extra=""; [ $k = crc ] && extra="--crc"
  timeout -k 10 200 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $O/tr_$k -o t -- python3 scripts/call_breakdown.py --mode device --nb 64 --calls 200 $extra --out $O/stamps_$k.json > $O/run_$k.log 2>&1; r=$?
  echo "$k rc=$r"; tail -1 $O/run_$k.log; [ $r -eq 0 ] || exit $r
  python3 scripts/call_breakdown.py --join $O/tr_$k --stamps $O/stamps_$k.json > $O/breakdown_$k.json 2>&1
  timeout -k 10 120 python3 scripts/call_breakdown.py --mode device --nb 64 --calls 300 $extra --out $O/plain_$k.json
done
cat $O/breakdown_md5.json $O/breakdown_crc.json
