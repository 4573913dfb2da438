#!/bin/bash
# Round-5 call S: rocprofv3 kernel-trace summaries of the other bench lines
# (c3q, crcq, fastcrc one launch, crc, ctx, c3), each beside the line's own
# HIP-event launch time.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05s
mkdir -p $O
prof() {  # name bench-args...
  local name=$1; shift
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o $name -- python3 bench.py "$@" --no-cpu-baseline > $O/$name.log 2>&1
  local r=$?; echo "rocprof $name rc $r"; [ $r = 0 ] || exit 1
  grep '^{' $O/$name.log | tail -1 > $O/$name.json
}
prof c3q --config c3q
prof crcq --config crcq
prof crc128 --config crc --fastcrc 128
prof crc --config crc
prof ctx --config ctx
prof c3 --config c3
echo done
