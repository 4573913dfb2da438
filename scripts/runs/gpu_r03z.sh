#!/bin/bash
# Round-3 call Z: does the caller polling its own launch change the c3q
# stream?  The same library with the polling on and off (an A/B build whose
# switch is an environment variable, never the product), interleaved, twice.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
cp build/abr03/libmd5hip_watch_switch.so sproxy_amd/lib/libmd5hip.so
for i in 1 2; do
  for w in on off; do
    if [ $w = off ]; then export MD5HIP_NO_WATCH_AB=1; else unset MD5HIP_NO_WATCH_AB; fi
    timeout -k 10 300 python3 bench.py --config c3q --steps 10 --no-cpu-baseline > $O/c3q_${w}_$i.json 2> $O/c3q_${w}_$i.err || { echo "c3q $w $i failed"; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/c3q_${w}_$i.json').read().strip().splitlines()[-1]);print('$w $i', d['value'], d['ms_per_step'], d['config']['queue']['launches'], d['config'].get('drained_gib_s'))"
  done
done
