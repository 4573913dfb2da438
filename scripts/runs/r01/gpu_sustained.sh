#!/bin/bash
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in xpose2 lds128 xpose1 lds64; do
  timeout -k 10 240 python bench.py --steps 40 --warmup 5 --variant $v --no-cpu-baseline > gpurun_out/sus_$v.json 2> gpurun_out/sus_$v.err; r=$?
  echo "$v rc=$r $(python3 -c "import json;d=json.load(open('gpurun_out/sus_$v.json'));print(d['value'],'GiB/s',d['roofline']['avg_launch_ms'],'ms',d['roofline']['frac'])")"
  [ $r -eq 0 ] || exit $r
done
timeout -k 10 300 python scripts/profile_kernels.py --rounds 3 --reps 20 --only xpose2,lds128,xpose1,compute_only > gpurun_out/sus_interleaved.json 2>/dev/null; echo "interleaved rc=$?"
python3 -c "
import json; d=json.load(open('gpurun_out/sus_interleaved.json'))
for k,v in sorted(d['results'].items(), key=lambda kv: kv[1]['ms_median']): print('%-14s %8.4f ms  %8.1f GB/s' % (k, v['ms_median'], v['payload_GBps']))"
