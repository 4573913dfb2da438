#!/bin/bash
# C3 bench line with each descriptor kernel forced, same box
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for V in xdma hybrid plan xdma hybrid; do
  timeout -k 10 300 python -u bench.py --config c3 --c3-variant $V --steps 20 --warmup 10 > gpurun_out/c3_$V.json 2> gpurun_out/c3_$V.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/c3_$V.json'));print('$V', d['ms_per_step'], d['config']['kernel'], d['roofline']['longest_alone_ms'], d['streamed']['ms_per_batch'])"
done
