#!/bin/bash
# kX3 product variant: full fixed-kernel parity + alternating bench lines on one box
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/pt.log 2>&1; r=$?; tail -2 gpurun_out/pt.log; [ $r -eq 0 ] || exit $r
for i in 1 2 3; do for v in xpose1nt xpose1ntx3; do
timeout -k 10 200 python bench.py --variant $v --no-cpu-baseline > gpurun_out/bx.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/bx.json'));print('$v', d['value'], d['roofline']['avg_launch_ms'], d['roofline']['frac'])"
done; done
