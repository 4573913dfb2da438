#!/bin/bash
# Round-3 call Y: the c3q stream dropped (launches 41 -> 71 per run) after the
# batcher's descriptor arrays became fine-grained: host write speed by
# hipHostMalloc flag, then bench --config c3q with the product library and
# with the library before the in-place descriptors (same box).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03y
mkdir -p $O
timeout -k 10 120 python3 -u scripts/diag/host_alloc_write.py > $O/host_alloc_write.json 2> $O/host_alloc_write.err; r=$?
cat $O/host_alloc_write.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 bench.py --config c3q --steps 10 --no-cpu-baseline > $O/c3q_product.json 2> $O/c3q_product.err; r=$?
python3 -c "import json;d=json.loads(open('$O/c3q_product.json').read().strip().splitlines()[-1]);print('product', d['value'], d['ms_per_step'], d['config']['queue']['launches'])"; [ $r -eq 0 ] || exit $r
cp build/abr03/libmd5hip_desc_copy.so sproxy_amd/lib/libmd5hip.so
timeout -k 10 300 python3 bench.py --config c3q --steps 10 --no-cpu-baseline > $O/c3q_desc_copy.json 2> $O/c3q_desc_copy.err; r=$?
python3 -c "import json;d=json.loads(open('$O/c3q_desc_copy.json').read().strip().splitlines()[-1]);print('desc_copy', d['value'], d['ms_per_step'], d['config']['queue']['launches'])"; [ $r -eq 0 ] || exit $r
cp build/abr03/libmd5hip_nosplit.so sproxy_amd/lib/libmd5hip.so
timeout -k 10 300 python3 bench.py --config c3q --steps 10 --no-cpu-baseline > $O/c3q_nosplit.json 2> $O/c3q_nosplit.err; r=$?
python3 -c "import json;d=json.loads(open('$O/c3q_nosplit.json').read().strip().splitlines()[-1]);print('nosplit', d['value'], d['ms_per_step'], d['config']['queue']['launches'])"; [ $r -eq 0 ] || exit $r
cp build/abr03/libmd5hip_lane_small.so sproxy_amd/lib/libmd5hip.so
timeout -k 10 300 python3 bench.py --config c3q --steps 10 --no-cpu-baseline > $O/c3q_lane_small.json 2> $O/c3q_lane_small.err; r=$?
python3 -c "import json;d=json.loads(open('$O/c3q_lane_small.json').read().strip().splitlines()[-1]);print('lane_small', d['value'], d['ms_per_step'], d['config']['queue']['launches'])"
exit $r
