#!/bin/bash
# Round-4 call V: BALANCED with two waves per SIMD (8-wave workgroups)
# against the final one-wave-per-SIMD library
# (build/abr04v/libmd5hip_final4.so): GPU tests that run BALANCED, the
# in-process A/B on 3 and 6 coalesced C3 batches, c3q twice.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04v
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_c3_full.py tests/test_queue.py tests/test_gpu_parity.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 400 python3 -u scripts/lib_ab.py --old build/abr04v/libmd5hip_final4.so --only c3k3_balanced,c3k6_balanced --rounds 7 > $O/balanced_2wps_ab.json 2> $O/balanced_2wps_ab.err || { echo "ab failed"; tail -3 $O/balanced_2wps_ab.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/balanced_2wps_ab.json').read().strip().splitlines()[-1]);print({k:(v['median_new_vs_old'],v['equal']) for k,v in d.items() if isinstance(v,dict) and 'equal' in v})"
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config c3q --no-cpu-baseline > $O/c3q_$r.json 2> $O/c3q_$r.err || { echo "c3q failed"; tail -3 $O/c3q_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c3q_$r.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['value'], d['parity']['ok'])"
done
echo done
