#!/bin/bash
# Round-4 call Z: BALANCED's persistent body without the unused split-queue
# and wide-stage paths (new code hash): the GPU suite, the in-process A/B
# against the library before (build/abr04z/libmd5hip_final4.so), c3q twice,
# and PMC traffic for every bench line's kernel.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 400 python3 -u scripts/lib_ab.py --old build/abr04z/libmd5hip_final4.so --only c3k3_balanced,c3k6_balanced --rounds 7 > $O/balanced_simplified_ab.json 2> $O/balanced_simplified_ab.err || { echo "ab failed"; tail -3 $O/balanced_simplified_ab.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/balanced_simplified_ab.json').read().strip().splitlines()[-1]);print({k:(v['median_new_vs_old'],v['equal']) for k,v in d.items() if isinstance(v,dict) and 'equal' in v})"
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --config c3q --no-cpu-baseline > $O/c3q_$r.json 2> $O/c3q_$r.err || { echo "c3q failed"; tail -3 $O/c3q_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c3q_$r.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['value'], d['parity']['ok'])"
done
bash scripts/gpu_pmc_traffic.sh $O/pmc || { echo "pmc failed"; exit 1; }
echo done
