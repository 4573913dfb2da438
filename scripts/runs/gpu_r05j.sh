#!/bin/bash
# Round-5 call J: BALANCED with a tail wave beside each head wave (8 waves per
# CU; the older head waves take the longest groups, the younger tail waves
# the shortest, filling the head waves' idle issue slots -- prio_fill probe,
# r05i).  Parity tests on the BALANCED paths, in-process A/B against the
# library before (build/abr05), then the c3q and c3 lines.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  tests/test_gpu_parity.py tests/test_queue.py tests/test_c3_full.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 300 python3 -u scripts/lib_ab.py --old build/abr05/libmd5hip_old.so --only c3k3_balanced,c3k6_balanced --rounds 9 > $O/balanced_tail_ab.json 2> $O/ab.err || { echo "ab failed"; tail -3 $O/ab.err; exit 1; }
tail -1 $O/balanced_tail_ab.json | cut -c1-600
timeout -k 10 300 python3 bench.py --config c3q --steps 5 --warmup 2 > $O/c3q.json 2> $O/c3q.err || { echo "c3q failed"; tail -3 $O/c3q.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['roofline']['frac'], 'drained', d['drained'], d.get('parity',{}).get('ok'))"
timeout -k 10 300 python3 bench.py --config c3 --steps 5 --warmup 2 > $O/c3.json 2> $O/c3.err || { echo "c3 failed"; tail -3 $O/c3.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3.json').read().strip().splitlines()[-1]);print('c3', d['value'], d['roofline']['frac'])"
echo done
