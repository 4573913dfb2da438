#!/bin/bash
# Round-6 call C: why a c3q launch (6 batches through the queue, ~0.63 per
# launch when drained) runs below a hand-coalesced 4-batch launch (0.697):
# hand-coalesced launches of 4, 5, 6 and 8 batches, then the c3q line alone;
# plus the C5 test of memory registered outside the library.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06c
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu tests/test_c5_pinned.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
for k in 4 6 5 8; do
  timeout -k 10 300 python3 -u bench.py --config c3 --c3-legs coalesced --c3-coalesce $k --steps 10 --warmup 4 \
    --no-cpu-baseline > $O/coal_k$k.json 2> $O/coal_k$k.err || { echo "coalesced k=$k failed"; tail -3 $O/coal_k$k.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/coal_k$k.json').read().strip().splitlines()[-1])['coalesced'];print('coal', d['batches'], d['value'], d['ms_per_launch'], d['roofline']['frac'], d['lpt']['util'], (d['parity'] or {}).get('ok'))"
done
timeout -k 10 300 python3 -u bench.py --config c3q --steps 10 --warmup 3 --no-cpu-baseline > $O/c3q.json 2> $O/c3q.err || { echo "c3q failed"; tail -3 $O/c3q.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['roofline']['frac'], d['drained'], d['parity']['ok'])"
echo done
