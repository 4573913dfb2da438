#!/bin/bash
# Round-4 call AF: the C2 kernel with two LDS bases (M0) per stage instead of
# eight, A/B in process against the library before (build/abr04af), 15
# interleaved rounds, twice; the C2 parity tests; the driver's command.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "fixed or c2 or full or fold" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
for r in 1 2; do
  timeout -k 10 300 python3 -u scripts/lib_ab.py --old build/abr04af/libmd5hip_c2old.so --only c2 --rounds 15 > $O/c2_twom0_ab_$r.json 2> $O/c2_ab_$r.err || { echo "ab failed"; tail -3 $O/c2_ab_$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/c2_twom0_ab_$r.json').read().strip().splitlines()[-1]);v=d['c2'];print('c2 ab', v['median_new_vs_old'], v['best_new_vs_old'], v['equal'])"
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err || { echo "c2 driver failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c2_driver.json').read().strip().splitlines()[-1]);print('c2 driver', d['value'], d['ms_per_step'], d['roofline']['frac'])"
echo done
