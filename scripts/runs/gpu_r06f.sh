#!/bin/bash
# Round-6 call F: the batcher's large slots ordered by md5hip_order_device_stable
# (rocPRIM radix sort: equal keys in chunk order).  The order / queue / C3 /
# pool GPU tests, the order A/B probe with the stable order added, then the
# c3q line and the default bench line.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06f
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  tests/test_queue.py tests/test_c3_full.py tests/test_pool.py tests/test_asio_scale.py \
  "tests/test_gpu_parity.py::test_order_device_stable_equals_host_order" \
  "tests/test_gpu_parity.py::test_order_device_is_a_longest_first_permutation" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; grep -E "FAILED|Error" $O/pytest.log | head; exit 1; }
timeout -k 10 400 python3 -u scripts/probes/order_ab.py --rounds 5 --out $O/order_ab.json > $O/order_ab.log 2>&1
rc=$?; tail -c 1800 $O/order_ab.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 -u bench.py --config c3q --steps 10 --warmup 3 --no-cpu-baseline > $O/c3q.json 2> $O/c3q.err || { echo "c3q failed"; tail -3 $O/c3q.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['roofline']['frac'], d['drained'], d['parity']['ok'])"
timeout -k 10 300 python3 -u bench.py --config c3 --c3-legs coalesced --c3-coalesce 6 --steps 10 --warmup 4 --no-cpu-baseline > $O/coal_k6.json 2> $O/coal_k6.err || { echo "coal failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/coal_k6.json').read().strip().splitlines()[-1])['coalesced'];print('coal', d['batches'], d['value'], d['ms_per_launch'], d['roofline']['frac'])"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err || { echo "bench failed"; tail -3 $O/c2_driver.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c2_driver.json').read().strip().splitlines()[-1]);print('c2', d['value'], d['roofline']['frac'], d['board'].get('gfxclk_mhz_median'), 'c3q', d['c3q']['value'], d['c3q']['roofline']['frac'], d['c3q']['parity']['ok'], 'c5', d['c5']['value'], d['c5']['parity']['ok'])"
echo done
