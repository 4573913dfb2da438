#!/bin/bash
# Round-5 call F: TAIL watcher with a progress-thread fallback (instead of
# blocking in hipEventSynchronize) against SPIN at 8/64/256 callers; the
# fastcrc stream and c3q after slot waits poll fast; 2 and 10 MiB blocks
# from 64 callers through 1 GiB slices; the driver's C2 command.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05f
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_asio_scale.py tests/test_c_site.py tests/test_queue.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 300 python3 -u scripts/asio_scale.py --matrix watch --secs 2 --rounds 2 --policies spin,tail --out $O/asio_watch.json > $O/asio_watch.log 2>&1 || { echo "watch matrix failed"; tail -3 $O/asio_watch.log; exit 1; }
echo watch done
timeout -k 10 300 python3 bench.py --config crcq --steps 10 --warmup 2 > $O/crcq.json 2> $O/crcq.err || { echo "crcq failed"; tail -3 $O/crcq.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/crcq.json').read().strip().splitlines()[-1]);print('crcq', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained'], d.get('parity',{}).get('ok'))"
timeout -k 10 300 python3 bench.py --config c3q --steps 5 --warmup 2 > $O/c3q.json 2> $O/c3q.err || { echo "c3q failed"; tail -3 $O/c3q.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['roofline']['frac'], 'drained', d['drained']['value'], d.get('parity',{}).get('ok'))"
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/c2_driver.json 2> $O/c2_driver.err || { echo "c2 driver failed"; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c2_driver.json').read().strip().splitlines()[-1]);print('c2 driver', d['value'], d['ms_per_step'], d['roofline']['frac'], d['cpu_baseline']['value'])"
timeout -k 10 300 python3 bench.py --config c5 --steps 5 --warmup 2 > $O/c5.json 2> $O/c5.err || { echo "c5 failed"; tail -3 $O/c5.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]);print('c5', d['value'], d.get('parity',{}).get('ok'))"
timeout -k 10 300 python3 -u scripts/asio_scale.py --matrix bigchunk --slice-mib 1024 --secs 2 --out $O/asio_bigchunk_1g.json > $O/asio_bigchunk_1g.log 2>&1 || { echo "bigchunk 1g failed"; tail -3 $O/asio_bigchunk_1g.log; exit 1; }
echo done
