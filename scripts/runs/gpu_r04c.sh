#!/bin/bash
# Round-4 call C: synchronous submits coalesce on a busy device, chained
# launches.  The whole GPU suite; the call site at ASIO scale; c3q with
# chaining on and off (interleaved) and its launch gaps; the single-caller
# queue latency; BALANCED with two images (A/B build build/abr04/bal2).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests \
  --deselect "tests/test_asio_scale.py::test_asio_scale_cpu_per_call_bounded" > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 240 python3 -u scripts/asio_scale.py --matrix threads --secs 3 --out $O/asio_threads.json > $O/asio_threads.log 2>&1 || { echo "threads matrix failed"; tail -3 $O/asio_threads.log; exit 1; }
for i in 1 2; do
  for c in 1 0; do
    timeout -k 10 200 python3 bench.py --config c3q --steps 10 --no-cpu-baseline --c3q-chain $c > $O/c3q_chain${c}_$i.json 2> $O/c3q_chain${c}_$i.err || { echo "c3q chain $c failed"; tail -3 $O/c3q_chain${c}_$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/c3q_chain${c}_$i.json').read().strip().splitlines()[-1]);print('chain $c run $i', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained']['value'], d['config']['queue']['launches'])"
  done
done
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/c3q_trace -o trace -- python3 bench.py --config c3q --steps 10 --no-cpu-baseline > $O/c3q_traced.json 2> $O/c3q_traced.err || { echo "c3q traced failed"; exit 1; }
python3 scripts/queue_gaps.py $O/c3q_trace > $O/c3q_gaps.json 2>&1
timeout -k 10 200 python3 scripts/latency_probe.py --iters 200 > $O/queue_latency.json 2> $O/queue_latency.err || { echo "latency probe failed"; exit 1; }
timeout -k 10 300 python3 -u scripts/lib_ab.py --rounds 9 --old sproxy_amd/lib/libmd5hip.so --extra bal2=build/abr04/bal2/libmd5hip.so --only c3k3_balanced,c3k6_balanced > $O/balanced_ab.log 2>&1 || { echo "balanced A/B failed"; tail -3 $O/balanced_ab.log; exit 1; }
echo done
