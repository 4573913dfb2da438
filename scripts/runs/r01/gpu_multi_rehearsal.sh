#!/bin/bash
# N>1 bench path rehearsed on one GPU (2 ranks, gloo control plane) + CRC clock
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export TMPDIR=/tmp
ok() { local r=$1; [ $r -eq 0 ] || [ $r -eq 1 ]; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err; r=$?
echo "n2 rc=$r"; cat gpurun_out/bench_n2_gloo.json; tail -3 gpurun_out/bench_n2_gloo.err; ok $r || exit $r
timeout -k 10 300 python -u scripts/clock_probe.py --kinds 48,51 > gpurun_out/clock_crc.json 2> gpurun_out/clock_crc.err; r=$?
echo "clock rc=$r"; cat gpurun_out/clock_crc.json; exit $r
