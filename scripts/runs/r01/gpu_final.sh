#!/bin/bash
# End-of-session evidence: the round evidence call, then the N>1 bench path
# rehearsed with two ranks on the one GPU (gloo control plane).
cd "$GRAFT_REPO_ROOT" || exit 1
bash scripts/gpu_evidence.sh; r=$?
[ $r -eq 0 ] || exit $r
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 --dist-backend gloo > gpurun_out/bench_n2_gloo.json 2> gpurun_out/bench_n2_gloo.err; r=$?
echo "n2 rc=$r"; cut -c1-400 gpurun_out/bench_n2_gloo.json; exit $r
