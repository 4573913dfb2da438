#!/bin/bash
# Round-6 call L: the N > 1 control plane bench.py now takes from
# sproxy_amd/shard.py, on the one-GPU box: the driver's own torch.distributed.run
# form with 2 ranks sharing the GPU, bench.py spawning its 2 ranks itself,
# one-rank gloo and RCCL groups, and the refusal of 2 ranks without --share-gpu.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06l
mkdir -p $O
show() { python3 -c "import json;d=json.loads([l for l in open('$O/$1.json').read().splitlines() if l.startswith('{')][-1]);print('$1', d['value'], d['n_gpus'], d['roofline'].get('avg_launch_ms'), d['ranks_seen']['backend'], d['ranks_seen']['world'], d['per_gpu'], d['parity']['ok'], d['parity']['checked'], d['config']['workload'][:40])"; }
timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --share-gpu --steps 10 --warmup 5 > $O/torchrun2.json 2> $O/torchrun2.err || { echo torchrun2 failed; tail -5 $O/torchrun2.err; exit 1; }; show torchrun2
timeout -k 10 400 python3 bench.py --gpus 2 --share-gpu --steps 10 --warmup 5 > $O/spawn2.json 2> $O/spawn2.err || { echo spawn2 failed; tail -5 $O/spawn2.err; exit 1; }; show spawn2
timeout -k 10 300 python3 bench.py --gpus 1 --dist-always --steps 10 --warmup 5 --no-cpu-baseline --extras none > $O/gloo1.json 2> $O/gloo1.err || { echo gloo1 failed; tail -3 $O/gloo1.err; exit 1; }; show gloo1
timeout -k 10 300 python3 bench.py --gpus 1 --dist-always --dist-backend nccl --steps 10 --warmup 5 --no-cpu-baseline --extras none > $O/nccl1.json 2> $O/nccl1.err || { echo nccl1 failed; tail -3 $O/nccl1.err; exit 1; }; show nccl1
timeout -k 10 120 python3 bench.py --gpus 2 --steps 2 --warmup 1 > $O/n2_refuse.out 2> $O/n2_refuse.err
r=$?; echo "n2 without --share-gpu rc=$r"; grep -m1 -o "LOCAL_RANK 1 but only 1 GPUs visible[^\"]*" $O/n2_refuse.err || true
[ $r -ne 0 ] || { echo "expected a refusal"; exit 1; }
echo done
