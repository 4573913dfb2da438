#!/bin/bash
# Round-5 call X: the control plane over gloo by default (bench.py
# --dist-backend).  The C2 line plain, with a one-rank group, under
# torch.distributed.run; two ranks sharing the one GPU (--share-gpu); and two
# ranks without it, which must refuse (one GPU visible).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
show() { python3 -c "import json;d=json.loads([l for l in open('$O/$1.json').read().splitlines() if l.startswith('{')][-1]);print('$1', d['value'], d['n_gpus'], d['roofline'].get('avg_launch_ms'), d['ranks_seen']['backend'], d['ranks_seen']['world'], d['parity']['ok'])"; }
B="--steps 20 --warmup 5 --no-cpu-baseline"
timeout -k 10 300 python3 bench.py --gpus 1 $B > $O/plain.json 2> $O/plain.err || { echo plain failed; exit 1; }; show plain
timeout -k 10 300 python3 bench.py --gpus 1 --dist-always $B > $O/group1.json 2> $O/group1.err || { echo group1 failed; tail -3 $O/group1.err; exit 1; }; show group1
timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --dist-always $B > $O/torchrun1.json 2> $O/torchrun1.err || { echo torchrun1 failed; tail -3 $O/torchrun1.err; exit 1; }; show torchrun1
timeout -k 10 400 python3 bench.py --gpus 2 --share-gpu --steps 10 --warmup 5 --no-cpu-baseline > $O/n2_share.json 2> $O/n2_share.err || { echo n2 failed; tail -3 $O/n2_share.err; exit 1; }; show n2_share
timeout -k 10 120 python3 bench.py --gpus 2 --steps 2 --warmup 1 --no-cpu-baseline > $O/n2_refuse.out 2> $O/n2_refuse.err
r=$?; echo "n2 without --share-gpu rc=$r"; grep -m1 -o "LOCAL_RANK 1 but only 1 GPUs visible[^\"]*" $O/n2_refuse.err || true
[ $r -ne 0 ] || { echo "expected a refusal"; exit 1; }
echo done
