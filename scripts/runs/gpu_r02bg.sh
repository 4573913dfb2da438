#!/bin/bash
# Round-2 call BG: the RCCL control plane on the one-GPU box -- bench.py with a one-rank
# nccl process group (--dist-always): plain, and under torch.distributed.run.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02bg
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --dist-always --steps 10 --warmup 5 --no-cpu-baseline > $O/nccl1.json 2> $O/nccl1.err; r=$?
echo "plain rc=$r"; [ $r -eq 0 ] || { tail -20 $O/nccl1.err; exit $r; }
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --dist-always --steps 10 --warmup 5 --no-cpu-baseline --config ctx > $O/nccl1_torchrun_ctx.json 2> $O/nccl1_torchrun_ctx.err; r=$?
echo "torchrun rc=$r"; [ $r -eq 0 ] || { tail -20 $O/nccl1_torchrun_ctx.err; exit $r; }
for f in nccl1 nccl1_torchrun_ctx; do python3 -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['n_gpus'], json.dumps(d['ranks_seen'])[:300])"; done
