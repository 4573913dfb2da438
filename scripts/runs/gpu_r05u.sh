#!/bin/bash
# Round-5 call U: the N > 1 bench path on the one-GPU box -- bench.py --gpus 2
# spawning its own two gloo ranks (each the C4 shard, 2,097,152 x 16 KiB),
# both on the one GPU; and the one-rank RCCL control plane (--dist-always).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05u
mkdir -p $O
timeout -k 10 400 python3 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 5 --no-cpu-baseline > $O/n2_gloo.json 2> $O/n2_gloo.err || { echo "n2 failed"; tail -5 $O/n2_gloo.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/n2_gloo.json').read().strip().splitlines()[-1]);print('n2', d['value'], d['n_gpus'], d['ms_per_step'], d['ranks_seen']['world'], d['parity']['ok'], d['config']['workload'])"
timeout -k 10 400 python3 bench.py --gpus 1 --dist-always --steps 10 --warmup 5 --no-cpu-baseline > $O/nccl1.json 2> $O/nccl1.err || { echo "nccl1 failed"; tail -5 $O/nccl1.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/nccl1.json').read().strip().splitlines()[-1]);print('nccl1', d['value'], d['ranks_seen']['backend'], d['ranks_seen']['world'], d['parity']['ok'])"
echo done
