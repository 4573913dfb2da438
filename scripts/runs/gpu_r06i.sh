#!/bin/bash
# Round-6 call I: the order A/B again with two more within-key orders (descending index, round-robin over batches) -- the same
# 6-batch layout under host / device (queue) / shuffled equal-key orders and
# through the queue itself (scripts/probes/order_ab.py).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r06i
mkdir -p $O
timeout -k 10 400 python3 -u scripts/probes/order_ab.py --rounds 5 --out $O/order_ab.json > $O/order_ab.log 2>&1
rc=$?; tail -c 1500 $O/order_ab.log; [ $rc = 0 ] || exit 1
echo done
