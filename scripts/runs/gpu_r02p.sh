#!/bin/bash
# Round-2 call P: per-wave cache policy in every LDS-DMA loader, 128-B
# staging -- full GPU suite, policy A/B against the product, C2 / CRC / C3 lines.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02p
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python3 -u scripts/desc_policy_ab.py --rounds 3 > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/ab.json | cut -c1-3000
timeout -k 10 300 python bench.py > $O/c2.json 2> $O/c2.err; r=$?
echo "c2 rc=$r"; [ $r -eq 0 ] || exit $r
cut -c1-300 $O/c2.json
for f in 0 128; do
  timeout -k 10 300 python bench.py --config crc --fastcrc $f > $O/crc_f$f.json 2> $O/crc_f$f.err; r=$?
  echo "crc f$f rc=$r"; [ $r -eq 0 ] || exit $r
  cut -c1-300 $O/crc_f$f.json
done
timeout -k 10 300 python bench.py --config c3q --c3q-inflight 1 --steps 5 --warmup 2 > $O/c3q_f1.json 2> $O/c3q_f1.err; r=$?
echo "c3q rc=$r"; [ $r -eq 0 ] || exit $r
cut -c1-300 $O/c3q_f1.json
