#!/bin/bash
# Round-2 call O: descriptor kernels (XDMA / HYBRID) -- nt vs default cache
# policy on line-aligned and 16-B-packed batches; HBM bytes on rag16 and c3.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02o
mkdir -p $O
timeout -k 10 400 python3 -u scripts/desc_policy_ab.py --rounds 3 > $O/ab.json 2> $O/ab.err; r=$?
echo "ab rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/ab.json | cut -c1-3500
for s in rag16 c3; do
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_$s -o pmc -- python3 scripts/desc_policy_ab.py --rounds 1 --sets $s > $O/pmc_$s.log 2>&1; r=$?
  echo "pmc $s rc=$r"; [ $r -eq 0 ] || exit $r
  python3 scripts/pmc_summary.py $O/pmc_$s > $O/pmc_${s}_summary.json || exit 1
  grep -E '"(diag|md5)|hbm_read_bytes|dur_ms' $O/pmc_${s}_summary.json
done
