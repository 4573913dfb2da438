#!/bin/bash
# Round-2 call L: BALANCED cache policy -- nt (product) vs default-policy
# LDS-DMA on coalesced C3 batches: time (A/B) and HBM bytes (FETCH_SIZE).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02l
mkdir -p $O
timeout -k 10 300 python3 -u scripts/c3_wide_ab.py --batches 3 5 --rounds 3 --kinds 0 19 5 18 6 16 10 17 > $O/wide.json 2> $O/wide.err; r=$?
echo "wide rc=$r"; [ $r -eq 0 ] || exit $r
tail -1 $O/wide.json | cut -c1-2500
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o pmc -- python3 scripts/c3_wide_ab.py --batches 3 --rounds 1 --kinds 6 16 10 17 19 > $O/pmc_fetch.log 2>&1; r=$?
echo "pmc rc=$r"; [ $r -eq 0 ] || exit $r
python3 scripts/pmc_summary.py $O/pmc_fetch > $O/pmc_fetch_summary.json; r=$?
grep -E '"(diag|md5)|FETCH|read_bytes|dur_ms' $O/pmc_fetch_summary.json
exit $r
