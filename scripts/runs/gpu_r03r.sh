#!/bin/bash
# Round-3 call R: (1) a lone chain's step mix (chain_probe.py --mix: the fed
# step with single adds instead of v_add3), (2) lone-wave VALU issue rates
# (valu_rate.py at one wave per SIMD), (3) the PMC bytes of fastcrc=128 with
# the paired-halves loads, for profiles/traffic.json.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 120 python3 -u scripts/diag/chain_probe.py --mix > $O/chain_mix.json 2> $O/chain_mix.err; r=$?
cat $O/chain_mix.json; [ $r -eq 0 ] || exit $r
timeout -k 10 200 python3 -u scripts/diag/valu_rate.py 1024 > $O/valu_rate_lone.json 2> $O/valu_rate_lone.err; r=$?
cat $O/valu_rate_lone.json; [ $r -eq 0 ] || exit $r
cp profiles/traffic.json $O/traffic.json
for c in FETCH_SIZE WRITE_SIZE VALU; do
  cs=$c; [ $c = VALU ] && cs="SQ_ACTIVE_INST_VALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
  timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d $O/pmc_crc128_$c -o pmc -- python3 bench.py --config crc --fastcrc 128 --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/pmc_crc128_$c.log 2>&1 || { echo "pmc $c failed"; exit 1; }
done
python3 scripts/traffic_json.py $O/pmc_crc128_FETCH_SIZE $O/pmc_crc128_WRITE_SIZE crc@1048576x16384f128 --valu $O/pmc_crc128_VALU --out $O/traffic.json --source "r03r: bench.py --config crc --fastcrc 128" ; r=$?
[ $r -eq 0 ] || exit $r
timeout -k 10 200 python3 bench.py --config crc --fastcrc 128 > $O/crc128.json 2> $O/crc128.err; r=$?
cut -c1-600 $O/crc128.json
exit $r
