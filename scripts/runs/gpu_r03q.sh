#!/bin/bash
# Round-3 call Q: fastcrc windows loaded with their two 64-B halves paired
# (bytes 0, 64, 16, 80, ...) instead of two runs of four -- CRC GPU tests,
# A/B against the old order (diag depth code 20) in one process, and the
# memory-side requests / FETCH_SIZE of the product at 1 M and 256 K blocks.
# Then: small batches (a netcache vector) through fed pairs (diag variant 9)
# beside the four product descriptor kernels, and the C3 batch with the
# longest groups' chains on CUs of their own (fed_ab.py, exclusive split).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_crc32.py -m gpu > $O/pytest_crc.log 2>&1; r=$?
tail -2 $O/pytest_crc.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/fastcrc_ab.py --rounds 5 > $O/fastcrc_ab.json 2> $O/fastcrc_ab.err; r=$?
tail -c 1200 $O/fastcrc_ab.json; [ $r -eq 0 ] || exit $r
pass() {  # name counters bench-args...
  local name=$1 cs=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d $O/$name -o pmc -- python3 bench.py "$@" --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/$name.log 2>&1 || { echo "pmc $name failed"; return 1; }
}
for w in "crc128|--config crc --fastcrc 128" "crc128q|--config crc --fastcrc 128 --chunks 262144" "crc64|--config crc --fastcrc 64"; do
  n=${w%%|*}; args=${w#*|}
  pass ${n}_a "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" $args && \
  pass ${n}_b "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" $args && \
  pass ${n}_f "FETCH_SIZE" $args || exit 1
  python3 scripts/ea_requests.py $O/${n}_a $O/${n}_b $O/${n}_f > $O/${n}.json && echo "$n ok"
done
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/ab_f -o pmc -- python3 scripts/diag/fastcrc_ab.py --rounds 1 --F 128 > $O/ab_f.log 2>&1; r=$?
echo "ab pmc rc=$r"; [ $r -eq 0 ] || exit $r
python3 scripts/pmc_summary.py $O/ab_f > $O/ab_fetch.json; r=$?
head -c 2000 $O/ab_fetch.json; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --fed --sizes 16,64,256,1024,4096,16384 > $O/small_fed_16k.json 2> $O/small_fed_16k.err; r=$?
cat $O/small_fed_16k.err; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python3 -u scripts/diag/small_batch_ab.py --fed --len 4096 --sizes 64,1024,16384 > $O/small_fed_4k.json 2> $O/small_fed_4k.err; r=$?
cat $O/small_fed_4k.err; [ $r -eq 0 ] || exit $r
timeout -k 10 400 python3 -u scripts/diag/fed_ab.py --rounds 5 --batches 2 > $O/fed_ab.json 2> $O/fed_ab.err; r=$?
tail -c 3000 $O/fed_ab.json; tail -3 $O/fed_ab.err
exit $r
