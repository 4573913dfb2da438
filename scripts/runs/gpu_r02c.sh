#!/bin/bash
# Round-2 call C: batched MD5Update/Final contexts, the full-scale C3 parity
# test, CRC-32 (conflict-free table order, fastcrc via LDS-DMA); the
# batcher-driven C3 stream at inflight 1/2/3; the C3 and CRC lines; PMC
# traffic of the C3 descriptor kernel and the CRC kernels, LDS conflicts.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_ctx.py tests/test_c3_full.py tests/test_crc32.py -x -v --timeout 400 --timeout-method thread > $O/pytest_ctx_c3_crc.log 2>&1; r=$?
tail -25 $O/pytest_ctx_c3_crc.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python bench.py --steps 20 --warmup 10 > $O/c2.json 2> $O/c2.err; r=$?
echo "c2 rc=$r"; cut -c1-300 $O/c2.json; [ $r -eq 0 ] || exit $r
for F in 0 128; do
  timeout -k 10 300 python bench.py --config crc --fastcrc $F --steps 20 --warmup 10 > $O/crc_f$F.json 2> $O/crc_f$F.err; r=$?
  echo "crc fastcrc $F rc=$r"; cut -c1-300 $O/crc_f$F.json; [ $r -eq 0 ] || exit $r
done
for f in 1 2 3; do
  timeout -k 10 300 python bench.py --config c3q --c3q-inflight $f --steps 5 --warmup 2 > $O/c3q_f$f.json 2> $O/c3q_f$f.err; r=$?
  echo "c3q inflight $f rc=$r"; cut -c1-330 $O/c3q_f$f.json; [ $r -eq 0 ] || exit $r
done
timeout -k 10 400 python bench.py --config c3 --steps 10 --warmup 3 > $O/c3.json 2> $O/c3.err; r=$?
echo "c3 rc=$r"; cut -c1-300 $O/c3.json; [ $r -eq 0 ] || exit $r
pmc() {  # pmc NAME COUNTERS ARGS...
  local nm=$1 ctr=$2; shift 2
  timeout -s KILL 240 rocprofv3 --pmc $ctr --output-format csv -d $O/pmc_$nm -o pmc -- python3 bench.py "$@" > $O/pmc_$nm.log 2>&1
  local r=$?; echo "pmc $nm rc=$r"; return $r
}
pmc c3_fetch FETCH_SIZE --config c3 --c3-legs main --steps 3 --warmup 1 --parity-sample 0 || exit 1
pmc c3_write WRITE_SIZE --config c3 --c3-legs main --steps 3 --warmup 1 --parity-sample 0 || exit 1
python3 scripts/traffic_json.py $O/pmc_c3_fetch $O/pmc_c3_write c3@17179869184s1000 --source "r02c: bench.py --config c3 --c3-legs main, 4 dispatches" || exit 1
for F in 0 128; do
  pmc crc${F}_fetch FETCH_SIZE --config crc --fastcrc $F --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  pmc crc${F}_write WRITE_SIZE --config crc --fastcrc $F --steps 3 --warmup 1 --no-cpu-baseline || exit 1
  python3 scripts/traffic_json.py $O/pmc_crc${F}_fetch $O/pmc_crc${F}_write crc@1048576x16384f$F --source "r02c: bench.py --config crc --fastcrc $F, 4 dispatches" || exit 1
  pmc crc${F}_lds "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE SQ_BUSY_CYCLES" --config crc --fastcrc $F --steps 3 --warmup 1 --no-cpu-baseline || exit 1
done
python3 scripts/pmc_summary.py $O/pmc_crc0_lds > $O/pmc_crc0_lds_summary.json; python3 scripts/pmc_summary.py $O/pmc_crc128_lds > $O/pmc_crc128_lds_summary.json
cp profiles/traffic.json $O/traffic.json
timeout -k 10 300 python bench.py --config crc --steps 20 --warmup 10 > $O/crc_f0_after.json 2>&1; cut -c1-300 $O/crc_f0_after.json
exit 0
