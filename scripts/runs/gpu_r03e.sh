#!/bin/bash
# Round-3 call E: (1) the pool's call site without Python in the timed path;
# (2) what fastcrc=128's "1.16x" HBM bytes are: memory-side
# read requests by size (TCC_EA0_RDREQ, _32B, _64B, _128B) for the fastcrc
# kernel at two batch sizes and for two streaming kernels that calibrate the
# counters (C2 MD5, C2-shape CRC), two counters per pass.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 300 python3 -u scripts/pool_latency_probe.py --iters 100 --threads 8 --secs 2 > $O/pool_latency.json 2> $O/pool_latency.err; r=$?
echo "pool probe rc=$r"; tail -2 $O/pool_latency.err; [ $r -eq 0 ] || exit $r
pass() {  # name counters bench-args...
  local name=$1 cs=$2; shift 2
  timeout -s KILL 120 rocprofv3 --pmc $cs --output-format csv -d $O/$name -o pmc -- python3 bench.py "$@" --steps 4 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/$name.log 2>&1 || { echo "pmc $name failed"; return 1; }
}
for w in "c2|" "crc0|--config crc" "crc128|--config crc --fastcrc 128" "crc128q|--config crc --fastcrc 128 --chunks 262144" "crc64|--config crc --fastcrc 64"; do
  n=${w%%|*}; args=${w#*|}
  pass ${n}_a "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum" $args && \
  pass ${n}_b "TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum" $args && \
  pass ${n}_f "FETCH_SIZE" $args || exit 1
  python3 scripts/ea_requests.py $O/${n}_a $O/${n}_b $O/${n}_f > $O/${n}.json && echo "$n ok"
done
exit 0
