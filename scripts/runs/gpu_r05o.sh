#!/bin/bash
# Round-5 call O: netcache's own stress configuration (driver_test.c:583-586,
# 256 KiB blocks, fastcrc 128) -- the GPU test, and the call-site matrix at
# 256 KiB blocks (queue vs the calling thread, 8 / 64-block vectors,
# 1 / 8 / 64 callers, pageable).
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05o
mkdir -p $O
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_crc32.py > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 400 python3 -u scripts/asio_scale.py --matrix chunk --sizes-kib 256 --secs 3 --out $O/asio_chunk256.json > $O/asio.log 2>&1
rc=$?; [ $rc = 0 ] || { echo "asio failed $rc"; tail -5 $O/asio.log; exit 1; }
python3 - "$O/asio_chunk256.json" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
for r in d["runs"]:
    print(r["target"], r["threads"], r["blocks"], r["block_bytes"], r["lat_us"]["p50"], r["gib_s"], r.get("thread_cpu_us_per_call", {}).get("mean"), r["mismatches"])
PY
echo done
