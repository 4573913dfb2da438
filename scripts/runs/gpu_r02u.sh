#!/bin/bash
# Round-2 call U: pipelined fastcrc kernel -- tests, f128 / f64 lines.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r02u
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_crc32.py -m gpu > $O/pytest.log 2>&1; r=$?
tail -3 $O/pytest.log; [ $r -eq 0 ] || exit $r
for f in 128 64 4096; do
  timeout -k 10 300 python bench.py --config crc --fastcrc $f > $O/crc_f$f.json 2> $O/crc_f$f.err; r=$?
  echo "crc f$f rc=$r"; [ $r -eq 0 ] || exit $r
  cut -c1-330 $O/crc_f$f.json
done
