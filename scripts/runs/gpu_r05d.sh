#!/bin/bash
# Round-5 call D: the round-5 tree's GPU suite; BALANCED with compiler-visible
# lgkm waits A/B'd in process against the library before (build/abr05), then
# the c3q line; SQ counter passes on c3q's BALANCED launches (and C2 for
# contrast); the fastcrc stream through the queue with PMC bytes; the
# window-read ceiling probe.
cd "$GRAFT_REPO_ROOT" || exit 1
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc = 0 ] || { echo "pytest failed $rc"; exit 1; }
timeout -k 10 300 python3 -u scripts/lib_ab.py --old build/abr05/libmd5hip_old.so --only c3k3_balanced,c3k6_balanced --rounds 9 > $O/balanced_waitcnt_ab.json 2> $O/ab.err || { echo "ab failed"; tail -3 $O/ab.err; exit 1; }
tail -1 $O/balanced_waitcnt_ab.json | cut -c1-400
timeout -k 10 300 python3 bench.py --config c3q --steps 5 --warmup 2 > $O/c3q.json 2> $O/c3q.err || { echo "c3q failed"; tail -3 $O/c3q.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/c3q.json').read().strip().splitlines()[-1]);print('c3q', d['value'], d['roofline']['frac'], 'drained', d['drained'], d.get('parity',{}).get('ok'))"
timeout -s KILL 60 rocprofv3 -L > $O/counters_avail.txt 2>&1; echo "list rc $?"
avail() { python3 - "$O/counters_avail.txt" "$@" <<'PY'
import re, sys
txt = open(sys.argv[1]).read()
have = set(re.findall(r"\b([A-Z][A-Z0-9_]+)\b", txt))
print(" ".join(c for c in sys.argv[2:] if c in have))
PY
}
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM"
P3="SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_FLAT SQ_INST_CYCLES_SALU SQ_IFETCH SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
pmc() {  # name counters bench-args...
  local name=$1 cs=$2; shift 2
  [ -n "$cs" ] || { echo "pmc $name: no counters available"; return 0; }
  timeout -s KILL 240 rocprofv3 --pmc $cs --output-format csv -d $O/$name -o pmc -- python3 bench.py "$@" --no-cpu-baseline --parity-sample 0 > $O/$name.log 2>&1
  local r=$?
  echo "pmc $name rc $r ($cs)"
  case $r in 124|134|137|139) exit 1;; esac
  return 0
}
pmc c3q_p1 "$(avail $P1)" --config c3q --steps 2 --warmup 1
pmc c3q_p2 "$(avail $P2)" --config c3q --steps 2 --warmup 1
pmc c3q_p3 "$(avail $P3) GRBM_GUI_ACTIVE" --config c3q --steps 2 --warmup 1
pmc c2_p1 "$(avail $P1)" --steps 3 --warmup 1
pmc c2_p2 "$(avail $P2)" --steps 3 --warmup 1
python3 scripts/pmc_stall.py --kernel balanced $O/c3q_p1 $O/c3q_p2 $O/c3q_p3 --out $O/c3q_balanced_stall.json > /dev/null || echo "stall summary c3q failed"
python3 scripts/pmc_stall.py --kernel md5_fixed_xdma1nt $O/c2_p1 $O/c2_p2 --out $O/c2_stall.json > /dev/null || echo "stall summary c2 failed"
timeout -k 10 300 python3 bench.py --config crcq --steps 10 --warmup 2 > $O/crcq.json 2> $O/crcq.err || { echo "crcq failed"; tail -3 $O/crcq.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/crcq.json').read().strip().splitlines()[-1]);print('crcq', d['value'], d['ms_per_step'], d['roofline']['frac'], d['drained'], d.get('parity',{}).get('ok'))"
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $O/crcq_$c -o pmc -- python3 bench.py --config crcq --steps 3 --warmup 1 --no-cpu-baseline --parity-sample 0 > $O/crcq_$c.log 2>&1
  r=$?; echo "crcq pmc $c rc $r"; case $r in 0) ;; *) exit 1;; esac
done
timeout -k 10 300 python3 -u scripts/probes/window_read.py --out $O/window_read.json > $O/window_read.log 2>&1 || { echo "window probe failed"; tail -3 $O/window_read.log; exit 1; }
tail -1 $O/window_read.log | cut -c1-600
echo done
