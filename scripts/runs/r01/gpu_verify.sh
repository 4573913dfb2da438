cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/v
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/v/pytest_gpu.log 2>&1; r=$?
echo "pytest rc=$r"; tail -2 gpurun_out/v/pytest_gpu.log; [ $r -eq 0 ] || exit $r
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/v/smoke.log 2>&1 && tail -1 gpurun_out/v/smoke.log &&
timeout -k 10 300 python bench.py > gpurun_out/v/bench.json 2> gpurun_out/v/bench.err && cat gpurun_out/v/bench.json
