# Round-end check: full GPU parity suite, smoke(), default bench (CPU baseline + live roofline), rocprof stats.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/end
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/end/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/end/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/end/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/end/smoke.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/end/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/end/prof.log" 2>&1; echo "prof rc=$?"
cd "$GRAFT_REPO_ROOT" && timeout -k 10 600 python bench.py > gpurun_out/end/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/end/bench.log
