# Full GPU check: parity tests, default bench (with CPU baseline), non-pipelined bench, rocprof stats.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -m pytest tests -m gpu -q -p no:cacheprovider -rf ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -12 gpurun_out/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 600 python bench.py ${BENCH_DEFAULT_ARGS:-} ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-prefetch --steps 10 --warmup 3 ${BENCH_ARGS:-} > gpurun_out/bench_noprefetch.log 2>&1; rc=$?; echo "bench-noprefetch rc=$rc"; tail -1 gpurun_out/bench_noprefetch.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof.log" 2>&1; echo "prof rc=$?"
if [ -n "${GEMM_BENCH:-}" ]; then cd "$GRAFT_REPO_ROOT" && timeout -k 10 300 python scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; echo "gemm_bench rc=$?"; fi
