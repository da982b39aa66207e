# Engine iteration: engine parity tests, per-shape GEMM timing, bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1; rc=$?
echo "pytest engine rc=$rc"; tail -4 gpurun_out/pytest_engine.log; [ $rc -eq 0 ] || exit $rc
GEMM_REPS=20 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1; rc=$?; echo "gemm rc=$rc"; grep -v amdgpu gpurun_out/gemm_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 --warmup 5 ${BENCH_ARGS:-} > gpurun_out/bench_iter.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_iter.log | cut -c1-700
