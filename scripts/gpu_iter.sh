# Iteration loop: engine GEMM parity (both kernel families), per-shape GEMM timing, bench.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py ${PYTEST_EXTRA:-} -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1; rc=$?
echo "pytest engine rc=$rc"; tail -5 gpurun_out/pytest_engine.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_lds.log 2>&1; echo "gemm lds rc=$?"; cat gpurun_out/gemm_lds.log | grep -v amdgpu
if [ -n "${GEMM_BOTH:-}" ]; then PCS_GEMM_PERSIST=0 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_nopersist.log 2>&1; echo "gemm nopersist rc=$?"; PCS_GEMM_IMPL=1 timeout -k 10 200 python scripts/gemm_bench.py > gpurun_out/gemm_direct.log 2>&1; echo "gemm direct rc=$?"; fi
if [ -n "${MODELS:-}" ]; then timeout -k 10 600 python -u -m pytest tests/test_gpu_models.py tests/test_gpu_ops.py -m gpu -q -x -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_models.log 2>&1; rc=$?; echo "pytest models rc=$rc"; tail -5 gpurun_out/pytest_models.log; [ $rc -eq 0 ] || exit $rc; fi
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 10 --warmup 3 > gpurun_out/bench_iter.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_iter.log | cut -c1-400
