set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -x -k fps > gpurun_out/fps_test.log 2>&1; rc=$?; tail -1 gpurun_out/fps_test.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python scripts/fps_bench.py 2>&1 | grep PCS || exit 1
timeout -k 10 300 python scripts/gemm_bench.py 2>&1 | grep -v amdgpu.ids
