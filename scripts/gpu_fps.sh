set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_ops.py -m gpu -q -x -k fps > gpurun_out/fps_test.log 2>&1; rc=$?; tail -2 gpurun_out/fps_test.log; [ $rc -eq 0 ] || exit $rc
for b in 256 512 1024; do PCS_FPS_BLOCK=$b timeout -k 10 120 python scripts/fps_bench.py 2>&1 | grep PCS || exit 1; done
timeout -k 10 120 python scripts/fps_bench.py 2>&1 | grep PCS
