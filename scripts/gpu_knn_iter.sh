# kNN iteration: exactness + oracle tests, then kernel timings (B=32, N=4096, k=20).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "knn" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/knn_tests.log 2>&1; rc=$?
tail -5 gpurun_out/knn_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/knn_variants.py > gpurun_out/knn_var.log 2>&1; rc=$?; cat gpurun_out/knn_var.log; exit $rc
