set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/knn_variants.py > gpurun_out/knn_var.log 2>&1; rc=$?; cat gpurun_out/knn_var.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/knn_bench.py > gpurun_out/knn_new.log 2>&1; rc=$?; cat gpurun_out/knn_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "knn or dgcnn or graph_feature or edge" > gpurun_out/pytest_knn.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_knn.log; exit $rc
