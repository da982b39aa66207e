set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 120 python -u scripts/knn_variants.py > gpurun_out/knn_var.log 2>&1; rc=$?; cat gpurun_out/knn_var.log; exit $rc
