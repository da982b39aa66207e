set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python tests/diag_precision.py > gpurun_out/diag.log 2>&1; echo "diag rc=$?"
