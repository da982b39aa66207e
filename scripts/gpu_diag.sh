set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python tests/diag_precision.py ${DIAG_MODELS:-} > gpurun_out/diag.log 2>&1; echo "diag rc=$?"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -2 gpurun_out/bench.log
