# graph-execution settings A/B, then the full GPU suite
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s3}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_graph_env.sh ${tag}_genv pointnetpp || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; exit $rc
