# The whole GPU suite (checkpoint), log under gpurun_out/r05_suite.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_suite; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $out/pytest_gpu.log; exit $rc
