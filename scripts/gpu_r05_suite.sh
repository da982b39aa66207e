# The whole GPU suite (checkpoint) and smoke(), logs under gpurun_out/r05_suite.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_suite; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 150 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.log; exit $rc
