# Run selected GPU tests (TESTS env: pytest args)
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest ${TESTS:-tests} -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_quick.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_quick.log | tail -25; tail -25 gpurun_out/pytest_quick.log | grep -E "Error|assert|passed|failed" | head -20; exit $rc
