# GPU suite + smoke + default bench (CPU baselines included) on one MI355X box (via gpurun).
# usage: scripts/gpu_check.sh <tag> [pytest -k expr]
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-check}; kexpr=${2:-}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
if [ -n "$kexpr" ]; then
  timeout -k 10 1100 python -u -m pytest tests -m gpu --maxfail=25 -q -s -p no:cacheprovider --timeout 900 --timeout-method thread -k "$kexpr" > $out/pytest_gpu.log 2>&1; rc=$?
else
  timeout -k 10 1100 python -u -m pytest tests -m gpu --maxfail=25 -q -s -p no:cacheprovider --timeout 900 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
fi
echo "pytest rc=$rc"; grep -E "passed|failed|error" $out/pytest_gpu.log | tail -3
[ $rc -eq 0 ] || { grep -E "^E |Error|assert" $out/pytest_gpu.log | head -30; exit $rc; }
