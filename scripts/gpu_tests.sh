# GPU parity tests (optionally a -k subset) on one MI355X box (via gpurun).
# usage: scripts/gpu_tests.sh <tag> [pytest -k expr]
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-tests}; kexpr=${2:-}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
args=(tests -m gpu --maxfail=25 -v -s -p no:cacheprovider --timeout 300 --timeout-method thread)
[ -n "$kexpr" ] && args+=(-k "$kexpr")
timeout -k 10 1000 python -u -m pytest "${args[@]}" > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" $out/pytest_gpu.log | tail -3
[ $rc -eq 0 ] || { grep -E "^E |FAILED|Error" $out/pytest_gpu.log | head -40; exit $rc; }
