# The whole GPU suite once against the bounds-checked library (make debug ->
# pcseg/libpcseg_debug.so, device-side PCS_DCHECK on every clamped operand access; loaded by PCS_LIB).
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-debug}; mkdir -p $out
export TMPDIR=/tmp
export PCS_LIB=$GRAFT_REPO_ROOT/3d-semantic-segmentation-benchmark_amd/pcseg/libpcseg_debug.so
timeout -k 10 1100 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_debug.log 2>&1; rc=$?
echo "pytest (debug library) rc=$rc"; tail -3 $out/pytest_debug.log
grep -c "pcs bounds" $out/pytest_debug.log || true
exit $rc
