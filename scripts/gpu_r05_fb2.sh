# Round 5: fused thin-layer backward with dA / dW on separate wave pairs (CI = 32): its GPU tests,
# then the step A/B against the round-4 wave assignment (libpcseg_nosplit.so).
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_fb2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_bwd.py tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_libs_ab.sh r05_ab11 3 "- _nosplit" || exit $?
