# Round 5: the PointNet++ B=32 three-way test, then the geometry prefetch point A/B (loss / backward / start).
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_pp; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_models.py -k "b32_bench_dispatch" -x -q -s -p no:cacheprovider --timeout 800 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_bench_ab.sh r05_ppab --prefetch-point "loss backward start" 3 --no-drop-in --others none
