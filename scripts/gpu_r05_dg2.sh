# Round 5: DGCNN head-buffer change (EdgeConv second output) -- its GPU tests, then the geometry
# stream A/B libraries on PointNet++ and the DGCNN bench line.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_dg2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_edgeconv.py tests/test_gpu_dropout.py tests/test_gpu_models.py tests/test_gpu_inference.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu_libs_ab.sh r05_ab8 3 "- _r1lo _ir1 _r2" || exit $?
timeout -k 10 300 python -u bench.py --model dgcnn --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none > $out/b_dgcnn.log 2>&1 || exit $?
tail -1 $out/b_dgcnn.log
