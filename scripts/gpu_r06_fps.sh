# Round 6: the spatially culled FPS (fps.hip fps_cull_kernel) -- FPS tests (bit-exact vs the oracle,
# goldens, sqrt tie), the geometry plan tests, smoke, then FPS + ball query timing at the SA1 shapes.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_fps}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "fps or ball_query" > $out/pytest_fps.log 2>&1; rc=$?
echo "pytest fps rc=$rc"; tail -3 $out/pytest_fps.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 600 --timeout-method thread -k "golden or geometry or prefetch" > $out/pytest_models.log 2>&1; rc=$?
echo "pytest models rc=$rc"; tail -3 $out/pytest_models.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ballq_ab.py > $out/ballq.log 2>&1; rc=$?; grep -v amdgpu.ids $out/ballq.log; exit $rc
