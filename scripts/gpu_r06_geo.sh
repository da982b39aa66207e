# Round 6: the ball-query paths (select.hip: staged heap with the unambiguous-ball fast path, the
# cell-grid kernel) -- the neighbour-op tests, the group golden, the model goldens that group, then
# the ball query alone at the PointNet++ / PointNeXt SA1 shapes.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_geo}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "ball_query or group or fps_golden or inverse" > $out/pytest_geo.log 2>&1; rc=$?
echo "pytest geo rc=$rc"; tail -3 $out/pytest_geo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_models.py -x -q -p no:cacheprovider --timeout 600 --timeout-method thread -k "golden" > $out/pytest_golden.log 2>&1; rc=$?
echo "pytest model goldens rc=$rc"; tail -3 $out/pytest_golden.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ballq_ab.py > $out/ballq.log 2>&1; rc=$?; grep -v amdgpu.ids $out/ballq.log; exit $rc
