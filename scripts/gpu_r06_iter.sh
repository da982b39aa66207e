# Round 6 iteration: ring tests + isolated ring timing, then the geometry tests + ball-query timing.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_iter}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bwd_ring.py tests/test_gpu_fused_bwd.py -x -q -p no:cacheprovider --timeout 150 --timeout-method thread > $out/pytest_ring.log 2>&1; rc=$?
echo "pytest ring rc=$rc"; tail -3 $out/pytest_ring.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ring_ab.py > $out/ring_ab.log 2>&1; rc=$?; grep -v amdgpu.ids $out/ring_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "ball_query or group or fps_golden" > $out/pytest_geo.log 2>&1; rc=$?
echo "pytest geo rc=$rc"; tail -3 $out/pytest_geo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ballq_ab.py > $out/ballq.log 2>&1; rc=$?; grep -v amdgpu.ids $out/ballq.log; exit $rc
