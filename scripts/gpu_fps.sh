# FPS A/B (indices must match the previous library's) + stamps + the FPS tests.
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-fps}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread -k fps > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/fps_ab.py > $out/ab.log 2>&1; rc=$?; cat $out/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/fps_stamps.py > $out/stamps.log 2>&1; rc=$?; cat $out/stamps.log; exit $rc
