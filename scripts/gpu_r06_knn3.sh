# Round 6: pruned kNN iteration -- diagnostics (diag library), kNN tests, the kNN A/B timings, the
# DGCNN bench step.  usage: gpu_r06_knn3.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_knn3}; mkdir -p $out
export TMPDIR=/tmp
PCS_LIB=$GRAFT_REPO_ROOT/3d-semantic-segmentation-benchmark_amd/pcseg/libpcseg_kdiag.so timeout -k 10 200 python -u scripts/knn_diag.py > $out/diag.log 2>&1; rc=$?
grep -v amdgpu $out/diag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "knn" > $out/pytest_knn.log 2>&1; rc=$?
echo "pytest knn rc=$rc"; grep -E "passed|failed|Error" $out/pytest_knn.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/knn_ab.py new > $out/knn_new.log 2>&1; rc=$?; grep -h "^\[" $out/knn_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --model dgcnn --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 30 --warmup 5 > $out/bench.log 2>&1; rc=$?
tail -1 $out/bench.log | grep -o '"ms_per_step":[ 0-9.]*'; exit $rc
