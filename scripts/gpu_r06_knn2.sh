# Round 6: the pruned kNN (pcs_knn_order + pcs_knn_pruned) -- its tests, the kNN A/B on DGCNN's
# own features, the DGCNN bench step.  usage: gpu_r06_knn2.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_knn2}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "knn" > $out/pytest_knn.log 2>&1; rc=$?
echo "pytest knn rc=$rc"; grep -E "passed|failed|Error|error" $out/pytest_knn.log | tail -5; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/knn_ab.py new > $out/knn_new.log 2>&1; rc=$?; grep -h "^\[" $out/knn_new.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "dgcnn or edgeconv" > $out/pytest_dgcnn.log 2>&1; rc=$?
echo "pytest dgcnn rc=$rc"; tail -2 $out/pytest_dgcnn.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --model dgcnn --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 30 --warmup 5 > $out/bench.log 2>&1; rc=$?
tail -1 $out/bench.log | grep -o '"ms_per_step":[ 0-9.]*'; exit $rc
