# Round 6: the pruned kNN as the DGCNN forward uses it -- kNN / DGCNN / EdgeConv GPU tests, the kNN
# A/B timings, two DGCNN bench steps.  usage: gpu_r06_knn4.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_knn4}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "knn or dgcnn or edgeconv" > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $out/pytest.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/knn_ab.py new > $out/knn_new.log 2>&1; rc=$?; grep -h "^\[" $out/knn_new.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --model dgcnn --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 30 --warmup 5 > $out/bench_$r.log 2>&1 || exit $?
  tail -1 $out/bench_$r.log | grep -o '"ms_per_step":[ 0-9.]*'
done
