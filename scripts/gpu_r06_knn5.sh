# Round 6: pruned kNN check -- kNN tests, per-graph timings, a rocprofv3 kernel summary of the
# timings script, one DGCNN bench step.  usage: gpu_r06_knn5.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_knn5}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "knn" > $out/pytest_knn.log 2>&1; rc=$?
echo "pytest knn rc=$rc"; grep -E "passed|failed" $out/pytest_knn.log | tail -2; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/knn_ab.py" new > "$GRAFT_REPO_ROOT/$out/knn_new.log" 2>&1; rc=$?
cd "$GRAFT_REPO_ROOT"; grep -h "^\[" $out/knn_new.log; [ $rc -eq 0 ] || exit $rc
f=$(find $out/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py "$f" 1 16 > $out/knn_prof.txt && grep -E "knn_(pruned|tiles|pairs|order|sqnorm)" $out/knn_prof.txt
timeout -k 10 300 python3 bench.py --model dgcnn --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 30 --warmup 5 > $out/bench.log 2>&1; rc=$?
tail -1 $out/bench.log | grep -o '"ms_per_step":[ 0-9.]*'; exit $rc
