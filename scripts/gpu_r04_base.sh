# Round-4 baseline: inverse-map tests, then the PointNet++ step as the bench runs it (prefetch +
# high priority) and as an unchanged harness-A step (no prefetch, default stream), plus a kernel
# trace of each.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r04_base; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_models.py -k "inverse or csr or geometry or plan or harness_a or knn or fps" -x -q -s -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_inv.log 2>&1; rc=$?
tail -3 $out/pytest_inv.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/fps_ab.py > $out/fps_ab.log 2>&1 || exit $?; cat $out/fps_ab.log
B="python3 $GRAFT_REPO_ROOT/bench.py --no-cpu-baseline --no-roofline --secondary none --steps 20 --warmup 5"
timeout -k 10 300 $B > $out/b_default.log 2>&1 || exit $?; tail -1 $out/b_default.log | cut -c1-200
timeout -k 10 300 $B --no-prefetch --stream-priority default > $out/b_dropin.log 2>&1 || exit $?; tail -1 $out/b_dropin.log | cut -c1-200
timeout -k 10 300 $B --model dgcnn > $out/b_dgcnn.log 2>&1 || exit $?; tail -1 $out/b_dgcnn.log | cut -c1-200
for v in default dropin; do
  extra=""; [ $v = dropin ] && extra="--no-prefetch --stream-priority default"
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_$v" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-roofline --secondary none --steps 10 --warmup 3 $extra \
     > "$GRAFT_REPO_ROOT/$out/prof_$v.log" 2>&1 || exit $?
  cd "$GRAFT_REPO_ROOT"
  f=$(find $out/prof_$v -name '*kernel_trace.csv' | head -1)
  python3 scripts/queue_breakdown.py "$f" > $out/queue_$v.txt; head -60 $out/queue_$v.txt
  python3 scripts/timeline.py "$f" 2 > $out/timeline_$v.txt
done
