# Clean per-step kernel trace of the bench step (no drop-in, no roofline probe) per model.
# usage: scripts/gpu_queues.sh <tag> [model ...]
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-prof}; shift || true
models=${*:-pointnetpp dgcnn}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for m in $models; do
  timeout -k 10 300 python3 bench.py --model $m --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 20 --warmup 5 > $out/b_$m.log 2>&1 || exit $?
  tail -1 $out/b_$m.log | cut -c1-150
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_$m" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --model $m --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 10 --warmup 3 \
     > "$GRAFT_REPO_ROOT/$out/prof_$m.log" 2>&1 || exit $?
  cd "$GRAFT_REPO_ROOT"
  f=$(find $out/prof_$m -name '*kernel_trace.csv' | head -1)
  mk=fps_kernel\<512; [ $m = dgcnn ] && mk=knn_order_kernel; [ $m = pointnext ] && mk=fps_cull_kernel\<1024
  python3 scripts/queue_breakdown.py "$f" "$mk" > $out/queue_$m.txt; head -40 $out/queue_$m.txt
  python3 scripts/timeline.py "$f" 2 "$mk" > $out/timeline_$m.txt
done
