# HIP-graph replay vs eager: bench lines + kernel traces of both (per-queue breakdown, one step timeline)
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-graph}; mkdir -p $out
export TMPDIR=/tmp
for v in eager graph; do
  extra=""; [ $v = graph ] && extra="--graph"
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-roofline --no-drop-in --secondary none $extra > $out/b_$v.log 2>&1 || exit $?
  tail -1 $out/b_$v.log | cut -c1-160
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$out/prof_$v" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-roofline --no-drop-in --secondary none --steps 10 --warmup 3 $extra \
     > "$GRAFT_REPO_ROOT/$out/prof_$v.log" 2>&1 || exit $?
  cd "$GRAFT_REPO_ROOT"
  f=$(find $out/prof_$v -name '*kernel_trace.csv' | head -1)
  python3 scripts/queue_breakdown.py "$f" > $out/queue_$v.txt; head -30 $out/queue_$v.txt
  python3 scripts/timeline.py "$f" 2 > $out/timeline_$v.txt
done
