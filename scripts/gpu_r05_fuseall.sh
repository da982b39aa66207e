# Round 5: every thin layer's backward fused (--bwd-fuse all) vs the default policy, and one traced
# step of each (per-queue kernel breakdown) to compare the WIDE fused launches with the dgrad + lane pairs.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_fuseall; mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_bench_ab.sh r05_fuseall_ab --bwd-fuse "default all" 2 --no-drop-in --others none || exit $?
for v in default all; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_$v" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --bwd-fuse $v --steps 10 --warmup 3 \
     > "$GRAFT_REPO_ROOT/$out/prof_$v.log" 2>&1 || exit $?
  cd "$GRAFT_REPO_ROOT"
  f=$(find $out/prof_$v -name '*kernel_trace.csv' | head -1)
  python3 scripts/queue_breakdown.py "$f" "fps_kernel<512" > $out/queue_$v.txt; head -30 $out/queue_$v.txt
done
