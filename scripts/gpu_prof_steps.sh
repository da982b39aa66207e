# Clean per-step kernel breakdown (no roofline probe, no replays): rocprofv3 --kernel-trace --stats
# over bench.py runs of W warm-up + S timed steps; summaries divide by (W + S).
# usage: scripts/gpu_prof_steps.sh <tag> [model ...]      (on the GPU box, via gpurun)
set -u
cd "$GRAFT_REPO_ROOT"
tag=${1:-r02}; shift || true
models=${*:-pointnetpp dgcnn}
out=gpurun_out/prof_$tag; mkdir -p $out
export TMPDIR=/tmp
for m in $models; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/$m" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --model $m --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --secondary none \
     > "$GRAFT_REPO_ROOT/$out/$m.log" 2>&1; rc=$?
  cd "$GRAFT_REPO_ROOT"; echo "$m prof rc=$rc"; tail -1 $out/$m.log | cut -c1-300
  [ $rc -eq 0 ] || exit $rc
  f=$(find $out/$m -name '*kernel_stats.csv' | head -1)
  python3 scripts/prof_summary.py "$f" 13 40 > $out/${m}_summary.txt && head -45 $out/${m}_summary.txt
done
