# Per-queue kernel breakdown of one model's bench step (marker = the kernel that starts a step).
# usage: scripts/gpu_prof_model.sh <tag> <model> <marker>
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; m=$2; mk=$3
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_$m" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --model $m --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 10 --warmup 3 \
   > "$GRAFT_REPO_ROOT/$out/prof_$m.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
f=$(find $out/prof_$m -name '*kernel_trace.csv' | head -1)
python3 scripts/queue_breakdown.py "$f" "$mk" > $out/queue_$m.txt; head -60 $out/queue_$m.txt
python3 scripts/timeline.py "$f" 2 "$mk" > $out/timeline_$m.txt
