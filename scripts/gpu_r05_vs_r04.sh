# Round 5 vs the round-4 tree (_r04/, its own library) on one model, standalone, interleaved rounds;
# then a kernel trace of the round-4 step.  usage: scripts/gpu_r05_vs_r04.sh <tag> <model> <rounds> <marker>
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; m=$2; n=$3; mk=$4
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for r in $(seq $n); do
  timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none > $out/new_$r.log 2>&1 || exit $?
  (cd _r04 && timeout -k 10 300 python -u bench.py --model $m --no-cpu-baseline --no-roofline --no-drop-in --secondary none) > $out/r04_$r.log 2>&1 || exit $?
  for v in new r04; do echo "$v round $r: $(tail -1 $out/${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'], d.get('host_runahead_wait_ms_per_step'))")"; done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_r04" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/_r04/bench.py" --model $m --no-cpu-baseline --no-roofline --no-drop-in --secondary none --steps 10 --warmup 3 \
   > "$GRAFT_REPO_ROOT/$out/prof_r04.log" 2>&1 || exit $?
cd "$GRAFT_REPO_ROOT"
f=$(find $out/prof_r04 -name '*kernel_trace.csv' | head -1)
python3 scripts/queue_breakdown.py "$f" "$mk" > $out/queue_r04_$m.txt; head -45 $out/queue_r04_$m.txt
