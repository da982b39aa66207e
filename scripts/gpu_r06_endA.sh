# Round-6 evidence, part A: the whole GPU suite, smoke(), rocprofv3 --stats of the default bench
# command, per-workload clean traces (per-queue breakdown, one step's timeline, --stats summary).
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r06_end; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 500 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --detail-out none > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1; rc=$?; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT" && bash scripts/gpu_queues.sh r06_endq pointnetpp dgcnn pointnetpp_msg pointnext > $out/queues.log 2>&1; echo "queues rc=$?"
for m in pointnetpp dgcnn pointnetpp_msg pointnext; do
  f=$(find gpurun_out/r06_endq/prof_$m -name '*kernel_stats.csv' | head -1)
  [ -n "$f" ] && { echo "# rocprofv3 --kernel-trace --stats -- python3 bench.py --model $m --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 10 --warmup 3 (this workload only: 13 steps)"; python3 scripts/prof_summary.py "$f" 13 30; } > $out/r06_${m}_rocprof_stats.txt
done
ls $out
