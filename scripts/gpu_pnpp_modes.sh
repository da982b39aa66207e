set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
for mode in "" "--graph" "--no-prefetch"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-roofline --steps 30 --warmup 5 $mode > gpurun_out/bench_mode.log 2>&1; rc=$?
  echo "mode[$mode] rc=$rc $(tail -1 gpurun_out/bench_mode.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"], d["host_enqueue_ms_per_step"])')"; [ $rc -eq 0 ] || exit $rc
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_pnpp" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > "$GRAFT_REPO_ROOT/gpurun_out/prof_pnpp.log" 2>&1; echo "prof rc=$?"
