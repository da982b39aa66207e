# Neighbour-selection iteration: ball-query / 3-NN parity tests, then PointNet++ bench (prefetch and not).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/sel
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -k "ball or three_nn or interpolate or inverse" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/sel/tests.log 2>&1; rc=$?
tail -3 gpurun_out/sel/tests.log; [ $rc -eq 0 ] || exit $rc
for a in "" "--no-prefetch"; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline $a > gpurun_out/sel/bench.log 2>&1 || exit $?
  echo "bench $a $(tail -1 gpurun_out/sel/bench.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
done
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/sel/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > "$GRAFT_REPO_ROOT/gpurun_out/sel/prof.log" 2>&1; echo "prof rc=$?"
grep -h "select_kernel\|three_nn\|fps_kernel" "$GRAFT_REPO_ROOT"/gpurun_out/sel/prof/run_kernel_stats.csv | cut -d, -f1-5 || true
