# Per-model bench lines (BASELINE configs 3-5 at their per-GPU sizes) + rocprofv3 kernel stats for DGCNN.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/models
export TMPDIR=/tmp
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python bench.py "$@" > gpurun_out/models/bench_$n.log 2>&1; local rc=$?
  echo "bench $n rc=$rc"; tail -1 gpurun_out/models/bench_$n.log; return $rc
}
run dgcnn_b32 --model dgcnn --batch 32 --cpu-batch 2 --cpu-steps 3 &&
run pointnext_b16_n24576 --model pointnext --batch 16 --npoints 24576 --no-cpu-baseline --steps 10 --warmup 3 &&
run pointnetpp_msg_b32 --model pointnetpp_msg --batch 32 --no-cpu-baseline &&
run pointnet_b32 --model pointnet --batch 32 --no-cpu-baseline || exit $?
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/models/prof_dgcnn" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --model dgcnn --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/models/prof_dgcnn.log" 2>&1; echo "prof dgcnn rc=$?"
