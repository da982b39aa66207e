# rocprofv3 kernel stats of one model's bench (MODEL env), summary under gpurun_out/prof_$MODEL.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
M=${MODEL:-dgcnn}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_$M" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --model $M --steps 5 --warmup 2 --no-cpu-baseline --no-roofline ${BENCH_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/prof_$M.log" 2>&1; rc=$?; echo "prof rc=$rc"; tail -1 "$GRAFT_REPO_ROOT/gpurun_out/prof_$M.log"; exit $rc
