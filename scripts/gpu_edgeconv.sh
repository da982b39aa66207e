set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_edgeconv.py tests/test_gpu_models.py -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "edgeconv or dgcnn" > gpurun_out/pytest_edge.log 2>&1; rc=$?; grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_edge.log | head -30; tail -3 gpurun_out/pytest_edge.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python bench.py --no-cpu-baseline --model dgcnn --steps 20 --warmup 5 > gpurun_out/bench_dgcnn.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_dgcnn.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof_dgcnn" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --model dgcnn --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > "$GRAFT_REPO_ROOT/gpurun_out/prof_dgcnn.log" 2>&1; echo "prof rc=$?"
