# Round measurement for DGCNN (BASELINE config 3): PMC HBM traffic (two passes) + bench line with CPU baseline.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/final
export TMPDIR=/tmp
R=${ROUND:-r01}
ARGS="--model dgcnn --steps 2 --warmup 1 --no-cpu-baseline --no-roofline"
cd /tmp
timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch_dgcnn" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/final/pmc_fetch_dgcnn.log" 2>&1; rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write_dgcnn" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/final/pmc_write_dgcnn.log" 2>&1; rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT"
python scripts/pmc_traffic.py gpurun_out/pmc_fetch_dgcnn gpurun_out/pmc_write_dgcnn --json profiles/${R}_pmc_dgcnn_b32_n4096.json > gpurun_out/final/${R}_pmc_dgcnn_b32_n4096.txt 2>&1; echo "pmc parse rc=$?"
cp profiles/${R}_pmc_dgcnn_b32_n4096.json gpurun_out/final/
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/final/prof_dgcnn" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --model dgcnn --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/final/prof_dgcnn.log" 2>&1; echo "prof rc=$?"
cd "$GRAFT_REPO_ROOT" && timeout -k 10 400 python bench.py --model dgcnn --cpu-batch 2 --cpu-steps 3 > gpurun_out/final/bench_dgcnn.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/final/bench_dgcnn.log
