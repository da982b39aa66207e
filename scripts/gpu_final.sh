# Round measurement: PMC HBM traffic (two passes), rocprofv3 kernel stats, default bench (CPU baseline + live roofline).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/final
export TMPDIR=/tmp
R=${ROUND:-r01}
ARGS="--steps 3 --warmup 2 --no-cpu-baseline --no-roofline"
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/final/pmc_fetch.log" 2>&1; rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/final/pmc_write.log" 2>&1; rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT"
python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --json profiles/${R}_pmc_pointnetpp_b32_n4096.json > gpurun_out/final/${R}_pmc_pointnetpp_b32_n4096.txt 2>&1; echo "pmc parse rc=$?"
cp profiles/${R}_pmc_pointnetpp_b32_n4096.json gpurun_out/final/
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/final/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 5 --warmup 2 --no-cpu-baseline > "$GRAFT_REPO_ROOT/gpurun_out/final/prof.log" 2>&1; echo "prof rc=$?"
cd "$GRAFT_REPO_ROOT" && timeout -k 10 600 python bench.py > gpurun_out/final/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/final/bench.log
