# HBM traffic per kernel from PMC counters (two separate passes, kernel-trace only; see
# MI355X_MICROARCH.md "HBM": FETCH_SIZE is doubled on gfx950, WRITE_SIZE exact).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
ARGS="--steps 3 --warmup 2 --no-cpu-baseline --no-roofline ${BENCH_ARGS:-}"
cd /tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/pmc_fetch.log" 2>&1; rc=$?; echo "pmc fetch rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/pmc_write" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" $ARGS > "$GRAFT_REPO_ROOT/gpurun_out/pmc_write.log" 2>&1; rc=$?; echo "pmc write rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT" && python scripts/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write > gpurun_out/pmc_traffic.txt 2>&1; echo "pmc parse rc=$?"; head -30 gpurun_out/pmc_traffic.txt
