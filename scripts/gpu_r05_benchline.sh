# The default bench line on the current tree (CPU baselines, rooflines, drop-in, configs 4/5) -> gpurun_out/r05_end/bench_final.log
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r05_end
timeout -k 10 700 python -u bench.py > gpurun_out/r05_end/bench_final.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/r05_end/bench_final.log | cut -c1-300; exit $rc
