set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/knn_pmc" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/knn_bench.py" > "$GRAFT_REPO_ROOT/gpurun_out/knn_pmc.log" 2>&1; echo "pmc rc=$?"
