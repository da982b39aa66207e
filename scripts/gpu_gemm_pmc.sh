# SQ counters of the engine GEMMs (gemm_bench shapes): MFMA busy, wait/issue stalls, LDS conflicts.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/gemm_pmc" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/gemm_bench.py" ${GEMM_ARGS:-} > "$GRAFT_REPO_ROOT/gpurun_out/gemm_pmc.log" 2>&1; echo "pmc rc=$?"
