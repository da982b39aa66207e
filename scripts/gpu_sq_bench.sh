# SQ counters (one --pmc pass, kernel trace only) of a short bench step: MFMA-busy fraction and the
# wave-cycle split per dispatch (scripts/sq_summary.py).  usage: scripts/gpu_sq_bench.sh <tag> [bench args]
# e.g. scripts/gpu_sq_bench.sh fused_all --bwd-fuse all     -> gpurun_out/sq_<tag>/sq.txt
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; shift
out=gpurun_out/sq_$tag; mkdir -p $out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace -d "$GRAFT_REPO_ROOT/$out/run" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none "$@" \
   > "$GRAFT_REPO_ROOT/$out/run.log" 2>&1; rc=$?
echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT"
python3 scripts/sq_summary.py "$(find $out/run -name '*counter_collection.csv' | head -1)" "pcs::" > $out/sq.txt
head -40 $out/sq.txt
