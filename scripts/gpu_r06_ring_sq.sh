# Round 6: SQ counters of the ring kernel and the dgrad / wgrad pair it replaces (scripts/ring_ab.py,
# one --pmc pass with kernel trace only), summarised per dispatch by scripts/sq_summary.py.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_ring_sq}; mkdir -p $out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace -d "$GRAFT_REPO_ROOT/$out/run" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/scripts/ring_ab.py" > "$GRAFT_REPO_ROOT/$out/run.log" 2>&1; rc=$?
echo "rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd "$GRAFT_REPO_ROOT"
python3 scripts/sq_summary.py "$(find $out/run -name '*counter_collection.csv' | head -1)" "pcs::" > $out/sq.txt
grep -E "bwd_ring|dgrad_kernel<true, 128|wgrad_kernel<128, 128" $out/sq.txt | sort | uniq | head -20
