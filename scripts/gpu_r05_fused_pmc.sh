# Round 5: SQ counters (one --pmc pass, kernel trace only) of the PointNet++ bench step with every
# thin layer fused (--bwd-fuse all) and with the default policy: MFMA busy fraction and the wave-cycle
# split of the WIDE fused kernel against the dgrad + lane wgrad pair it would replace.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_fpmc; mkdir -p $out
export TMPDIR=/tmp
C="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"
for v in all default; do
  cd /tmp && timeout -s KILL 150 rocprofv3 --pmc $C --kernel-trace -d "$GRAFT_REPO_ROOT/$out/$v" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --bwd-fuse $v --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none \
     > "$GRAFT_REPO_ROOT/$out/$v.log" 2>&1; rc=$?
  echo "$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
  cd "$GRAFT_REPO_ROOT"
  f=$(find $out/$v -name '*counter_collection.csv' | head -1)
  python3 scripts/sq_summary.py "$f" "pcs::" > $out/sq_$v.txt
  grep -E "fused_bwd|dgrad_kernel<true, 128, 2, 1>|wgrad_kernel<128, 128, 2, 1" $out/sq_$v.txt | head -24
done
