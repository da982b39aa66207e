# Round-4 final evidence on the final tree: full GPU suite + smoke, the rocprofv3 kernel-trace stats of
# the default bench command (GPU work; the CPU-baseline subprocess runs no kernel) and of the drop-in
# harness-A step alone, per-queue breakdowns, then the default bench line itself.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r04_final; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- \
   python3 "$GRAFT_REPO_ROOT/bench.py" --no-cpu-baseline > "$GRAFT_REPO_ROOT/$out/prof_bench.log" 2>&1; rc=$?
cd "$GRAFT_REPO_ROOT"; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
for m in pointnetpp dgcnn; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof_dropin_$m" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/scripts/drop_in_step.py" $m 10 > "$GRAFT_REPO_ROOT/$out/prof_dropin_$m.log" 2>&1; rc=$?
  cd "$GRAFT_REPO_ROOT"; echo "prof drop-in $m rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_r04_prof.sh r04_final/queues pointnetpp dgcnn > $out/queues.log 2>&1 || { tail $out/queues.log; exit 1; }
timeout -k 10 900 python -u bench.py > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-300
exit $rc
