# bench lines of the other BASELINE model families (no CPU baseline), then the full GPU suite and smoke()
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/models_r03; mkdir -p $out
export TMPDIR=/tmp
for m in pointnext pointnetpp_msg pointnet; do
  timeout -k 10 300 python -u bench.py --model $m --secondary none --no-cpu-baseline > $out/bench_$m.log 2>&1; rc=$?
  echo "bench $m rc=$rc"; tail -1 $out/bench_$m.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.log; exit $rc
