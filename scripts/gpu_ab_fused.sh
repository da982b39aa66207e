# Fused thin-layer backward: parity tests, then the bench with the fused path on / off (A/B).
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-fused}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_bwd.py tests/test_gpu_models.py tests/test_gpu_engine.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E "^E |Error|assert" $out/pytest.log | head -30; exit $rc; }
for f in 1 0; do
  PCS_FUSED_BWD=$f timeout -k 10 300 python -u bench.py --no-cpu-baseline --secondary none > $out/bench_f$f.log 2>&1; rc=$?
  echo "bench fused=$f rc=$rc"; tail -1 $out/bench_f$f.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'], d['roofline']['kernel'], d['roofline']['avg_launch_us'], d['roofline'].get('frac'))"
  [ $rc -eq 0 ] || exit $rc
done
