# Round-6 final check on the committed tree: the whole GPU suite, smoke(), the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r06_final; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed" $out/pytest_gpu.log | tail -1; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --detail-out $out/bench_detail.json > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-300; exit $rc
