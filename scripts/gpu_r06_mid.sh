# Round 6 checkpoint: the whole GPU suite, smoke(), then the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_mid}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1500 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 600 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python -u bench.py --detail-out $out/bench_detail.json > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log
