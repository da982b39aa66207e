# DGCNN gemm_nt tile A/B, then the round-end sequence on the final tree (full GPU suite, smoke, default bench line)
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/final3; mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_libs_ab.sh s12_ab 2 "- _b256" --model dgcnn || exit $?
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -1 $out/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log | cut -c1-300
exit $rc
