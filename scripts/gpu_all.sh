# Full GPU parity suite, kNN timing, bench of PointNet++ and DGCNN (no CPU baseline).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u scripts/knn_bench.py > gpurun_out/knn_new.log 2>&1; rc=$?; cat gpurun_out/knn_new.log | grep knn; [ $rc -eq 0 ] || exit $rc
for m in ${MODELS_TO_BENCH:-pointnetpp dgcnn}; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --model $m --steps 20 --warmup 5 > gpurun_out/bench_$m.log 2>&1; rc=$?
  echo "bench $m rc=$rc $(tail -1 gpurun_out/bench_$m.log | cut -c1-330)"; [ $rc -eq 0 ] || exit $rc
done
