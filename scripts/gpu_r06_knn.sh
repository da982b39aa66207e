# Round 6: the software-pipelined kNN wave kernel -- A/B against the previous library (lists
# bitwise), the kNN / DGCNN tests, the DGCNN bench step.  usage: gpu_r06_knn.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_knn}; mkdir -p $out
export TMPDIR=/tmp
P=$GRAFT_REPO_ROOT/3d-semantic-segmentation-benchmark_amd/pcseg/libpcseg_prev.so
PCS_LIB=$P timeout -k 10 200 python -u scripts/knn_ab.py prev > $out/knn_prev.log 2>&1 || exit $?
timeout -k 10 200 python -u scripts/knn_ab.py new prev > $out/knn_new.log 2>&1 || exit $?
grep -h "^\[" $out/knn_prev.log $out/knn_new.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "knn or dgcnn or edgeconv" > $out/pytest_knn.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $out/pytest_knn.log; [ $rc -eq 0 ] || exit $rc
for lib in prev new; do
  if [ $lib = prev ]; then export PCS_LIB=$P; else unset PCS_LIB; fi
  timeout -k 10 300 python3 bench.py --model dgcnn --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none --steps 30 --warmup 5 > $out/bench_$lib.log 2>&1 || exit $?
  echo "$lib $(tail -1 $out/bench_$lib.log | grep -o '"ms_per_step": [0-9.]*')"
done
