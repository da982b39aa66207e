# CapturedStep tests + bench eager vs graph (PointNet++ and DGCNN).
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-gs}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_graphs.py tests/test_gpu_optim.py tests/test_gpu_models.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "graph or adam or prefetch or bitwise" > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || { grep -E "^E " $out/pytest.log | head -20; exit $rc; }
for mode in eager graph; do
  fl=""; [ $mode = graph ] && fl="--graph"
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-roofline $fl > $out/bench_$mode.log 2>&1; rc=$?
  echo "bench $mode rc=$rc"; [ $rc -eq 0 ] || { tail -5 $out/bench_$mode.log; exit $rc; }
  tail -1 $out/bench_$mode.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['secondary']; print('$mode', d['ms_per_step'], d['host_enqueue_ms_per_step'], '| dgcnn', s['ms_per_step'], s['host_enqueue_ms_per_step'])"
done
