# kNN prefetch-wait fix: kNN tests, isolated seeded/unseeded timing, DGCNN step
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/knnfix; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_edgeconv.py -k "knn or edge" -x -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { tail -30 $out/pytest.log; exit 1; }
tail -2 $out/pytest.log
timeout -k 10 200 python -u scripts/knn_seed_ab.py > $out/knn_ab.log 2>&1 || { tail $out/knn_ab.log; exit 1; }
grep -v amdgpu.ids $out/knn_ab.log | tail -12
for i in 1 2; do
  timeout -k 10 200 python -u bench.py --model dgcnn --secondary none --no-cpu-baseline --no-drop-in --no-roofline > $out/b$i.json 2>$out/b$i.err || { tail -5 $out/b$i.err; exit 1; }
  echo "dgcnn $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'])" $out/b$i.json)"
done
