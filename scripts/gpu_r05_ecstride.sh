# Round 5: EdgeConv backward reading its output gradient in place (row stride): EdgeConv / DGCNN GPU tests,
# then the DGCNN bench line twice.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_ecs; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_edgeconv.py tests/test_gpu_models.py -k "edgeconv or dgcnn or EdgeConv" -x -q -p no:cacheprovider --timeout 800 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python -u bench.py --model dgcnn --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none > $out/b_$r.log 2>&1 || exit $?
  echo "dgcnn round $r: $(tail -1 $out/b_$r.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
done
