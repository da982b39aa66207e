# Bench each model family once at its BASELINE per-GPU size (no CPU baseline), after engine tests.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/q
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_models.py -q -p no:cacheprovider --timeout 120 --timeout-method thread > gpurun_out/q/t.log 2>&1; rc=$?; tail -1 gpurun_out/q/t.log; [ $rc -eq 0 ] || exit $rc
for m in pointnetpp dgcnn pointnext pointnetpp_msg pointnet; do
  a="--model $m"; [ $m = pointnext ] && a="$a --batch 16 --npoints 24576 --steps 10"
  timeout -k 10 200 python bench.py $a --no-cpu-baseline > gpurun_out/q/b_$m.log 2>&1 || exit $?
  echo "$m $(tail -1 gpurun_out/q/b_$m.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["value"])')"
done
