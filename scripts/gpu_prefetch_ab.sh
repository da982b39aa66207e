# A/B of where the next step's geometry plan is enqueued (PointNet++ B=32), plus graph mode.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for v in loss backward loss backward; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --prefetch-point $v ${BENCH_ARGS:-} > gpurun_out/ab/$v.log 2>&1 || exit $?
  echo "$v $(tail -1 gpurun_out/ab/$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
done
for m in pointnext pointnetpp_msg; do for v in loss backward; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-roofline --model $m --prefetch-point $v $( [ $m = pointnext ] && echo --batch 16 --npoints 24576 --steps 10 ) > gpurun_out/ab/${m}_$v.log 2>&1 || exit $?
  echo "$m $v $(tail -1 gpurun_out/ab/${m}_$v.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["host_enqueue_ms_per_step"])')"
done; done
