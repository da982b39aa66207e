# A/B of the remaining engine env knobs against the defaults (PointNet++ and DGCNN B=32).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for m in pointnetpp dgcnn; do for rep in 1 2; do
  for v in X=0 PCS_GEMM_PERSIST=0 PCS_WGRAD_STAGES=4 PCS_WGRAD_THIN32=1; do
    env $v timeout -k 10 200 python bench.py --model $m --no-cpu-baseline --no-roofline > gpurun_out/ab/k.log 2>&1 || exit $?
    echo "$m $v $(tail -1 gpurun_out/ab/k.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done; done; done
