# A/B of the wgrad row-split target (PCS_WGRAD_BLOCKS).
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for m in pointnetpp dgcnn; do for rep in 1 2; do for v in 1024 512 2048; do
  PCS_WGRAD_BLOCKS=$v timeout -k 10 200 python bench.py --model $m --no-cpu-baseline --no-roofline > gpurun_out/ab/w.log 2>&1 || exit $?
  echo "$m $v $(tail -1 gpurun_out/ab/w.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done; done; done
