# A/B of the data-gradient GEMM tile policy (PCS_DGRAD_TILES), per model family at its BASELINE size.
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
for m in pointnetpp dgcnn pointnext pointnetpp_msg; do
  a="--model $m"; [ $m = pointnext ] && a="$a --batch 16 --npoints 24576 --steps 10"
  for rep in 1 2; do for v in auto legacy; do
    PCS_DGRAD_TILES=$v timeout -k 10 200 python bench.py $a --no-cpu-baseline --no-roofline > gpurun_out/ab/d.log 2>&1 || exit $?
    echo "$m $v $(tail -1 gpurun_out/ab/d.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
  done; done
done
