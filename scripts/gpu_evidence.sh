# Round evidence on one MI355X box: per-step kernel stats (no probe, no replays), PMC HBM traffic
# per kernel (FETCH_SIZE / WRITE_SIZE passes), then bench lines for every BASELINE model family.
# usage: scripts/gpu_evidence.sh <tag>    -> gpurun_out/prof_<tag>, gpurun_out/pmc_<tag>, gpurun_out/models_<tag>
set -u
cd "$GRAFT_REPO_ROOT"
tag=${1:-r02}
bash scripts/gpu_prof_steps.sh $tag pointnetpp dgcnn || exit $?
bash scripts/gpu_pmc.sh $tag pointnetpp dgcnn || exit $?
out=gpurun_out/models_$tag; mkdir -p $out
for m in pointnext pointnetpp_msg pointnet; do
  timeout -k 10 300 python bench.py --model $m --secondary none --no-cpu-baseline > $out/bench_$m.log 2>&1; rc=$?
  echo "bench $m rc=$rc"; tail -1 $out/bench_$m.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
done
