# FPS checks + A/B, dgrad two-build A/B, graph-mode lines, per-step kernel stats, default bench line.
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s2}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_fps.sh ${tag}_fps || exit $?
bash scripts/gpu_libs_ab.sh ${tag}_ab 2 "- _ref _dg256" || exit $?
bash scripts/gpu_libs_ab.sh ${tag}_abd 1 "- _ref _dg256" --model dgcnn || exit $?
for m in pointnetpp dgcnn; do
  timeout -k 10 300 python -u bench.py --graph --model $m --secondary none --no-cpu-baseline --no-roofline > $out/graph_$m.log 2>&1; rc=$?
  echo "graph $m rc=$rc: $(tail -1 $out/graph_$m.log | cut -c1-400)"; [ $rc -eq 0 ] || exit $rc
done
bash scripts/gpu_prof_steps.sh $tag pointnetpp dgcnn || exit $?
timeout -k 10 600 python -u bench.py > $out/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -1 $out/bench.log
