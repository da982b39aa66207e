# Round-5 iteration on one GPU lease: the named GPU tests, then the PointNet++ (and optionally DGCNN)
# bench line and a per-queue kernel breakdown of the bench step.
# usage: scripts/gpu_r05_iter.sh <tag> "<pytest selection>" [model ...]
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; sel=$2; shift 2
models=${*:-pointnetpp}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
if [ -n "$sel" ]; then
  timeout -k 10 600 python -u -m pytest $sel -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
  echo "pytest rc=$rc"; tail -3 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
fi
bash scripts/gpu_r04_prof.sh $tag $models > $out/queues.log 2>&1 || { tail -20 $out/queues.log; exit 1; }
for m in $models; do head -45 $out/queue_$m.txt; done
