# stream-priority A/B: the step on a high-priority stream vs the default, PointNet++ x2, DGCNN x1
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/s13; mkdir -p $out
export TMPDIR=/tmp
ms() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])"; }
for r in 1 2; do
  for p in high default; do
    timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline --no-roofline --stream-priority $p > $out/pn_${p}_$r.log 2>&1 || exit $?
    echo "pointnetpp $p: $(ms $out/pn_${p}_$r.log)"
  done
done
for p in high default; do
  timeout -k 10 300 python -u bench.py --model dgcnn --secondary none --no-cpu-baseline --no-roofline --stream-priority $p > $out/dg_${p}.log 2>&1 || exit $?
  echo "dgcnn $p: $(ms $out/dg_${p}.log)"
done
