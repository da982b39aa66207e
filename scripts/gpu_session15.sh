# under the high-priority step stream: backward fuse policy and prefetch point A/B (PointNet++, 2 rounds)
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/s15; mkdir -p $out
export TMPDIR=/tmp
ms() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])"; }
for r in 1 2; do
  for v in "--bwd-fuse default" "--bwd-fuse off" "--bwd-fuse all" "--prefetch-point backward"; do
    tag=$(echo $v | tr -d ' -')
    timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline --no-roofline $v > $out/pn_${tag}_$r.log 2>&1 || exit $?
    echo "pointnetpp $v: $(ms $out/pn_${tag}_$r.log)"
  done
done
