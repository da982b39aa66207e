# kernel traces of the PointNet++ and DGCNN steps (rocprofv3 --kernel-trace --stats), per-queue breakdown
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-prof}; shift || true; models=${*:-pointnetpp dgcnn}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for m in $models; do
  cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/$m" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --model $m --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --secondary none \
     > "$GRAFT_REPO_ROOT/$out/$m.log" 2>&1; rc=$?
  cd "$GRAFT_REPO_ROOT"; echo "$m prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
  f=$(find $out/$m -name '*kernel_trace.csv' | head -1)
  python3 scripts/queue_breakdown.py "$f" > $out/${m}_queues.txt; head -40 $out/${m}_queues.txt
done
