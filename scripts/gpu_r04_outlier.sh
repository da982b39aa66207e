# DGCNN-after-PointNet++ slow-step reproduction: per-step host enqueue times
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/outlier; mkdir -p $out
export TMPDIR=/tmp PCS_BENCH_STEPLOG=1
for i in 1 2 3 4; do
  timeout -k 10 180 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-drop-in --no-roofline > $out/b$i.json 2>$out/b$i.err || exit 1
  grep -E "host ms|stall|GiB" $out/b$i.err | cut -c1-300 | head -8
done
for i in; do
  timeout -k 10 180 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-roofline > $out/b$i.json 2>$out/b$i.err || exit 1
  grep -E "host ms|stall|GiB" $out/b$i.err | cut -c1-300 | head -8
done
