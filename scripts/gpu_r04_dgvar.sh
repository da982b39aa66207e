# Round-4 A/B of the DMA data-gradient variants (PCS_DGRAD_VAR): bitwise test, isolated timing,
# PointNet++ step
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/dgvar; mkdir -p $out
export TMPDIR=/tmp
for v in 64x3 128x2 128x3 64x3 128x2 128x3; do
  PCS_DGRAD_VAR=$v timeout -k 10 180 python -u bench.py --steps 30 --warmup 10 --no-cpu-baseline --no-drop-in > $out/bench_$v.json 2>$out/bench_$v.err || exit 1
  echo "$v $(python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline'], d['secondary']['ms_per_step'])" $out/bench_$v.json)"
done
