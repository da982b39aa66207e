# bench lines of the other BASELINE configs' per-GPU halves (MSG B=32, PointNeXt-B B=16 x 24576) and PointNet
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/models_r04; mkdir -p $out
export TMPDIR=/tmp
for m in pointnetpp_msg pointnext pointnet; do
  timeout -k 10 400 python -u bench.py --model $m --secondary none --no-cpu-baseline > $out/$m.json 2>$out/$m.err || { tail -5 $out/$m.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['value'], (d.get('drop_in') or {}).get('ms_per_step'), d['roofline']['kernel'], d['roofline']['frac'], d['step_roofline'])" $out/$m.json $m
done
