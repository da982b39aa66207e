# Kernel traces of the default workload with an env knob on / off (A/B of one change):
# usage: scripts/gpu_prof_ab.sh <tag> <ENVVAR> [model]
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-ab}; var=${2:-PCS_FUSED_BWD}; model=${3:-pointnetpp}
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for v in 1 0; do
  cd /tmp && env $var=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/v$v" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" --model $model --steps 10 --warmup 3 --no-cpu-baseline --no-roofline --secondary none \
     > "$GRAFT_REPO_ROOT/$out/v$v.log" 2>&1; rc=$?
  cd "$GRAFT_REPO_ROOT"; echo "$var=$v rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for v in 1 0; do
  env $var=$v timeout -k 10 300 python -u bench.py --model $model --no-cpu-baseline --secondary none --roofline-replay > $out/bench_v$v.log 2>&1 || exit $?
  tail -1 $out/bench_v$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$var=$v', d['ms_per_step'], r['kernel'], r['avg_launch_us'], r.get('isolated_replay'))"
done
