# Interleaved A/B of bench.py variants on one box (PointNet++ only unless flags say otherwise).
# usage: scripts/gpu_r04_ab.sh <tag> <rounds> "<ENV=.. ..>|<bench flags>" ...   (either side may be empty)
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for r in $(seq $rounds); do
  i=0
  for v in "$@"; do
    i=$((i+1)); envs=${v%%|*}; flags=${v#*|}
    env $envs timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --no-drop-in --secondary none $flags > $out/v${i}_r$r.log 2>&1 || exit $?
    echo "[$v] round $r: $(tail -1 $out/v${i}_r$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], 'ms, host', d['host_enqueue_ms_per_step'])")"
  done
done
