# Default bench (PointNet++ only) under each value of one env knob, R rounds interleaved.
# usage: scripts/gpu_bench_ab.sh <tag> <ENVVAR | --bench-flag> "<values>" [rounds] [extra bench args]
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; var=$2; vals=$3; rounds=${4:-2}; shift 4 || shift $#
out=gpurun_out/$tag; mkdir -p $out
for r in $(seq $rounds); do
  for v in $vals; do
    if [ "${var#--}" != "$var" ]; then knob=(env); flag=("$var" "$v"); else knob=(env "$var=$v"); flag=(); fi
    "${knob[@]}" timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --secondary none "${flag[@]}" "$@" > $out/b_${v}_$r.log 2>&1 || exit $?
    echo "$var=$v round $r: $(tail -1 $out/b_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])")"
  done
done
