# A/B of several library builds (pcseg/libpcseg*.so by suffix: "" = libpcseg.so), R interleaved rounds.
# usage: scripts/gpu_libs_ab.sh <tag> <rounds> "<suffixes>" [bench args]   e.g. "- _ref _dg256"
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; rounds=$2; sfx=$3; shift 3
out=gpurun_out/$tag; mkdir -p $out
P=3d-semantic-segmentation-benchmark_amd/pcseg
for r in $(seq $rounds); do
  for v in $sfx; do
    s=$v; [ "$v" = "-" ] && s=""
    PCS_LIB=$GRAFT_REPO_ROOT/$P/libpcseg$s.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none "$@" > $out/b${s}_$r.log 2>&1 || exit $?
    echo "lib$s round $r: $(tail -1 $out/b${s}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])")"
  done
done
