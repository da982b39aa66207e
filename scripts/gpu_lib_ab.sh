# A/B of two library builds (pcseg/libpcseg.so vs pcseg/libpcseg_ref.so), R interleaved rounds.
# usage: scripts/gpu_lib_ab.sh <tag> <rounds> [bench args]
set -u
cd "$GRAFT_REPO_ROOT"; tag=$1; rounds=$2; shift 2
out=gpurun_out/$tag; mkdir -p $out
P=3d-semantic-segmentation-benchmark_amd/pcseg
for r in $(seq $rounds); do
  for v in new ref; do
    lib=$P/libpcseg.so; [ $v = ref ] && lib=$P/libpcseg_ref.so
    PCS_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-roofline --secondary none "$@" > $out/b_${v}_$r.log 2>&1 || exit $?
    echo "$v round $r: $(tail -1 $out/b_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])")"
  done
done
