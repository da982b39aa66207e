# Round 5: the fused 128 x 128 backward on eight waves (two per SIMD, W in LDS): its tests, then the
# step with every thin layer fused (--bwd-fuse all) on this library vs the four-wave build (now8),
# and the default policy, PointNet++ B=32; kernel times from one traced step of each 'all' run.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/r05_w8; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused_bwd.py -x -q -p no:cacheprovider --timeout 200 --timeout-method thread > $out/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 $out/pytest.log; [ $rc -eq 0 ] || exit $rc
P=3d-semantic-segmentation-benchmark_amd/pcseg
A="--no-cpu-baseline --no-roofline --no-drop-in --secondary none --others none"
for r in 1 2 3; do
  for v in "default -" "all -" "all _now8"; do
    set -- $v; s=$2; [ "$s" = "-" ] && s=""
    PCS_LIB=$GRAFT_REPO_ROOT/$P/libpcseg$s.so timeout -k 10 300 python -u bench.py $A --bwd-fuse $1 > $out/b_${1}${s}_${r}.log 2>&1 || exit $?
    echo "fuse=$1 lib$s round $r: $(tail -1 $out/b_${1}${s}_${r}.log | python3 -c "import json,sys; print(json.loads(sys.stdin.read())['ms_per_step'])")"
  done
done
for s in "" _now8; do
  cd /tmp && PCS_LIB=$GRAFT_REPO_ROOT/$P/libpcseg$s.so timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof$s" -o run --output-format csv -- \
     python3 "$GRAFT_REPO_ROOT/bench.py" $A --bwd-fuse all --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/$out/prof$s.log" 2>&1 || exit $?
  cd "$GRAFT_REPO_ROOT"; f=$(find $out/prof$s -name '*kernel_stats.csv' | head -1)
  echo "lib$s:"; grep "fused_bwd_kernel<128" "$f" | cut -d, -f1-6 | head -4
done
