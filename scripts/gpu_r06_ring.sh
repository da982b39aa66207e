# Round 6: the fused 128-wide backward ring (bwd_ring.hip) -- its tests and the fused-backward suite,
# its isolated timing (scripts/ring_ab.py), then the PointNet++ bench step alone and its rocprof stats.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_ring}; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bwd_ring.py tests/test_gpu_fused_bwd.py -x -v -p no:cacheprovider --timeout 150 --timeout-method thread > $out/pytest_ring.log 2>&1; rc=$?
echo "pytest ring rc=$rc"; tail -3 $out/pytest_ring.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u scripts/ring_ab.py > $out/ring_ab.log 2>&1; rc=$?; grep -v amdgpu.ids $out/ring_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model pointnetpp --secondary none --others none --no-cpu-baseline --no-drop-in --detail-out $out/bench_pp.json > $out/bench_pp.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 1500 $out/bench_pp.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --model pointnetpp --secondary none --others none --no-cpu-baseline --no-drop-in --no-roofline --steps 10 --warmup 3 > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1; echo "prof rc=$?"
cd "$GRAFT_REPO_ROOT" && f=$(find $out/prof -name '*kernel_stats.csv' | head -1) && python3 scripts/prof_summary.py "$f" 13 25 > $out/pp_stats.txt; head -16 $out/pp_stats.txt
