# Round 6: pruned kNN diagnostics -- scanned tiles per wave (diag library) and a rocprofv3 kernel
# summary of scripts/knn_ab.py.  usage: gpu_r06_kdiag.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_kdiag}; mkdir -p $out
export TMPDIR=/tmp
PCS_LIB=$GRAFT_REPO_ROOT/3d-semantic-segmentation-benchmark_amd/pcseg/libpcseg_kdiag.so timeout -k 10 200 python -u scripts/knn_diag.py > $out/diag.log 2>&1; rc=$?
grep -v amdgpu $out/diag.log; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/knn_ab.py" new > "$GRAFT_REPO_ROOT/$out/prof.log" 2>&1; rc=$?
cd "$GRAFT_REPO_ROOT"; echo "prof rc=$rc"; [ $rc -eq 0 ] || exit $rc
f=$(find $out/prof -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && python3 scripts/prof_summary.py "$f" 1 14 > $out/knn_prof.txt; cat $out/knn_prof.txt
