# inverse-map chunk-size A/B (isolated, batched as the models call it; checksums must match)
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/inv_r04; mkdir -p $out
export TMPDIR=/tmp
P=$PWD/3d-semantic-segmentation-benchmark_amd/pcseg
timeout -k 10 120 python -u scripts/inverse_ab.py base > $out/base.log 2>&1 || { tail $out/base.log; exit 1; }
for n in ${VARIANTS:-}; do
  PCS_LIB=$P/libpcseg_inv_$n.so timeout -k 10 120 python -u scripts/inverse_ab.py $n > $out/$n.log 2>&1 || { tail $out/$n.log; exit 1; }
done
grep -h -E "batched|total|dgcnn_knn|pnpp_sa1" $out/*.log
