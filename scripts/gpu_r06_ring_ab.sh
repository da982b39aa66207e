# Round 6: the ring kernel's diagnostic builds (no dZ transform / no data-gradient MFMAs / no
# weight-gradient MFMAs) against the product build, scripts/ring_ab.py each.
set -u
cd "$GRAFT_REPO_ROOT"; out=gpurun_out/${1:-r06_ring_ab}; shift || true; mkdir -p $out
P=3d-semantic-segmentation-benchmark_amd/pcseg
for v in ${*:-- _noxf _noa _now}; do
  s=$v; [ "$v" = "-" ] && s=""
  echo "== lib$s"
  PCS_LIB=$GRAFT_REPO_ROOT/$P/libpcseg$s.so timeout -k 10 200 python -u scripts/ring_ab.py > $out/ab$s.log 2>&1; rc=$?
  cat $out/ab$s.log | grep -v amdgpu.ids; [ $rc -eq 0 ] || exit $rc
done
