# host phase split (3 prefetch points), then the full GPU suite
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s4}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
for p in loss backward none; do
  timeout -k 10 200 python -u scripts/host_phases.py pointnetpp $p > $out/host_$p.log 2>&1 || exit $?
  grep -v amdgpu.ids $out/host_$p.log
done
timeout -k 10 200 python -u scripts/host_phases.py dgcnn none > $out/host_dgcnn.log 2>&1 || exit $?
grep -v amdgpu.ids $out/host_dgcnn.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; exit $rc
