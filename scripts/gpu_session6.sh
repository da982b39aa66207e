# DGCNN inverse-map placement A/B, PointNet++ grouped-rows dX-from-column-3 A/B, then the full GPU suite
set -u
cd "$GRAFT_REPO_ROOT"; tag=${1:-s6}; out=gpurun_out/$tag; mkdir -p $out
export TMPDIR=/tmp
ms() { tail -1 $1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['host_enqueue_ms_per_step'])"; }
for r in 1 2; do
  for e in deferred backward side; do
    timeout -k 10 300 python -u bench.py --model dgcnn --secondary none --no-cpu-baseline --no-roofline --edge-inverse $e > $out/edge_${e}_$r.log 2>&1 || exit $?
    echo "dgcnn edge-inverse $e: $(ms $out/edge_${e}_$r.log)"
  done
  timeout -k 10 300 python -u bench.py --secondary none --no-cpu-baseline --no-roofline > $out/pn_dx3_$r.log 2>&1 || exit $?
  echo "pointnetpp dx_from=3: $(ms $out/pn_dx3_$r.log)"
  timeout -k 10 300 python -u -c "
import sys; sys.argv = ['bench.py', '--secondary', 'none', '--no-cpu-baseline', '--no-roofline']
sys.path[:0] = ['.', '3d-semantic-segmentation-benchmark_amd']
import pcseg.common as c
orig = c.MiniPointNet.forward_rows
c.MiniPointNet.forward_rows = lambda self, x, kin=None, pool_k=0, dx_from=0: orig(self, x, kin, pool_k, 0)
import bench; bench.main()" > $out/pn_dx0_$r.log 2>&1 || exit $?
  echo "pointnetpp dx_from=0: $(ms $out/pn_dx0_$r.log)"
done
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 120 --timeout-method thread > $out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 $out/pytest_gpu.log; exit $rc
